# Round 3: DG1 zero-prefix waves paced with s_sleep 8/32/127 between stages
# (S3DG_DIAG_KSZSLEEP) vs the base build, with DG1 c1 and K2 as controls
# (tools/zero_power_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3z}
mkdir -p $OUT
LAB_NAMES=base,zs8,zs32,zs127 LAB_REPS=2 LAB_SEG_S=1.5 LAB_POINTS="dg1c2,dg1,k2" \
  timeout -k 10 400 python -u tools/zero_power_lab.py > $OUT/ks_zero_pace.log 2>&1 || { tail -30 $OUT/ks_zero_pace.log; exit 1; }
python - $OUT/ks_zero_pace.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d = json.loads(l)
    if "GBps" not in d: print(d); continue
    acc = d["accumulation_counter_delta"] or 1
    print(d["rep"], d["point"], d["variant"], d["GBps"], "ppt%%", round(100 * d["ppt_residency_acc_delta"] / acc),
          "gfx", d["current_gfxclk_med"], "P", d["current_socket_power_med"], "Tmem", d["temperature_mem_max"],
          "umc", d["average_umc_activity_med"], "soc", d["current_socclk_med"], "Vgfx", d["voltage_gfx_med"], "Vsoc", d["voltage_soc_med"], "Vmem", d["voltage_mem_med"])
PY
LAB_VARIANTS="base=;zs8=-DS3DG_DIAG_KSZSLEEP=8;zs32=-DS3DG_DIAG_KSZSLEEP=32;zs127=-DS3DG_DIAG_KSZSLEEP=127" LAB_POINTS="dg1c2_8g:0:0:0:-1:0" LAB_REPS=4 LAB_N=10000 \
  timeout -k 10 300 python -u tools/variant_lab.py > $OUT/ks_zero_pace_8g.log 2>&1 || { tail -20 $OUT/ks_zero_pace_8g.log; exit 1; }
grep '^{' $OUT/ks_zero_pace_8g.log

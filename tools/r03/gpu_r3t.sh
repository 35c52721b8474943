# Round 3: config 5 (d2 c3) and d1 c3 uncapped vs cap 30 on another box, and
# the keystream (K2, DG1 c1/c2) power and clock, base build
# (tools/zero_power_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3t}
mkdir -p $OUT
LAB_NAMES=base LAB_REPS=2 LAB_SEG_S=1.5 LAB_POINTS="cfg2,cfg5,cfg5@30,d1c3,d1c3@30,cfg3,cfg3@30,k2,dg1,dg1c2" \
  timeout -k 10 400 python -u tools/zero_power_lab.py > $OUT/power_c3_ks.log 2>&1 || { tail -30 $OUT/power_c3_ks.log; exit 1; }
python - $OUT/power_c3_ks.log <<'PY'
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

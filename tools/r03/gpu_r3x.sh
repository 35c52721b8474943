# Round 3: wall-clock pacing of the stores (S3DG_DIAG_RTPACE = 100..300 ticks
# of 10 ns after workgroup start) on uncapped launches of config 2/3/5 and
# d1 c3/c4, against the base build (tools/zero_power_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3x}
mkdir -p $OUT
LAB_NAMES=base,rt100,rt150,rt200,rt300 LAB_REPS=2 LAB_SEG_S=1.5 LAB_POINTS="cfg2@0,cfg3@0,cfg5@0,d1c3@0,d1c4@0,cfg3@30" \
  timeout -k 10 400 python -u tools/zero_power_lab.py > $OUT/rtpace.log 2>&1 || { tail -30 $OUT/rtpace.log; exit 1; }
python - $OUT/rtpace.log <<'PY'
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

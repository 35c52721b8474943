# Round 3: GPU power / clocks / PPT residency per data pattern (d, c) and
# occupancy cap, base build only (tools/zero_power_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3p}
mkdir -p $OUT
LAB_NAMES=base LAB_REPS=2 LAB_SEG_S=2.0 LAB_POINTS="cfg2,cfg3,cfg5,d1c3,d1c2,d1c4,d4c1,cfg3@28,cfg3@24,cfg2@28,d1c4@24" \
  timeout -k 10 300 python -u tools/zero_power_lab.py > $OUT/power_patterns.log 2>&1 || { tail -30 $OUT/power_patterns.log; exit 1; }
python - $OUT/power_patterns.log <<'PY'
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

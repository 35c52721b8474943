# Round 3: rate / power / clock per data pattern (zero-prefix fraction) and
# batch occupancy cap (32 resident = uncapped, 30, 28, 26), base build only
# (tools/zero_power_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3q}
mkdir -p $OUT
LAB_NAMES=base LAB_REPS=2 LAB_SEG_S=1.5 LAB_POINTS="cfg2,cfg2@30,cfg2@28,cfg2@26,d1c15,d1c15@30,d1c15@28,d1c15@26,cfg3,cfg3@30,cfg3@28,cfg3@26,d1c2,d1c2@30,d1c2@28,d1c2@26,cfg5,cfg5@30,cfg5@28,cfg5@26,d1c4,d1c4@30,d1c4@28,d1c4@26,d1c8,d1c8@30,d1c8@28,d1c8@26" \
  timeout -k 10 400 python -u tools/zero_power_lab.py > $OUT/power_caps.log 2>&1 || { tail -30 $OUT/power_caps.log; exit 1; }
python - $OUT/power_caps.log <<'PY'
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

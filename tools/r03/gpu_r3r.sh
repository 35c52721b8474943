# Round 3: which zero-prefix lengths want the batch occupancy cap: d1 at
# compress 1..64 and rational ratios, uncapped vs 30 (29 resident), base build
# (tools/zero_power_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3r}
mkdir -p $OUT
LAB_NAMES=base LAB_REPS=2 LAB_SEG_S=1.5 LAB_POINTS="f0x1,f0x1@30,f1x2,f1x2@30,f3x4,f3x4@30,f7x8,f7x8@30,f15x16,f15x16@30,f31x32,f31x32@30,f63x64,f63x64@30,f1x4,f1x4@30,f4x5,f4x5@30,f5x6,f5x6@30,f6x7,f6x7@30,f2x5,f2x5@30,f1x3,f1x3@30,f2x3,f2x3@30" \
  timeout -k 10 400 python -u tools/zero_power_lab.py > $OUT/power_rule.log 2>&1 || { tail -30 $OUT/power_rule.log; exit 1; }
python - $OUT/power_rule.log <<'PY'
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

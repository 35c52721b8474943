# Round 3: cap {none, 30} x wall-clock store floor {0..200 ticks} for
# config 3, d1 c4, d1 c3, and small floors for config 2, base build
# (tools/zero_power_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3kk}
mkdir -p $OUT
LAB_NAMES=base LAB_REPS=2 LAB_SEG_S=1.2 LAB_POINTS="cfg3@0%0,cfg3@0%50,cfg3@0%100,cfg3@0%150,cfg3@0%200,cfg3@30%0,cfg3@30%50,cfg3@30%100,cfg3@30%150,cfg3@30%200,d1c4@0%0,d1c4@0%50,d1c4@0%100,d1c4@0%150,d1c4@0%200,d1c4@30%0,d1c4@30%50,d1c4@30%100,d1c4@30%150,d1c4@30%200,d1c3@0%0,d1c3@0%50,d1c3@0%100,d1c3@0%150,d1c3@0%200,d1c3@30%0,d1c3@30%50,d1c3@30%100,d1c3@30%150,d1c3@30%200,cfg2@0%0,cfg2@0%25,cfg2@0%50" \
  timeout -k 10 400 python -u tools/zero_power_lab.py > $OUT/cap_floor_sweep.log 2>&1 || { tail -30 $OUT/cap_floor_sweep.log; exit 1; }
python - $OUT/cap_floor_sweep.log <<'PY'
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

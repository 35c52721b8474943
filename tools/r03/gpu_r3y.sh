# Round 3: the per-launch batch rule (default: cap 30 for line-aligned zero
# prefixes, a 100-tick store floor for mid-line prefixes of >= half a block)
# against uncapped, uncapped + floor 100 and cap 30, per pattern.  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3y}
mkdir -p $OUT
LAB_NAMES=base LAB_REPS=2 LAB_SEG_S=1.5 LAB_POINTS="cfg2,cfg2@0%0,cfg2@0%100,cfg2@30%0,d1c15,d1c15@0%0,d1c15@0%100,d1c15@30%0,f1x4,f1x4@0%0,f1x4@0%100,f1x4@30%0,f2x5,f2x5@0%0,f2x5@0%100,f2x5@30%0,cfg3,cfg3@0%0,cfg3@0%100,cfg3@30%0,d1c2,d1c2@0%0,d1c2@0%100,d1c2@30%0,cfg5,cfg5@0%0,cfg5@0%100,cfg5@30%0,d1c3,d1c3@0%0,d1c3@0%100,d1c3@30%0,d1c4,d1c4@0%0,d1c4@0%100,d1c4@30%0,f4x5,f4x5@0%0,f4x5@0%100,f4x5@30%0,d1c8,d1c8@0%0,d1c8@0%100,d1c8@30%0" \
  timeout -k 10 400 python -u tools/zero_power_lab.py > $OUT/rule2.log 2>&1 || { tail -30 $OUT/rule2.log; exit 1; }
python - $OUT/rule2.log <<'PY'
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
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "floor or occupancy or batch_mixed or tiled" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log

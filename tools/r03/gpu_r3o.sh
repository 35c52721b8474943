# Round 3: config 3's zero data vs GPU power, clocks and throttle residency
# (tools/zero_power_lab.py; base and zconst builds).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3o}
mkdir -p $OUT
timeout -k 10 300 python -u tools/zero_power_lab.py > $OUT/zero_power_lab.log 2>&1 || { tail -30 $OUT/zero_power_lab.log; exit 1; }
python - $OUT/zero_power_lab.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d = json.loads(l)
    if "GBps" not in d: print(d); continue
    print(d["rep"], d["point"], d["variant"], d["GBps"], "E", d["energy_acc_delta"], "clk", d["sys_clock_delta"],
          "ppt", d["ppt_residency_acc_delta"], "thm", d["socket_thm_residency_acc_delta"], "acc", d["accumulation_counter_delta"],
          "vppt", d["viol_acc_ppt_pwr_delta"], "vhbm", d["viol_acc_hbm_thrm_delta"], "vcnt", d["viol_acc_counter_delta"],
          "uclk", d["current_uclk_med"], "gfx", d["current_gfxclk_med"], "P", d["current_socket_power_med"],
          "Thbm", d["temperature_hbm_max"], "Tmem", d["temperature_mem_max"], "umc", d["average_umc_activity_med"],
          "thr", d["throttle_status_set"], d["indep_throttle_status_set"])
PY

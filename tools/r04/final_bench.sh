# Round-4 final tree: one bench line per config (config 2 = the driver's
# command) with CPU baseline, D2H-inclusive rate and store-only references;
# CFGS selects the configs (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r4final_bench}
mkdir -p $OUT
for c in ${CFGS:-2 3 4 5 6 8 9 10}; do
  if [ "$c" = 2 ]; then
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_cfg2.log 2>&1 || { tail $OUT/bench_cfg2.log; exit 1; }
  elif [ "$c" = 5full ]; then
    timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --d2h-full > $OUT/bench_cfg5_d2h_full.log 2>&1 || { tail $OUT/bench_cfg5_d2h_full.log; exit 1; }
  else
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $OUT/bench_cfg$c.log 2>&1 || { tail $OUT/bench_cfg$c.log; exit 1; }
  fi
  echo "cfg$c done"
done
grep -h '^{' $OUT/bench_cfg*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); r = d['roofline']; c = d['cpu_baseline'] or {}
    print(d['config']['workload'][:60], '| value', d['value'], '| achieved', r['achieved'], r['frac'], '| traffic', r.get('traffic'), '| d2h', d['d2h_inclusive'] and d['d2h_inclusive']['value'], '| cpu', c.get('value'), c.get('min_med_max_GiBps'), '| ok', d['verified_vs_oracle'])"

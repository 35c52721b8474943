# Final-tree evidence, part 2: one bench line per config (the driver's command
# for config 2), then the DG1 caller A/B (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2v}
mkdir -p $OUT
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_cfg2.log 2>&1 || { tail $OUT/bench_cfg2.log; exit 1; }
echo "cfg2 done"
for c in 3 4 5 6 8 9 10 11 12 13 14 15 16 17; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $OUT/bench_cfg$c.log 2>&1 || { tail $OUT/bench_cfg$c.log; exit 1; }
  echo "cfg$c done"
done
grep -h '^{' $OUT/bench_cfg*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); r = d['roofline']
    print(d['config']['workload'][:50], '| value', d['value'], '| achieved', r['achieved'], r['frac'], '| traffic', r['traffic'], '| d2h', d['d2h_inclusive'] and d['d2h_inclusive']['value'], '| cpu', d['cpu_baseline'] and d['cpu_baseline']['value'], '| ok', d['verified_vs_oracle'])"
timeout -k 10 300 python -u tools/dg1_launch_ab.py > $OUT/dg1_launch_ab.log 2>&1 || { tail -20 $OUT/dg1_launch_ab.log; exit 1; }
grep '^{' $OUT/dg1_launch_ab.log

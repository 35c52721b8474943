# J-word preload in the scalar jump: GPU tests; events-between-launches lab;
# DG1 / K2 bench lines (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2p}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u tools/event_gap_lab.py > $OUT/event_gap_lab.log 2>&1 || { tail -20 $OUT/event_gap_lab.log; exit 1; }
grep '^{' $OUT/event_gap_lab.log
for c in 6 14 16; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-d2h > $OUT/bench_cfg$c.log 2>&1 || { tail $OUT/bench_cfg$c.log; exit 1; }
  grep -h '^{' $OUT/bench_cfg$c.log | python -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d['roofline']
print(d['config']['workload'][:60], '| value', d['value'], '| achieved', r['achieved'], r['frac'], r['avg_launch_ms'], '| ok', d['verified_vs_oracle'])"
done

# Final tree re-check: GPU tests, smoke, the driver's bench command (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2z}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log | tail -1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_cfg2.log 2>&1 || { tail $OUT/bench_cfg2.log; exit 1; }
grep -h '^{' $OUT/bench_cfg2.log | python -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d['roofline']
print(d['value'], r['achieved'], r['frac'], r['traffic'], r['source_digest'], d['verified_vs_oracle'], d['cpu_baseline']['value'], d['d2h_inclusive']['value'])"

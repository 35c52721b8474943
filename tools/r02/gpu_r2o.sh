# Keystream lanes of 2048/4096 draws + s3dg_dgen_fill_stream: GPU tests, then
# bench lines for the keystream/DG1 configs (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2o}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for c in 6 14 15 16 17; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $OUT/bench_cfg$c.log 2>&1 || { tail $OUT/bench_cfg$c.log; exit 1; }
  grep -h '^{' $OUT/bench_cfg$c.log | python -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d['roofline']
print(d['config']['workload'][:60], '| value', d['value'], '| achieved', r['achieved'], r['frac'], '| d2h', d['d2h_inclusive'] and d['d2h_inclusive']['value'], '| cpu', d['cpu_baseline'] and d['cpu_baseline']['value'], '| ok', d['verified_vs_oracle'])"
done

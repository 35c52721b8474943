# Round 3: the compress-ratio x cap rule lab (gpu_r3r.sh), then the product
# with the per-launch batch occupancy rule: parity/batch tests and bench
# lines for configs 2-5.  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3s}
mkdir -p $OUT
bash tools/r03/gpu_r3r.sh ${1:-r3s} || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in 2 3 4 5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-d2h > $OUT/bench_cfg$c.log 2>&1 || { tail $OUT/bench_cfg$c.log; exit 1; }
  grep -h '^{' $OUT/bench_cfg$c.log | python -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print(d['config']['workload'][:40], '| value', d['value'], '| achieved', r['achieved'], r['frac'], '| ok', d['verified_vs_oracle'])"
done

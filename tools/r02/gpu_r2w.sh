# Keystream tail part: GPU tests, A/B vs no tail part (S3DG_KS_NOTAIL=1), bench lines (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2w}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
P="k2:1:0:2048:2:16;k2_8g:1:0:2048:2:16;dg1:1:0:2048:2:16;dg1_8g:1:0:2048:2:16;dg1c2_8g:4:0:512:2:32"
LAB_VARIANTS="tail=;notail=-DS3DG_KS_NOTAIL=1" LAB_POINTS="$P" LAB_REPS=4 LAB_N=10000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/ks_tail_ab.log 2>&1 || { tail -20 $OUT/ks_tail_ab.log; exit 1; }
grep '^{' $OUT/ks_tail_ab.log
for c in 6 14 15 16 17; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-d2h > $OUT/bench_cfg$c.log 2>&1 || { tail $OUT/bench_cfg$c.log; exit 1; }
  grep -h '^{' $OUT/bench_cfg$c.log | python -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d['roofline']
print(d['config']['workload'][:60], '| value', d['value'], '| achieved', r['achieved'], r['frac'], r['avg_launch_ms'], '| ok', d['verified_vs_oracle'])"
done

# GPU tests, smoke and one bench line per config (tooling; run on the GPU box).
# usage: bash tools/round_check.sh <out-subdir> [configs...]
set -o pipefail
OUT=gpurun_out/${1:-check}
shift
CFGS=${*:-3 4 5 6 8 9 10 11 12 13 14 15}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_cfg2.log 2>&1 || { tail $OUT/bench_cfg2.log; exit 1; }
echo "cfg2 done"
for c in $CFGS; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $OUT/bench_cfg$c.log 2>&1 || { tail $OUT/bench_cfg$c.log; exit 1; }
  echo "cfg$c done"
done
grep -h '^{' $OUT/bench_cfg*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); r = d['roofline']
    print(d['config']['workload'][:50], '| value', d['value'], '| achieved', r['achieved'], r['frac'], '| ceiling', r.get('write_ceiling_GBps'), r.get('frac_of_write_ceiling'), '| d2h', d['d2h_inclusive'] and d['d2h_inclusive']['value'], '| cpu', d['cpu_baseline'] and d['cpu_baseline']['value'], '| ok', d['verified_vs_oracle'])"

# Re-check of the restored tree (tests, smoke, cfg2 line) and a kernel trace of
# the single-buffer configs (per-call kernel time vs gap) (tooling).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2j}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_cfg2.log 2>&1 || { tail $OUT/bench_cfg2.log; exit 1; }
grep '^{' $OUT/bench_cfg2.log | cut -c1-400
for c in 11 13; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg$c -o run --output-format csv -- \
      python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-verify > $OUT/bench_trace_cfg$c.log 2>&1 || { tail $OUT/bench_trace_cfg$c.log; exit 1; }
  echo "cfg$c traced"
done

# Per-object DG1 launches: bench-style vs lab-style callers in one process (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2t}
mkdir -p $OUT
timeout -k 10 300 python -u tools/dg1_launch_ab.py > $OUT/dg1_launch_ab.log 2>&1 || { tail -20 $OUT/dg1_launch_ab.log; exit 1; }
grep '^{' $OUT/dg1_launch_ab.log
timeout -k 10 300 python bench.py --config 14 --steps 20 --warmup 5 --no-cpu-baseline --no-d2h --no-ceiling > $OUT/bench_cfg14.log 2>&1 || { tail $OUT/bench_cfg14.log; exit 1; }
grep -h '^{' $OUT/bench_cfg14.log | cut -c1-300

# rocprofv3 evidence for the bench lines (tooling; run on the GPU box):
#   kernel trace + stats for cfg2/cfg4 bench runs, then one PMC pass per
#   counter (WRITE_SIZE, FETCH_SIZE) with no tracing domains.
# usage: bash tools/profile_round.sh <out-subdir>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
for c in 2 4 6; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg$c -o run --output-format csv -- \
      python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-d2h > $OUT/bench_trace_cfg$c.log 2>&1 || exit 1
  for ctr in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/pmc_${ctr}_cfg$c -o run --output-format csv -- \
        python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-d2h --no-verify > $OUT/bench_pmc_${ctr}_cfg$c.log 2>&1 || exit 1
  done
done
find $OUT -name "*.csv" | sort

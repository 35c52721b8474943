# rocprofv3 evidence for the bench lines (tooling; run on the GPU box):
#   kernel trace + stats of a bench run per config (the driver's step count),
#   then one PMC pass per counter (WRITE_SIZE, FETCH_SIZE) with no tracing
#   domains over a one-step run.  Condense with tools/prof_summary.py.
# usage: bash tools/profile_round.sh <out-subdir> [configs...]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
shift
CFGS=${*:-2 3 4 5 6}
mkdir -p $OUT
for c in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg$c -o run --output-format csv -- \
      python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-d2h > $OUT/bench_trace_cfg$c.log 2>&1 || { tail $OUT/bench_trace_cfg$c.log; exit 1; }
  for ctr in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d $OUT/pmc_${ctr}_cfg$c -o run --output-format csv -- \
        python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-d2h --no-verify --no-ceiling > $OUT/bench_pmc_${ctr}_cfg$c.log 2>&1 || { tail $OUT/bench_pmc_${ctr}_cfg$c.log; exit 1; }
  done
  echo "cfg$c profiled"
done

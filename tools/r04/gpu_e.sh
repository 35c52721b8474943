#!/bin/bash
# Round 4, session e: the full GPU suite after the host-path and batch
# changes; host-call floor; host and CPU-baseline bench lines (unpinned vs
# pinned); library A/B (late LDS image, dense records back to round 3's);
# FETCH_SIZE of config 10's records, interleaved vs linear.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04e
mkdir -p $OUT
step() { echo "== $*" >&2; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
step host_floor
timeout -k 10 200 tools/_build/host_floor 300 > $OUT/host_floor.log 2>&1 || exit 1
cat $OUT/host_floor.log
summ() {
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = d["cpu_baseline"] or {}
print(sys.argv[1], d["value"], d["roofline"].get("avg_call_ms") or d["roofline"].get("avg_launch_ms"), d["roofline"]["achieved"],
      d["verified_vs_oracle"], c.get("value"), c.get("min_med_max_GiBps"), c.get("spread"), d["roofline"].get("zero_tune"))
PY
}
b() {  # name, args...
  local name=$1; shift
  step bench $name
  timeout -k 10 300 python -u bench.py "$@" > $OUT/bench_$name.log 2>&1 || { tail -20 $OUT/bench_$name.log; exit 1; }
  summ $OUT/bench_$name.log
}
b cfg18 --config 18 --steps 3 --warmup 1 --cpu-seconds 5
b cfg18_pinned --config 18 --steps 3 --warmup 1 --host-mem pinned --cpu-seconds 5
b cfg19 --config 19 --steps 3 --warmup 1 --cpu-seconds 5
b cfg20 --config 20 --steps 3 --warmup 1 --cpu-seconds 5
b cfg23 --config 23 --steps 3 --warmup 1 --cpu-seconds 5
b cfg2 --config 2 --steps 10 --warmup 2 --cpu-seconds 5
b cfg2_pin --config 2 --steps 10 --warmup 2 --cpu-pin --no-d2h --no-ceiling
b cfg3 --config 3 --steps 10 --warmup 2 --cpu-seconds 5
b cfg5 --config 5 --steps 3 --warmup 1 --cpu-seconds 5
b cfg8 --config 8 --steps 10 --warmup 2 --cpu-seconds 5 --no-ceiling
b cfg9 --config 9 --steps 10 --warmup 2 --cpu-seconds 5 --no-ceiling
step lib_ab
LAB_AB="r03=dedd5d0;head=.;head_lateimg=.:-DS3DG_DIAG_LATEIMG=1" LAB_POINTS="cfg2;cfg3;cfg4;cfg10" LAB_REPS=10 \
    timeout -k 10 500 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 || exit 1
grep -v "rep " $OUT/lib_ab.log
step pmc
for v in dint head; do
  LAB_AB="$v=." LAB_POINTS="cfg10" LAB_REPS=1 LAB_LAUNCHES=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$v -o run --output-format csv -- python3 tools/r04/lib_ab.py > $OUT/pmc_fetch_$v.log 2>&1 || exit 1
done
echo done

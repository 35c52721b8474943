#!/bin/bash
# Round 4, session f: validation of the candidate final tree: the GPU suite,
# host-call floor, the library A/B against round 3, the 1 MiB host lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
step() { echo "== $*" >&2; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
step host_floor
timeout -k 10 200 tools/_build/host_floor 300 > $OUT/host_floor.log 2>&1 || exit 1
grep -o '"bytes": [0-9]*, "drop_pageable": [0-9.]*, "drop_pinned": [0-9.]*' $OUT/host_floor.log
summ() {
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = d["cpu_baseline"] or {}
print(sys.argv[1], d["value"], d["roofline"].get("avg_call_ms") or d["roofline"].get("avg_launch_ms"), d["roofline"]["achieved"],
      d["verified_vs_oracle"], c.get("value"), c.get("min_med_max_GiBps"), c.get("spread"))
PY
}
b() {
  local name=$1; shift
  step bench $name
  timeout -k 10 300 python -u bench.py "$@" > $OUT/bench_$name.log 2>&1 || { tail -20 $OUT/bench_$name.log; exit 1; }
  summ $OUT/bench_$name.log
}
b cfg18 --config 18 --steps 3 --warmup 1 --no-cpu-baseline
b cfg18_pinned --config 18 --steps 3 --warmup 1 --host-mem pinned --no-cpu-baseline
step lib_ab
LAB_AB="r03=dedd5d0;head=." LAB_POINTS="cfg2;cfg3;cfg5;cfg4;cfg10" LAB_REPS=8 \
    timeout -k 10 500 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 || exit 1
grep -v "rep " $OUT/lib_ab.log

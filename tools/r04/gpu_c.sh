#!/bin/bash
# Round 4, session c: GPU tests (new small-call path and read-ahead ring),
# host-call floor lab, library A/B, host / chunk bench lines.
set -o pipefail
OUT=gpurun_out/r04c
mkdir -p $OUT
step() { echo "== $*" >&2; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
step host_floor
timeout -k 10 200 tools/_build/host_floor 300 > $OUT/host_floor.log 2>&1 || exit 1
cat $OUT/host_floor.log
for c in 18 22 23 24 26; do
  step bench $c
  timeout -k 10 240 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 5 > $OUT/bench_cfg$c.log 2>&1 || { tail -20 $OUT/bench_cfg$c.log; exit 1; }
  python - $OUT/bench_cfg$c.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[1], d["value"], d["roofline"].get("avg_call_ms"), d["verified_vs_oracle"], (d["cpu_baseline"] or {}).get("value"))
PY
done
step lib_ab
LAB_AB="r02=aa93058;r03=dedd5d0;head=.;head_dlin=.:-DS3DG_DIAG_DENSE_LINEAR=1" LAB_POINTS="cfg2;cfg3;cfg5;cfg4;cfg10" LAB_REPS=8 timeout -k 10 500 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 || exit 1
grep -v "rep " $OUT/lib_ab.log

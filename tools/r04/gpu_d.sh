#!/bin/bash
# Round 4, session d: small-call copy-out helpers, the 16 MiB host-call check
# (size order reversed), host / chunk bench lines, the CPU-baseline spread on
# configs 2, 8 and 9, and the library A/B with the dense layout split out.
set -o pipefail
OUT=gpurun_out/r04d
mkdir -p $OUT
step() { echo "== $*" >&2; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_small.py tests/test_gpu_datagen.py tests/test_gpu_batch.py \
    tests/test_capi_binding.py tests/test_objects.py tests/test_npz.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
step host_floor
timeout -k 10 200 tools/_build/host_floor 300 rev > $OUT/host_floor_rev.log 2>&1 || exit 1
timeout -k 10 200 tools/_build/host_floor 300 > $OUT/host_floor.log 2>&1 || exit 1
cat $OUT/host_floor_rev.log $OUT/host_floor.log
summ() {
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = d["cpu_baseline"] or {}
print(sys.argv[1], d["value"], d["roofline"].get("avg_call_ms") or d["roofline"].get("avg_launch_ms"), d["roofline"]["achieved"],
      d["verified_vs_oracle"], c.get("value"), c.get("min_med_max_GiBps"), c.get("spread"))
PY
}
for c in 18 19 20 23 24 26 27; do
  step bench $c
  timeout -k 10 240 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 5 > $OUT/bench_cfg$c.log 2>&1 || { tail -20 $OUT/bench_cfg$c.log; exit 1; }
  summ $OUT/bench_cfg$c.log
done
step bench 18 pinned
timeout -k 10 240 python -u bench.py --config 18 --steps 3 --warmup 1 --host-mem pinned --cpu-seconds 5 > $OUT/bench_cfg18_pinned.log 2>&1 || exit 1
summ $OUT/bench_cfg18_pinned.log
step bench 20 small_max=0
S3DLIO_HOST_SMALL_MAX=0 timeout -k 10 240 python -u bench.py --config 19 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_cfg19_dma.log 2>&1 || exit 1
summ $OUT/bench_cfg19_dma.log
for c in 2 3 5 8 9; do
  step bench $c
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 > $OUT/bench_cfg$c.log 2>&1 || { tail -20 $OUT/bench_cfg$c.log; exit 1; }
  summ $OUT/bench_cfg$c.log
done
step lib_ab
LAB_AB="r03=dedd5d0;head=.;head_dlin=.:-DS3DG_DIAG_DENSE_LINEAR=1;head_lateimg=.:-DS3DG_DIAG_LATEIMG=1" LAB_POINTS="cfg2;cfg4;cfg4@8;cfg4@16;cfg4@64;cfg4@256;cfg10;cfg3" LAB_REPS=8 timeout -k 10 500 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 || exit 1
grep -v "rep " $OUT/lib_ab.log

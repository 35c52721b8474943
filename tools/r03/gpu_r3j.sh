# Round 3: batch launch grid cap A/B (2^26-ish vs 2^22 workgroups per launch),
# the split-path test, and copy tracing with each tracer alone.  Tooling.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3j}
mkdir -p $OUT
LAB_VARIANTS="cap26=;cap22=-DS3DG_DIAG_GRID_CAP=4194304" LAB_POINTS="stream2:0:-1:-1:-1;stream3:0:-1:-1:-1;stream5:0:-1:-1:-1;cfg4:0:-1:-1:-1;cfg7:0:-1:-1:-1" LAB_REPS=8 LAB_N=10000 \
  timeout -k 10 300 python -u tools/variant_lab.py > $OUT/grid_cap_ab.log 2>&1 || { tail -20 $OUT/grid_cap_ab.log; exit 1; }
grep '^{' $OUT/grid_cap_ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/parity_tests.log 2>&1 || { tail -30 $OUT/parity_tests.log; exit 1; }
tail -1 $OUT/parity_tests.log
bash tools/r03/gpu_r3i.sh ${1:-r3j}

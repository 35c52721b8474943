# Scalar-unit jump sequence in k_keystream: GPU tests, A/B vs the per-lane
# vector jump (S3DG_KS_JUMP=1) on K2/DG1 launches of 8 GiB and 80 GiB, and the
# wave timeline of 8/64 GiB launches (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2m}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
P="k2:4:0:1024:2;k2_8g:4:0:1024:2;k2_8g:4:0:2048:2;dg1:4:0:1024:2;dg1_8g:4:0:1024:2;dg1_8g:4:0:2048:2;dg1c2_8g:4:0:1024:2;dg1c2_8g:4:0:512:2"
LAB_VARIANTS="new=;old=-DS3DG_KS_JUMP=1" LAB_POINTS="$P" LAB_REPS=3 LAB_N=10000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/ks_jump_ab.log 2>&1 || { tail -20 $OUT/ks_jump_ab.log; exit 1; }
grep '^{' $OUT/ks_jump_ab.log
timeout -k 10 300 python -u tools/ks_trace_lab.py > $OUT/ks_trace.log 2>&1 || { tail -20 $OUT/ks_trace.log; exit 1; }
grep '^{' $OUT/ks_trace.log | cut -c1-600

# Two-chunk waves (32 lanes per chunk): GPU tests, A/B of DG1 lanes 2048 vs 4096 draws (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2y}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
P="dg1:1:0:2048:2:16;dg1:1:0:4096:2:16;dg1_8g:1:0:2048:2:16;dg1_8g:1:0:4096:2:16;dg1:1:0:4096:2:32;dg1_8g:1:0:4096:2:32;k2:1:0:4096:2:16"
LAB_VARIANTS="cur=" LAB_POINTS="$P" LAB_REPS=4 LAB_N=10000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/dg1_draws_ab.log 2>&1 || { tail -20 $OUT/dg1_draws_ab.log; exit 1; }
grep '^{' $OUT/dg1_draws_ab.log

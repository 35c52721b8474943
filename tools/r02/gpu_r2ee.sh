# 128-draw stages (1 KiB rows, one row per store instruction) vs 64 (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2ee}
mkdir -p $OUT
P="k2:1:0:4096:2:16;k2@128:1:0:4096:2:16;k2@128:1:0:4096:2:8;k2@128:2:0:4096:2:16;k2_8g:1:0:4096:2:16;k2_8g@128:1:0:4096:2:16"
P="$P;dg1:1:0:2048:2:16;dg1@128:1:0:2048:2:16;dg1@128:2:0:2048:2:16;dg1_8g:1:0:2048:2:16;dg1_8g@128:1:0:2048:2:16;dg1c2_8g:4:0:512:2:32;dg1c2_8g@128:2:0:512:2:32;dg1c2_8g@128:1:0:512:2:16"
LAB_VARIANTS="cur=" LAB_POINTS="$P" LAB_REPS=3 LAB_N=10000 \
  timeout -k 10 500 python -u tools/variant_lab.py > $OUT/ks_d128.log 2>&1 || { tail -20 $OUT/ks_d128.log; exit 1; }
grep '^{' $OUT/ks_d128.log

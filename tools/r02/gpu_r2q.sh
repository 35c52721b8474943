# XCD-grouped workgroup remap in k_keystream (diagnostic variants) x waves per
# workgroup (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2q}
mkdir -p $OUT
P="k2:1:0:2048:2;k2:4:0:2048:2;k2:1:0:4096:2;k2:4:0:4096:2;dg1:1:0:2048:2;dg1:4:0:2048:2;dg1_8g:1:0:2048:2;dg1_8g:4:0:2048:2"
LAB_VARIANTS="base=;g4=-DS3DG_KS_XCDG=4;g16=-DS3DG_KS_XCDG=16" LAB_POINTS="$P" LAB_REPS=3 LAB_N=10000 \
  timeout -k 10 500 python -u tools/variant_lab.py > $OUT/ks_xcd_group.log 2>&1 || { tail -20 $OUT/ks_xcd_group.log; exit 1; }
grep '^{' $OUT/ks_xcd_group.log

# k_keystream draws-per-lane / waves sweep with the scalar jump (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2n}
mkdir -p $OUT
P="k2:4:0:1024:2;k2:4:0:2048:2;k2:4:0:4096:2;k2:2:0:2048:2;k2:1:0:2048:2;k2_8g:4:0:1024:2;k2_8g:4:0:2048:2;k2_8g:4:0:4096:2"
P="$P;dg1:4:0:1024:2;dg1:4:0:2048:2;dg1:2:0:2048:2;dg1_8g:4:0:1024:2;dg1_8g:4:0:2048:2;dg1c2_8g:4:0:512:2;dg1c2_8g:4:0:2048:2"
LAB_VARIANTS="new=" LAB_POINTS="$P" LAB_REPS=3 LAB_N=10000 \
  timeout -k 10 500 python -u tools/variant_lab.py > $OUT/ks_draws_sweep.log 2>&1 || { tail -20 $OUT/ks_draws_sweep.log; exit 1; }
grep '^{' $OUT/ks_draws_sweep.log

# k_keystream stage depth x waves x XCD group at the new defaults (runtime knobs, tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2dd}
mkdir -p $OUT
P="k2:1:0:4096:2:16;k2@32:1:0:4096:2:16;k2@32:1:0:4096:2:32;k2@32:2:0:4096:2:16;k2@16:1:0:4096:2:16;k2@16:4:0:4096:2:32"
P="$P;dg1:1:0:2048:2:16;dg1@32:1:0:2048:2:16;dg1@32:2:0:2048:2:32;dg1@16:1:0:2048:2:16"
LAB_VARIANTS="cur=" LAB_POINTS="$P" LAB_REPS=3 LAB_N=10000 \
  timeout -k 10 500 python -u tools/variant_lab.py > $OUT/ks_stage_sweep.log 2>&1 || { tail -20 $OUT/ks_stage_sweep.log; exit 1; }
grep '^{' $OUT/ks_stage_sweep.log

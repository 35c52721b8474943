# First-round stagger A/B for k_keystream, sustained per-object launches (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2bb}
mkdir -p $OUT
LAB_VARIANTS="base=;st8=-DS3DG_KS_STAGGER=8;st32=-DS3DG_KS_STAGGER=32;st127=-DS3DG_KS_STAGGER=127" \
  timeout -k 10 400 python -u tools/ks_sustained_ab.py > $OUT/ks_stagger_ab.log 2>&1 || { tail -20 $OUT/ks_stagger_ab.log; exit 1; }
grep '^{' $OUT/ks_stagger_ab.log

# XCD-group size sweep for k_keystream (runtime knob) and GPU tests (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2r}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
P=""
for k in k2:4096 k2_8g:2048 dg1:2048 dg1_8g:2048 dg1c2_8g:512; do
  kind=${k%%:*}; dr=${k##*:}
  for wx in 4:4 4:16 4:32 4:64 4:128 1:16 1:32 1:64 1:128; do
    w=${wx%%:*}; x=${wx##*:}
    P="$P;$kind:$w:0:$dr:2:$x"
  done
done
P=${P#;}
LAB_VARIANTS="cur=" LAB_POINTS="$P" LAB_REPS=3 LAB_N=10000 \
  timeout -k 10 600 python -u tools/variant_lab.py > $OUT/ks_xcd_sweep.log 2>&1 || { tail -20 $OUT/ks_xcd_sweep.log; exit 1; }
grep '^{' $OUT/ks_xcd_sweep.log

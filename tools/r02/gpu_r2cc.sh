# Fill kernel (tiled path): XCD runs of G adjacent slots instead of the dealing order (diagnostic A/B, tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2cc}
mkdir -p $OUT
D=4294967295
LAB_VARIANTS="base=;x2=;x4=;x8=;x32=" LAB_POINTS="stream2:0:-1:$D:-1;stream3:0:-1:$D:-1;cfg4:0:-1:$D:-1;kb64:0:-1:$D:-1" LAB_REPS=4 LAB_N=10000 \
  timeout -k 10 500 python -u tools/variant_lab.py > $OUT/fill_xcd_runs_ab.log 2>&1 || { tail -20 $OUT/fill_xcd_runs_ab.log; exit 1; }
grep '^{' $OUT/fill_xcd_runs_ab.log

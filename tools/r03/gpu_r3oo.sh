# Round 3: where config 4's structure loses against uniform 8 MiB batches:
# its sizes at d1 c1, rounded up to whole 64-block tiles, and sorted largest
# first, against config 7 (tools/variant_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3oo}
mkdir -p $OUT
LAB_VARIANTS="base=" LAB_POINTS="cfg4d1:0:-1:-1:-1;cfg4r:0:-1:-1:-1;cfg4desc:0:-1:-1:-1;cfg7:0:-1:-1:-1;cfg4:0:-1:-1:-1" LAB_REPS=6 LAB_N=10000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/cfg4_structure.log 2>&1 || { tail -20 $OUT/cfg4_structure.log; exit 1; }
grep '^{' $OUT/cfg4_structure.log

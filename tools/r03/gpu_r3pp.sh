# Round 3: config 4 with forced tile sizes (64/32/16/8 blocks per record):
# dead slots vs records (tools/variant_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3pp}
mkdir -p $OUT
LAB_VARIANTS="base=" LAB_POINTS="cfg4:0:-1:-1:-1:0;cfg4:0:-1:-1:-1:64;cfg4:0:-1:-1:-1:32;cfg4:0:-1:-1:-1:16;cfg4:0:-1:-1:-1:8;cfg7:0:-1:-1:-1:0;cfg7:0:-1:-1:-1:16;kb64:0:-1:-1:-1:0;kb64:0:-1:-1:-1:16" LAB_REPS=6 LAB_N=10000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/cfg4_tiles.log 2>&1 || { tail -20 $OUT/cfg4_tiles.log; exit 1; }
grep '^{' $OUT/cfg4_tiles.log

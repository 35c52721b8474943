# Round 3: batch tile-size choice, new tiled cost model (base) vs the first
# model (old), on config 4, its d1 sizes, log-uniform small objects, 1 MiB +
# 123 B objects, 64 KiB and 20 KiB + 5 B objects, uniform 8 MiB
# (tools/variant_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3qq}
mkdir -p $OUT
LAB_VARIANTS="base=;old=-DS3DG_DIAG_OLDTILECOST=1" LAB_POINTS="cfg4:0:-1:-1:-1;cfg4d1:0:-1:-1:-1;small:0:-1:-1:-1;mid:0:-1:-1:-1;cfg7:0:-1:-1:-1" LAB_REPS=10 LAB_ALTERNATE=1 LAB_N=10000 \
  timeout -k 10 500 python -u tools/variant_lab.py > $OUT/tile_cost_ab.log 2>&1 || { tail -20 $OUT/tile_cost_ab.log; exit 1; }
grep '^{' $OUT/tile_cost_ab.log

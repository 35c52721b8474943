# Round 3: config 4's sizes through the dense per-granule layout vs the
# per-launch choice (64-block tiles), one process (tools/variant_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3n}
mkdir -p $OUT
LAB_VARIANTS="base=" LAB_POINTS="cfg4:0:-1:-1:-1;cfg4:0:-1:-1:-1:1;cfg4:0:-1:-1:3:1;cfg4d1:0:-1:-1:-1;cfg4d1:0:-1:-1:-1:1;cfg7:0:-1:-1:-1;cfg7:0:-1:-1:-1:1;kb20:0:-1:-1:-1;kb20:0:-1:-1:3:1" LAB_REPS=6 LAB_N=10000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/cfg4_dense_ab.log 2>&1 || { tail -20 $OUT/cfg4_dense_ab.log; exit 1; }
grep '^{' $OUT/cfg4_dense_ab.log

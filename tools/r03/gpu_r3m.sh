# Round 3: where config 4 (d2 c1.5, log-uniform sizes) loses against uniform
# 8 MiB batches: the same sizes at d1 c1 and d2 c1, interleaved in one
# process with config 2/3 streams as controls (tools/variant_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3m}
mkdir -p $OUT
LAB_VARIANTS="base=" LAB_POINTS="cfg4:0:-1:-1:-1;cfg4d1:0:-1:-1:-1;cfg4c1:0:-1:-1:-1;cfg7:0:-1:-1:-1;stream2:0:-1:-1:-1;stream3:0:-1:-1:-1;kb20:0:-1:-1:-1" LAB_REPS=6 LAB_N=10000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/cfg4_data_ab.log 2>&1 || { tail -20 $OUT/cfg4_data_ab.log; exit 1; }
grep '^{' $OUT/cfg4_data_ab.log

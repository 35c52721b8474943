# CRC A/B on random data: row-advance tables in LDS vs global (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2i}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_npz.py tests/test_put.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_crc_tests.log 2>&1 || { tail -40 $OUT/gpu_crc_tests.log; exit 1; }
tail -1 $OUT/gpu_crc_tests.log
for v in global lds global lds; do
  S3DG_CRC_TROW=$v LAB_REPS=3 LAB_GIB=17 LAB_KINDS=crcr timeout -k 10 200 python -u tools/lab_r2.py > $OUT/lab_$v.log 2>&1 || { tail -20 $OUT/lab_$v.log; exit 1; }
  echo "$v $(grep '^{' $OUT/lab_$v.log)"
done

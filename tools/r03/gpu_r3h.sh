# Round 3: CRC region sizing + PUT region CRCs written by the kernel into the
# pinned slot: tests, CRC A/B, PUT throughput, CRC overlap timeline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3h}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_put.py tests/test_capi_binding.py tests/test_npz.py tests/test_gpu_regress.py tests/test_gpu_datagen.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for k in 0 1; do
  S3DG_CRC_KERNEL=$k timeout -k 10 120 python -u tools/crc_lab.py >> $OUT/crc_lab.log 2>&1 || { tail $OUT/crc_lab.log; exit 1; }
done
grep '^{' $OUT/crc_lab.log
PUT_N=1024 timeout -k 10 300 python -u tools/bench_put.py > $OUT/put_bench.log 2>&1 || { tail $OUT/put_bench.log; exit 1; }
grep '^{' $OUT/put_bench.log
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/crc_tl -o t --output-format csv -- python3 tools/crc_timeline.py run > $OUT/crc_tl.log 2>&1 || { tail $OUT/crc_tl.log; exit 1; }
python3 tools/crc_timeline.py summarize $OUT/crc_tl | tee $OUT/crc_tl_summary.json
timeout -k 10 200 python -u tools/hostbuf_lab.py > $OUT/hostbuf_lab.log 2>&1 || { tail $OUT/hostbuf_lab.log; exit 1; }
grep '^{' $OUT/hostbuf_lab.log

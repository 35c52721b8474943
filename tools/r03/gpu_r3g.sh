# Round 3: PUT pipeline reorder (fill + CRC of chunk k+1 before chunk k's D2H):
# tests, throughput, CRC overlap timeline; CRC kernel counters (both forms).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3g}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_put.py tests/test_capi_binding.py tests/test_npz.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_put.log 2>&1 || { tail -30 $OUT/gpu_tests_put.log; exit 1; }
tail -1 $OUT/gpu_tests_put.log
PUT_N=1024 timeout -k 10 300 python -u tools/bench_put.py > $OUT/put_bench.log 2>&1 || { tail $OUT/put_bench.log; exit 1; }
grep '^{' $OUT/put_bench.log
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/crc_tl -o t --output-format csv -- python3 tools/crc_timeline.py run > $OUT/crc_tl.log 2>&1 || { tail $OUT/crc_tl.log; exit 1; }
python3 tools/crc_timeline.py summarize $OUT/crc_tl | tee $OUT/crc_tl_summary.json
for k in 0 1; do
  S3DG_CRC_KERNEL=$k CRC_GIB=8 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_crc$k -o p --output-format csv -- python3 tools/crc_lab.py > $OUT/pmc_crc$k.log 2>&1 || { tail $OUT/pmc_crc$k.log; exit 1; }
  echo "crc pmc $k done"
done

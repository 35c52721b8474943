# Round 3: tests touched by the k_batch_map / NPZ / stream-release changes, the
# NPZ output-buffer lab and the CRC overlap timeline again.  Tooling; GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3e}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fuzz.py tests/test_npz.py tests/test_gpu_regress.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_subset.log 2>&1 || { tail -30 $OUT/gpu_tests_subset.log; exit 1; }
tail -1 $OUT/gpu_tests_subset.log
timeout -k 10 200 python -u tools/npz_lab.py > $OUT/npz_lab.log 2>&1 || { tail $OUT/npz_lab.log; exit 1; }
grep '^{' $OUT/npz_lab.log
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/crc_tl -o t --output-format csv -- python3 tools/crc_timeline.py run > $OUT/crc_tl.log 2>&1 || { tail $OUT/crc_tl.log; exit 1; }
python3 tools/crc_timeline.py summarize $OUT/crc_tl | tee $OUT/crc_tl_summary.json

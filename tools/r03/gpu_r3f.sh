# Round 3: full GPU test suite, CRC kernel A/B (conflict-free vs round 2), NPZ
# output-buffer lab, CRC overlap timeline.  Tooling; GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3f}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for k in 0 1 0 1; do
  S3DG_CRC_KERNEL=$k timeout -k 10 120 python -u tools/crc_lab.py >> $OUT/crc_lab.log 2>&1 || { tail $OUT/crc_lab.log; exit 1; }
done
grep '^{' $OUT/crc_lab.log
timeout -k 10 200 python -u tools/npz_lab.py > $OUT/npz_lab.log 2>&1 || { tail $OUT/npz_lab.log; exit 1; }
grep '^{' $OUT/npz_lab.log
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/crc_tl -o t --output-format csv -- python3 tools/crc_timeline.py run > $OUT/crc_tl.log 2>&1 || { tail $OUT/crc_tl.log; exit 1; }
python3 tools/crc_timeline.py summarize $OUT/crc_tl | tee $OUT/crc_tl_summary.json

# Round 3: GPU test suite at the current tree, then the CRC overlap timeline
# (VERDICT r02 next #6).  Tooling; GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3d}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/crc_tl -o t --output-format csv -- python3 tools/crc_timeline.py run > $OUT/crc_tl.log 2>&1 || { tail $OUT/crc_tl.log; exit 1; }
python3 tools/crc_timeline.py summarize $OUT/crc_tl | tee $OUT/crc_tl_summary.json

# Round 3: are D2H copies blit kernels only under the memory-copy tracer?
# The same NPZ + PUT run traced with --kernel-trace alone and with
# --memory-copy-trace alone.  Tooling; GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3i}
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/kt -o t --output-format csv -- python3 tools/crc_timeline.py run > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
timeout -k 10 240 rocprofv3 --memory-copy-trace -d $OUT/mc -o t --output-format csv -- python3 tools/crc_timeline.py run > $OUT/mc.log 2>&1 || { tail $OUT/mc.log; exit 1; }
find $OUT -name "*.csv" | xargs wc -l

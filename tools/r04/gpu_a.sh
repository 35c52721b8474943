#!/bin/bash
# Round 4, first GPU session: library A/B on config 2 (r02 vs r03 vs this
# tree, bisection variants) and the host-call floor lab.
set -o pipefail
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 400 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 && \
timeout -k 10 200 tools/_build/host_floor 300 > $OUT/host_floor.log 2>&1
rc=$?
tail -30 $OUT/lib_ab.log
cat $OUT/host_floor.log
exit $rc

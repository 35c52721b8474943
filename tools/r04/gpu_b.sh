#!/bin/bash
# Round 4, session b: library A/B with the floor-free batch instantiation;
# host-call floor lab with and without SDMA copies.
set -o pipefail
OUT=gpurun_out/r04b
mkdir -p $OUT
LAB_AB="r02=aa93058;r03=dedd5d0;head=." LAB_REPS=8 timeout -k 10 400 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 && \
timeout -k 10 200 tools/_build/host_floor 300 > $OUT/host_floor.log 2>&1 && \
HSA_ENABLE_SDMA=0 timeout -k 10 200 tools/_build/host_floor 300 > $OUT/host_floor_nosdma.log 2>&1
rc=$?
grep -v "rep " $OUT/lib_ab.log
cat $OUT/host_floor.log $OUT/host_floor_nosdma.log
exit $rc

#!/bin/bash
# Round 4, session g: the LDS image written after wave 0's plan (diagnostic
# build) against this tree, interleaved in one process.
set -o pipefail
OUT=gpurun_out/r04g
mkdir -p $OUT
LAB_AB="head=.;imgplan=.:-DS3DG_DIAG_IMGPLAN=1" LAB_POINTS="cfg2;cfg3;cfg5;cfg4;cfg10" LAB_REPS=10 \
    timeout -k 10 500 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 || exit 1
grep -v "rep " $OUT/lib_ab.log

#!/bin/bash
# Round 4, session i: dead batch slots that still prefetch their span's
# records (diagnostic build -DS3DG_DIAG_DEADPF=1) against this tree (the
# prefetch moved into a lambda) and the round-4 final sources (013b5e5),
# interleaved in one process; dpfup adds the descriptor upload and record map
# on a high-priority stream (-DS3DG_DIAG_UPPRIO=1).  kb20g: 2 000 000 x 20 KiB
# at a 24 KiB stride.
set -o pipefail
OUT=gpurun_out/${1:-r04i}
mkdir -p $OUT
LAB_AB="r04=013b5e5;head=.;dpf=.:-DS3DG_DIAG_DEADPF=1;dpfup=.:-DS3DG_DIAG_DEADPF=1 -DS3DG_DIAG_UPPRIO=1" LAB_POINTS="cfg2;cfg4;cfg10;kb20g;cfg3;cfg5" LAB_REPS=8 \
    timeout -k 10 600 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 || { tail -20 $OUT/lib_ab.log; exit 1; }
grep -v "rep " $OUT/lib_ab.log

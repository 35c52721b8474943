#!/bin/bash
# Round 4, session l: DG1 with a zero prefix under 1-wave / 4-wave and static /
# persistent launch shapes (tools/r04/ks_c2_lab.py).
set -o pipefail
OUT=gpurun_out/${1:-r04l}
mkdir -p $OUT
timeout -k 10 500 python -u tools/r04/ks_c2_lab.py > $OUT/ks_c2.log 2>&1 || { tail -20 $OUT/ks_c2.log; exit 1; }
grep '^{' $OUT/ks_c2.log

#!/bin/bash
# Round 4, session m: per-XCD end times of the fill (tools/r04/fill_xcd_lab.py,
# diagnostic copy of the library).
set -o pipefail
OUT=gpurun_out/${1:-r04m}
mkdir -p $OUT
timeout -k 10 400 python -u tools/r04/fill_xcd_lab.py > $OUT/fill_xcd.log 2>&1 || { tail -20 $OUT/fill_xcd.log; exit 1; }
grep '^{' $OUT/fill_xcd.log

#!/bin/bash
# Round 4, session j: DG1 wave timelines, ten 8 GiB launches vs one 80 GiB
# launch (tools/r04/ks_rounds_lab.py, diagnostic trace build).
set -o pipefail
OUT=gpurun_out/${1:-r04j}
mkdir -p $OUT
timeout -k 10 400 python -u tools/r04/ks_rounds_lab.py > $OUT/ks_rounds.log 2>&1 || { tail -20 $OUT/ks_rounds.log; exit 1; }
grep '^{' $OUT/ks_rounds.log

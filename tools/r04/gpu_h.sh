#!/bin/bash
# Round 4, session h: what a batch workgroup costs.  Kernel traces of the
# fill over layouts that differ only in their slots: config 10's objects
# (20 KiB + 5 B at 24 KiB: 5 full slots + one 5-byte slot), the same objects
# without the 5 bytes packed (5 slots) and at 24 KiB (5 slots + one dead
# slot), config 4's sizes as they are and rounded to 64-block tiles, and
# uniform 8 MiB objects.  One process per kind; tools/r04/wg_cost.py reads
# the traces (fill time per workgroup slot and per byte).
set -o pipefail
OUT=gpurun_out/${1:-r04h}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for k in kb20 kb20n kb20g cfg4d1 cfg4r cfg7; do
    LAB_VARIANTS="base=" LAB_POINTS="$k:0:-1:-1:-1:0" LAB_REPS=3 LAB_N=10000 LAB_NSMALL=2000000 \
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$k -o run -- \
        python3 -u tools/variant_lab.py > $OUT/$k.log 2>&1 || { tail -20 $OUT/$k.log; exit 1; }
    grep '^{' $OUT/$k.log
done
python3 tools/r04/wg_cost.py $OUT

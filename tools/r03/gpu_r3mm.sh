# Round 3: what the 5-byte tail workgroups of config 10 cost: 2 M objects of
# 20 KiB + 5 B (6 live slots), 20 KiB at a 24 KiB stride (5 live + 1 dead),
# 20 KiB packed (5 live), batch API, per-launch layout (tools/variant_lab.py).
set -o pipefail
OUT=gpurun_out/${1:-r3mm}
mkdir -p $OUT
LAB_VARIANTS="base=" LAB_POINTS="kb20:0:-1:-1:-1;kb20g:0:-1:-1:-1;kb20n:0:-1:-1:-1;stream2:0:-1:-1:-1" LAB_REPS=6 LAB_N=1000 LAB_NSMALL=2000000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/tail_cost.log 2>&1 || { tail -20 $OUT/tail_cost.log; exit 1; }
grep '^{' $OUT/tail_cost.log

# Round 3, config-3 diagnosis and the keystream EA counter
# pass (next #5).  Tooling; run on the GPU box after
#   LAB_VARIANTS="base=;zconst=-DS3DG_DIAG_ZERO=1;zlds=-DS3DG_DIAG_ZERO=2;zff=-DS3DG_DIAG_ZERO=1 -DS3DG_DIAG_ZVAL=0xFFFFFFFFu" \
#     python tools/variant_lab.py --build-only
# Variants: zconst = zero pieces store 0x5A5A5A5A (same instructions, other
# data), zff = 0xFFFFFFFF, zlds = zero pieces also read their LDS piece (same
# data, store stream paced like a prefix-free block).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3a}
mkdir -p $OUT
ALLV="base=;zconst=-DS3DG_DIAG_ZERO=1;zlds=-DS3DG_DIAG_ZERO=2;zff=-DS3DG_DIAG_ZERO=1 -DS3DG_DIAG_ZVAL=0xFFFFFFFFu"
P="stream2:0:-1:-1:-1;stream3:0:-1:-1:-1;sd1x1x2:0:-1:-1:-1;sd1x3x4:0:-1:-1:-1;sd4x0x1:0:-1:-1:-1"
LAB_VARIANTS="$ALLV" LAB_POINTS="$P" LAB_REPS=8 LAB_N=10000 \
  timeout -k 10 300 python -u tools/variant_lab.py > $OUT/cfg3_zero_ab.log 2>&1 || { tail -20 $OUT/cfg3_zero_ab.log; exit 1; }
grep '^{' $OUT/cfg3_zero_ab.log
# EA write counters per variant (one --pmc pass each, no tracing domains)
PC="stream2:0:-1:-1:-1;stream3:0:-1:-1:-1;sd1x3x4:0:-1:-1:-1"
for v in base zconst zlds; do
  spec=$(echo "$ALLV" | tr ';' '\n' | grep "^$v=")
  LAB_VARIANTS="$spec" LAB_POINTS="$PC" LAB_REPS=1 LAB_N=10000 \
    timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE \
      -d $OUT/pmc_$v -o p --output-format csv -- python3 tools/variant_lab.py > $OUT/pmc_$v.log 2>&1 || { tail $OUT/pmc_$v.log; exit 1; }
  echo "pmc $v done"
done
# keystream (K2 one launch = config 6, DG1 8 GiB launches = config 14) vs the fill (config 2)
PK="stream2:0:-1:-1:-1;k2:0:0:0:-1;dg1_8g:0:0:0:-1"
LAB_VARIANTS="base=" LAB_POINTS="$PK" LAB_REPS=1 LAB_N=10000 \
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE \
    -d $OUT/pmc_ks -o p --output-format csv -- python3 tools/variant_lab.py > $OUT/pmc_ks.log 2>&1 || { tail $OUT/pmc_ks.log; exit 1; }
echo "pmc ks done"
find $OUT -name "*counter_collection.csv"

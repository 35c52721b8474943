# Round 3: two 4 KiB block slots per batch-kernel workgroup (S3DG_DIAG_BPW=2)
# vs one, interleaved in one process (tools/variant_lab.py).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3bb}
mkdir -p $OUT
LAB_VARIANTS="base=;bpw2=-DS3DG_DIAG_BPW=2" LAB_POINTS="stream2:0:-1:-1:-1;stream3:0:-1:-1:-1;stream5:0:-1:-1:-1;cfg4:0:-1:-1:-1;cfg7:0:-1:-1:-1;kb64:0:-1:-1:-1;kb20:0:-1:-1:-1" LAB_REPS=6 LAB_N=10000 \
  timeout -k 10 400 python -u tools/variant_lab.py > $OUT/bpw_ab.log 2>&1 || { tail -20 $OUT/bpw_ab.log; exit 1; }
grep '^{' $OUT/bpw_ab.log

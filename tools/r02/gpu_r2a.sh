# Round-2 diagnosis pass on the GPU box (tooling): lab rates, a kernel trace of
# the lab, the counter list, and PMC passes on the CRC kernel and on the fill
# vs the store-only shapes.  Every step has its own time limit; the first
# failure ends the script.
# usage: bash tools/r02/gpu_r2a.sh <out-subdir>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2a}
mkdir -p $OUT
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 400 python -u tools/lab_r2.py > $OUT/lab.log 2>&1 || { tail -20 $OUT/lab.log; exit 1; }
grep '^{' $OUT/lab.log
LAB_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o lab --output-format csv -- \
    python3 tools/lab_r2.py > $OUT/lab_trace.log 2>&1 || { tail -20 $OUT/lab_trace.log; exit 1; }
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
export LAB_REPS=1
LAB_KINDS=crc timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d $OUT/pmc_crc1 -o p --output-format csv -- python3 tools/lab_r2.py > $OUT/pmc_crc1.log 2>&1 || { tail $OUT/pmc_crc1.log; exit 1; }
LAB_KINDS=crc timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
    -d $OUT/pmc_crc2 -o p --output-format csv -- python3 tools/lab_r2.py > $OUT/pmc_crc2.log 2>&1 || { tail $OUT/pmc_crc2.log; exit 1; }
LAB_KINDS=cfg2,ceil_tiled,ceil timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE \
    -d $OUT/pmc_wr1 -o p --output-format csv -- python3 tools/lab_r2.py > $OUT/pmc_wr1.log 2>&1 || { tail $OUT/pmc_wr1.log; exit 1; }
find $OUT -name "*.csv" | sort

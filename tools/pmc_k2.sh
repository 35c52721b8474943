# SQ/GRBM counters of the K2 keystream kernel (tooling; run on the GPU box).
# Two --pmc passes (no tracing domains) over tools/k2_lab.py at one shape;
# k_keystream dispatches alternate K2 (mode 0) and DG1 (mode 1).
# usage: bash tools/pmc_k2.sh [out-subdir]
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_k2}
mkdir -p $OUT
export LAB_REPS=1 LAB_POINTS='64:4:0:2048:2' LAB_GIB=31.25
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/p1 -o p1 --output-format csv -- python3 tools/k2_lab.py > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR -d $OUT/p2 -o p2 --output-format csv -- python3 tools/k2_lab.py > $OUT/p2.log 2>&1
find $OUT -name "*counter_collection.csv"

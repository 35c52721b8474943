# Double-buffered batch maps check + CRC bank conflicts on random data (tooling).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2h}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fuzz.py -x -q --timeout 240 --timeout-method thread > $OUT/gpu_batch.log 2>&1 || { tail -40 $OUT/gpu_batch.log; exit 1; }
tail -1 $OUT/gpu_batch.log
LAB_KINDS=b20k,b20k@1,b64k,cfg2,crc timeout -k 10 300 python -u tools/lab_r2.py > $OUT/lab.log 2>&1 || { tail -20 $OUT/lab.log; exit 1; }
grep '^{' $OUT/lab.log
LAB_REPS=1 LAB_KINDS=crc,cfg2,crc timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
    -d $OUT/pmc_crc_random -o p --output-format csv -- python3 tools/lab_r2.py > $OUT/pmc_crc.log 2>&1 || { tail $OUT/pmc_crc.log; exit 1; }
echo done

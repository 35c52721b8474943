# Full GPU suite, CRC/keystream lab at the new defaults, and the N=8 launcher
# rehearsal on one GPU (8 ranks on device 0; a launcher test, not scaling).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
LAB_KINDS=crc,dg1c1,dg1c2,k2,cfg2 timeout -k 10 300 python -u tools/lab_r2.py > $OUT/lab.log 2>&1 || { tail -20 $OUT/lab.log; exit 1; }
grep '^{' $OUT/lab.log
LAB_REPS=1 LAB_KINDS=crc timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
    -d $OUT/pmc_crc -o p --output-format csv -- python3 tools/lab_r2.py > $OUT/pmc_crc.log 2>&1 || { tail $OUT/pmc_crc.log; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 8 --device-override 0 --objects 64 --config 2 --steps 3 --warmup 1 > $OUT/rehearsal_n8_cfg2.log 2>&1 || { tail -30 $OUT/rehearsal_n8_cfg2.log; exit 1; }
grep '^{' $OUT/rehearsal_n8_cfg2.log | cut -c1-400
timeout -k 10 400 python -u bench.py --gpus 8 --device-override 0 --objects 800 --config 5 --steps 3 --warmup 1 > $OUT/rehearsal_n8_cfg5.log 2>&1 || { tail -30 $OUT/rehearsal_n8_cfg5.log; exit 1; }
grep '^{' $OUT/rehearsal_n8_cfg5.log | cut -c1-400
echo done

# Dense-batch prefetch check and the CRC clock hypothesis (tooling).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2g}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 240 --timeout-method thread > $OUT/gpu_batch.log 2>&1 || { tail -40 $OUT/gpu_batch.log; exit 1; }
tail -1 $OUT/gpu_batch.log
LAB_KINDS=b20k,b20k@1,b20k@8,b64k,s20k timeout -k 10 300 python -u tools/lab_r2.py > $OUT/lab.log 2>&1 || { tail -20 $OUT/lab.log; exit 1; }
grep '^{' $OUT/lab.log
LAB_REPS=2 LAB_KINDS=crc,cfg2,crc timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_INSTS_VALU \
    -d $OUT/pmc_clk -o p --output-format csv -- python3 tools/lab_r2.py > $OUT/pmc_clk.log 2>&1 || { tail $OUT/pmc_clk.log; exit 1; }
echo done

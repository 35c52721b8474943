# Batch host-prep check (tooling): batch tests, then small-object lab and a
# kernel trace of it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2e}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $OUT/gpu_batch.log 2>&1 || { tail -40 $OUT/gpu_batch.log; exit 1; }
tail -1 $OUT/gpu_batch.log
LAB_KINDS=b64k,b20k,b20k@1,b20k@8,cfg2 timeout -k 10 300 python -u tools/lab_r2.py > $OUT/lab.log 2>&1 || { tail -20 $OUT/lab.log; exit 1; }
grep '^{' $OUT/lab.log
LAB_REPS=1 LAB_KINDS=b20k,b20k@1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o lab --output-format csv -- python3 tools/lab_r2.py > $OUT/lab_trace.log 2>&1 || { tail -20 $OUT/lab_trace.log; exit 1; }
echo done

# Batch host-prep + CRC + keystream-shape check (tooling).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2e}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_npz.py tests/test_put.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
LAB_KINDS=b64k,b20k,b20k@1,b20k@8,cfg2,crc timeout -k 10 300 python -u tools/lab_r2.py > $OUT/lab.log 2>&1 || { tail -20 $OUT/lab.log; exit 1; }
grep '^{' $OUT/lab.log
LAB_REPS=1 LAB_KINDS=b20k,b20k@1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o lab --output-format csv -- python3 tools/lab_r2.py > $OUT/lab_trace.log 2>&1 || { tail -20 $OUT/lab_trace.log; exit 1; }
LAB_K2KINDS=dg1c1,dg1,k2 LAB_GIB=32 LAB_REPS=2 LAB_POINTS="16:2:0:1024:0;64:4:0:2048:2;64:4:0:1024:2;64:2:0:1024:2;32:2:0:1024:2;32:4:0:2048:2;16:4:0:2048:2;64:4:0:2048:0" timeout -k 10 300 python -u tools/k2_lab.py > $OUT/k2_lab.log 2>&1 || { tail -20 $OUT/k2_lab.log; exit 1; }
grep '^{' $OUT/k2_lab.log
echo done

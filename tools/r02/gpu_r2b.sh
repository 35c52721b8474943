# Round-2 check (tooling): new batch/slot tests, the whole GPU suite, smoke,
# then the lab on the batch path and the ceilings.
# usage: bash tools/r02/gpu_r2b.sh <out-subdir>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2b}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 240 --timeout-method thread > $OUT/gpu_batch.log 2>&1 || { tail -40 $OUT/gpu_batch.log; exit 1; }
tail -2 $OUT/gpu_batch.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
LAB_KINDS=${LAB_KINDS:-b64k,b64k@1,b20k,b20k@1,b20k@8,s64k,cfg2,ceil_fill,ceil_tiled,cfg3} timeout -k 10 400 python -u tools/lab_r2.py > $OUT/lab.log 2>&1 || { tail -20 $OUT/lab.log; exit 1; }
grep '^{' $OUT/lab.log

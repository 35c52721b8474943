# Round-4 final tree: GPU tests, smoke, fuzz soak x15 (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r4final_tests}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
echo smoke ok
S3DG_FUZZ_SOAK=15 timeout -k 10 700 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/fuzz_soak_x15.log 2>&1 || { tail -30 $OUT/fuzz_soak_x15.log; exit 1; }
tail -1 $OUT/fuzz_soak_x15.log

# Round 3, final tree: a longer seeded fuzz soak (x50 = 1300 cases) (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r3nn}
mkdir -p $OUT
S3DG_FUZZ_SOAK=50 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 800 --timeout-method thread > $OUT/fuzz_soak_x50.log 2>&1 || { tail -30 $OUT/fuzz_soak_x50.log; exit 1; }
tail -1 $OUT/fuzz_soak_x50.log

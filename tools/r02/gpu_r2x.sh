# Final tree: fuzz soak x15 and the N=8 launcher rehearsal on one GPU (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2x}
mkdir -p $OUT
S3DG_FUZZ_SOAK=15 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/fuzz_soak_x15.log 2>&1 || { tail -30 $OUT/fuzz_soak_x15.log; exit 1; }
tail -1 $OUT/fuzz_soak_x15.log
timeout -k 10 300 python bench.py --gpus 8 --device-override 0 --objects 64 --config 2 --steps 3 --warmup 1 --no-ceiling > $OUT/rehearsal_n8_cfg2.log 2>&1 || { tail -20 $OUT/rehearsal_n8_cfg2.log; exit 1; }
grep -h '^{' $OUT/rehearsal_n8_cfg2.log | cut -c1-300

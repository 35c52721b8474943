set -o pipefail
mkdir -p gpurun_out/k2
timeout -k 10 300 python -m pytest tests/test_gpu_datagen.py tests/test_npz.py tests/test_gpu_parity.py -m gpu -x -q -k "xoshiro or keystream or k2 or npz or dgen or generator or Generator or crc" > gpurun_out/k2/tests_default.log 2>&1
S3DLIO_K2_MIN_DRAWS=128 timeout -k 10 300 python -m pytest tests/test_gpu_datagen.py tests/test_npz.py tests/test_gpu_parity.py -m gpu -x -q -k "xoshiro or keystream or k2 or npz or dgen or generator or Generator or crc" > gpurun_out/k2/tests_md128.log 2>&1
for md in 2048 1024 512 256 128; do
  S3DLIO_K2_MIN_DRAWS=$md timeout -k 10 200 python bench.py --config 6 --steps 3 --warmup 1 --no-cpu-baseline --no-d2h > gpurun_out/k2/bench_md$md.log 2>&1 || exit 1
done

# GPU parity for the fill kernels, then cfg2/3/4 bench lines (tooling)
set -o pipefail
mkdir -p gpurun_out/bs
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_capi.py -m gpu -x -q > gpurun_out/bs/tests.log 2>&1 || exit 1
for c in 2 4 3; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-d2h > gpurun_out/bs/bench_cfg$c.log 2>&1 || exit 1
done

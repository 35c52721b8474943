mkdir -p gpurun_out/bis
for f in test_gpu_datagen test_npz test_objects test_gpu_parity test_capi; do
  timeout -k 10 300 python -m pytest tests/$f.py tests/test_put.py -m gpu -q -k "not concurrent" > gpurun_out/bis/$f.log 2>&1
  echo "$f rc=$?" >> gpurun_out/bis/summary.txt
done

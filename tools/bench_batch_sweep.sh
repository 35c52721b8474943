set -o pipefail
mkdir -p gpurun_out/bw
for c in 4 7; do for w in 1 2 4; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-d2h --waves-per-block $w > gpurun_out/bw/cfg${c}_w$w.log 2>&1 || exit 1
done; done

# D2H diagnosis (tooling): per-stream copy rates with SDMA and with blit
# kernels, then the config-8 D2H-inclusive sample three times in one process.
set -o pipefail
OUT=gpurun_out/${1:-r2d}
mkdir -p $OUT
timeout -k 10 200 python -u tools/d2h_lab2.py > $OUT/d2h_sdma.log 2>&1 || { tail $OUT/d2h_sdma.log; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 200 python -u tools/d2h_lab2.py > $OUT/d2h_blit.log 2>&1 || { tail $OUT/d2h_blit.log; exit 1; }
cat $OUT/d2h_sdma.log $OUT/d2h_blit.log | grep '^{'
timeout -k 10 300 python -u bench.py --config 8 --steps 1 --warmup 0 --no-cpu-baseline --no-ceiling --d2h-reps 3 > $OUT/bench_cfg8_d2h.log 2>&1 || { tail $OUT/bench_cfg8_d2h.log; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u bench.py --config 8 --steps 1 --warmup 0 --no-cpu-baseline --no-ceiling --d2h-reps 3 > $OUT/bench_cfg8_d2h_blit.log 2>&1 || { tail $OUT/bench_cfg8_d2h_blit.log; exit 1; }
grep -h '^{' $OUT/bench_cfg8_d2h*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)['d2h_inclusive']; print(d['value'], d.get('all_samples_GiBps'), d['copy_GiBps_min_med_max'])"

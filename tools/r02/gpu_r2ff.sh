# Launcher rehearsal for the DG1 configs at N>1 on one GPU (tooling; not scaling).
set -o pipefail
OUT=gpurun_out/${1:-r2ff}
mkdir -p $OUT
for c in 14 16; do
  timeout -k 10 300 python bench.py --gpus 4 --device-override 0 --config $c --objects 2 --steps 2 --warmup 1 --no-ceiling > $OUT/rehearsal_n4_cfg$c.log 2>&1 || { tail -20 $OUT/rehearsal_n4_cfg$c.log; exit 1; }
  grep -h '^{' $OUT/rehearsal_n4_cfg$c.log | python -c "
import sys, json
d = json.loads(sys.stdin.read())
print(d['config']['workload'][:50], '| n_gpus', d['n_gpus'], '| objects/rank', d['config']['objects_per_rank'], '| ok', d['verified_vs_oracle'], '| d2h agg', d['d2h_inclusive'] and d['d2h_inclusive']['aggregate_all_ranks'])"
done

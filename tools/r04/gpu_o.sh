#!/bin/bash
# Round 4, session o: more bench lines at digest a681e2bdce23fef5 on another
# box: config 2 (the driver's command) twice, configs 6 and 16 (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r04o}
mkdir -p $OUT
for k in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_cfg2_$k.log 2>&1 || { tail $OUT/bench_cfg2_$k.log; exit 1; }
done
for c in 6 16; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $OUT/bench_cfg$c.log 2>&1 || { tail $OUT/bench_cfg$c.log; exit 1; }
done
grep -h '^{' $OUT/bench_cfg*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); r = d['roofline']
    print(d['config']['workload'][:40], d['value'], r['achieved'], r['frac'], r.get('traffic'), r.get('library_digest'), d['verified_vs_oracle'])"

# Round-4 final tree: N=8 / N=4 launcher rehearsals on one GPU (every rank on
# device 0; a launcher test, not a scaling measurement) (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r4rehearsal}
mkdir -p $OUT
timeout -k 10 300 python bench.py --gpus 8 --device-override 0 --objects 64 --config 2 --steps 3 --warmup 1 --no-ceiling > $OUT/rehearsal_n8_cfg2.log 2>&1 || { tail -30 $OUT/rehearsal_n8_cfg2.log; exit 1; }
echo n8 done
timeout -k 10 300 python bench.py --gpus 4 --device-override 0 --objects 400 --config 5 --steps 2 --warmup 1 --d2h-full --no-ceiling > $OUT/rehearsal_n4_cfg5_d2h_full.log 2>&1 || { tail -30 $OUT/rehearsal_n4_cfg5_d2h_full.log; exit 1; }
echo n4 done
grep -h '^{' $OUT/*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); x = d['d2h_inclusive'] or {}
    print(d['n_gpus'], d['config']['workload'][:40], d['config']['objects_per_rank'], d['value'], d['verified_vs_oracle'], x.get('whole_job_GiBps'), x.get('verified_vs_oracle'), d['roofline'].get('library_digest'))"

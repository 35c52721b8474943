# Round-3 final tree: host-buffer drop-in configs 18-22 (defaults), config 5
# as BASELINE states it (--d2h-full, N=1), and launcher rehearsals at N=8 /
# N=4 on one GPU (configs 2, 3, 5 with --d2h-full).  Tooling; GPU box.
set -o pipefail
OUT=gpurun_out/${1:-r3ii}
mkdir -p $OUT
show() { python3 -c "import sys,json; d=json.loads(open('$1').read().strip().splitlines()[-1]); c=d['cpu_baseline']; print('$2', d['value'], d['roofline'].get('avg_call_ms'), d['verified_vs_oracle'], c and c['value'], c and c['cores'])"; }
for c in 18 19 20 21 22; do
  L=$OUT/host_cfg${c}_pageable_direct.log
  timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 8 > $L 2>&1 || { tail $L; exit 1; }
  grep -h '^{' $L > $L.json; show $L.json "$c pageable direct devs=all"
done
L=$OUT/cfg5_d2h_full_n1.log
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --d2h-full --no-cpu-baseline --no-ceiling > $L 2>&1 || { tail $L; exit 1; }
grep -h '^{' $L | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); x=d['d2h_inclusive']; print('cfg5 N=1 full', d['value'], x['value'], x['whole_job_GiBps'], x['seconds'], x['bytes'], x['verified_vs_oracle'], x['copy_GiBps_min_med_max'])"
for spec in "8 2 64" "4 3 64"; do
  set -- $spec
  L=$OUT/rehearsal_n$1_cfg$2.log
  timeout -k 10 300 python bench.py --gpus $1 --device-override 0 --config $2 --objects $3 --steps 3 --warmup 1 --no-ceiling > $L 2>&1 || { tail -20 $L; exit 1; }
  grep -h '^{' $L | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('rehearsal', d['n_gpus'], d['config']['workload'][:30], d['value'], d['verified_vs_oracle'])"
done
L=$OUT/cfg5_d2h_full_rehearsal_n8.log
timeout -k 10 300 python bench.py --gpus 8 --device-override 0 --config 5 --objects 800 --steps 3 --warmup 1 --d2h-full --no-ceiling > $L 2>&1 || { tail -20 $L; exit 1; }
grep -h '^{' $L | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); x=d['d2h_inclusive']; print('cfg5 N=8 rehearsal full', d['n_gpus'], d['value'], x['value'], x['whole_job_GiBps'], x['aggregate_all_ranks'], x['verified_vs_oracle'])"

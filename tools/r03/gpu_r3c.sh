# Round 3: the host-buffer drop-in configs 18-22 with
# the D2H-mode, buffer-kind and slot A/Bs.  Tooling; GPU box.
set -o pipefail
OUT=gpurun_out/${1:-r3c}
mkdir -p $OUT
show() { python3 -c "import sys,json; d=json.loads(open('$1').read().strip().splitlines()[-1]); c=d['cpu_baseline']; print('$2', d['value'], d['roofline']['avg_call_ms'], d['verified_vs_oracle'], c and c['value'], c and c['cores'])"; }
for c in 18 19 20 21 22; do
  L=$OUT/host_cfg${c}_pageable_direct.log
  timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 8 > $L 2>&1 || { tail $L; exit 1; }
  grep -h '^{' $L > $L.json; show $L.json "$c pageable direct devs=all"
done
for mem in pinned pageable; do for mode in direct staged; do for devs in 0 0,0; do
  [ "$mem$mode$devs" = "pageabledirect0" ] && continue
  for c in 18 19 20 21 22; do
    L=$OUT/host_cfg${c}_${mem}_${mode}_d${devs}.log
    S3DLIO_GPU_DEVICES=$devs S3DLIO_HOST_D2H=$mode timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --host-mem $mem > $L 2>&1 || { tail $L; exit 1; }
    grep -h '^{' $L > $L.json; show $L.json "$c $mem $mode devs=$devs"
  done
done; done; done
# config 5 as BASELINE states it: the whole object range through the pinned ring
L=$OUT/cfg5_d2h_full_n1.log
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --d2h-full --no-cpu-baseline --no-ceiling > $L 2>&1 || { tail $L; exit 1; }
grep -h '^{' $L | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); x=d['d2h_inclusive']; print('cfg5 N=1 full', d['value'], x['value'], x['whole_job_GiBps'], x['seconds'], x['bytes'], x['verified_vs_oracle'], x['copy_GiBps_min_med_max'])"
L=$OUT/cfg5_d2h_full_rehearsal_n8.log
timeout -k 10 300 python bench.py --gpus 8 --device-override 0 --config 5 --objects 800 --steps 3 --warmup 1 --d2h-full --no-ceiling > $L 2>&1 || { tail -20 $L; exit 1; }
grep -h '^{' $L | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); x=d['d2h_inclusive']; print('cfg5 N=8 rehearsal full', d['n_gpus'], d['value'], x['value'], x['whole_job_GiBps'], x['aggregate_all_ranks'], x['verified_vs_oracle'])"

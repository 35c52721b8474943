# Round 3: zero-prefix store order / policy variants (config-3 mechanism), the
# host-buffer drop-in configs 18-22 with the D2H-mode
# and buffer-kind A/Bs, and the host-slot GPU tests.  Tooling; GPU box.
set -o pipefail
OUT=gpurun_out/${1:-r3b}
mkdir -p $OUT
V="base=;zconst=-DS3DG_DIAG_ZERO=1;zrev=-DS3DG_DIAG_ZERO=4;zpnt=-DS3DG_DIAG_ZPOL=1;zpplain=-DS3DG_DIAG_ZPOL=0;zpntsc1=-DS3DG_DIAG_ZPOL=3"
P="stream2:0:-1:-1:-1;stream3:0:-1:-1:-1;sd1x3x4:0:-1:-1:-1"
LAB_VARIANTS="$V" LAB_POINTS="$P" LAB_REPS=8 LAB_N=10000 \
  timeout -k 10 300 python -u tools/variant_lab.py > $OUT/zero_order_policy_ab.log 2>&1 || { tail -20 $OUT/zero_order_policy_ab.log; exit 1; }
grep '^{' $OUT/zero_order_policy_ab.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -k "host_slots" -x -v --timeout 300 --timeout-method thread > $OUT/host_tests.log 2>&1 || { tail -30 $OUT/host_tests.log; exit 1; }
tail -1 $OUT/host_tests.log
# host drop-ins: default (pageable, direct, every visible GPU) with the CPU baseline
for c in 18 19 20 21 22; do
  timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 8 > $OUT/host_cfg${c}_pageable_direct.log 2>&1 || { tail $OUT/host_cfg${c}_pageable_direct.log; exit 1; }
  grep -h '^{' $OUT/host_cfg${c}_pageable_direct.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($c, 'pageable direct', d['value'], d['roofline']['avg_call_ms'], d['verified_vs_oracle'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
done
# A/Bs without the CPU baseline
for mem in pinned pageable; do for mode in direct staged; do for devs in 0 0,0; do
  [ "$mem$mode$devs" = "pageabledirect0" ] && continue
  for c in 18 19 20 21 22; do
    S3DLIO_GPU_DEVICES=$devs S3DLIO_HOST_D2H=$mode timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --host-mem $mem > $OUT/host_cfg${c}_${mem}_${mode}_d${devs}.log 2>&1 || { tail $OUT/host_cfg${c}_${mem}_${mode}_d${devs}.log; exit 1; }
    grep -h '^{' $OUT/host_cfg${c}_${mem}_${mode}_d${devs}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($c, '$mem $mode devs=$devs', d['value'], d['roofline']['avg_call_ms'], d['verified_vs_oracle'])"
  done
done; done; done

# Round-2 check (tooling): the binding ABI program, every bench config once
# (short), the paced store-only ceilings, and EA write-stall counters on the
# fill vs its ablated form.
# usage: bash tools/r02/gpu_r2c.sh <out-subdir>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2c}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_capi_binding.py tests/test_gpu_batch.py -x -v --timeout 240 --timeout-method thread > $OUT/gpu_binding.log 2>&1 || { tail -40 $OUT/gpu_binding.log; exit 1; }
tail -1 $OUT/gpu_binding.log
for c in 2 3 4 5 6 7 8 9 10 11 12 13 14 15; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 3 > $OUT/bench_cfg$c.log 2>&1 || { tail -20 $OUT/bench_cfg$c.log; exit 1; }
  echo "cfg$c $(grep -c '^{' $OUT/bench_cfg$c.log)"
done
LAB_KINDS=cfg2,ceil_fill,ceil_fill_p1,ceil_fill_p2,ceil_fill_p3,ceil_fill_p4,ceil_fill_p6,ceil_fill_p8,ceil_fill_p12,ceil_fill_p16,ceil_tiled timeout -k 10 300 python -u tools/lab_r2.py > $OUT/lab.log 2>&1 || { tail -20 $OUT/lab.log; exit 1; }
grep '^{' $OUT/lab.log
LAB_REPS=1 LAB_KINDS=cfg2,ceil_fill,ceil_fill_p4 timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE \
    -d $OUT/pmc_wr2 -o p --output-format csv -- python3 tools/lab_r2.py > $OUT/pmc_wr2.log 2>&1 || { tail $OUT/pmc_wr2.log; exit 1; }
echo done

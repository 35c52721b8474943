# EA write counters of bench configs 2 and 3 on the default tiled path
# (tooling; run on the GPU box).  usage: bash tools/pmc_cfg23.sh <out-subdir>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc23}
mkdir -p $OUT
for c in 2 3; do
  for p in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
    tag=$(echo $p | cut -d' ' -f1)
    timeout -s KILL 150 rocprofv3 --pmc $p -d $OUT/cfg${c}_$tag -o p --output-format csv -- \
        python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-d2h --no-verify --no-ceiling \
        > $OUT/cfg${c}_$tag.log 2>&1 || { tail $OUT/cfg${c}_$tag.log; exit 1; }
    echo "cfg$c $tag done"
  done
done
# knob probes for config 3 vs 2 (HIP-event rates)
for a in "--store ntsc1" "--store plain" "--waves-per-block 2" "--prefetch 0" "--prefetch 128"; do
  for c in 2 3; do
    timeout -k 10 200 python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-d2h --no-verify \
        --no-ceiling $a > $OUT/probe.log 2>&1 || { tail $OUT/probe.log; exit 1; }
    grep -h '^{' $OUT/probe.log | python3 -c "import sys,json; [print('cfg$c $a', j['roofline']['achieved']) for j in map(json.loads, sys.stdin)]"
  done
done

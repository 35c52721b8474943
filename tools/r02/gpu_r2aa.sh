# DG1 per-object vs one-launch: effective clock per dispatch (GRBM_GUI_ACTIVE
# over the dispatch time) and SQ issue counters (tooling).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2aa}
mkdir -p $OUT
for c in 14 16; do
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $OUT/pmc_clk_cfg$c -o p --output-format csv -- \
      python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-d2h --no-ceiling --no-verify > $OUT/pmc_clk_cfg$c.log 2>&1 || { tail $OUT/pmc_clk_cfg$c.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $OUT/pmc_sq_cfg$c -o p --output-format csv -- \
      python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-d2h --no-ceiling --no-verify > $OUT/pmc_sq_cfg$c.log 2>&1 || { tail $OUT/pmc_sq_cfg$c.log; exit 1; }
  echo "cfg$c done"
done

# Round-3 final tree: the seeded fuzz soak x15 (390 cases: stream, batch,
# tiled stream, random layout, K2, DG1 with random launch knobs, now also the
# per-launch occupancy / store-floor rule and forced floors).  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3aa}
mkdir -p $OUT
S3DG_FUZZ_SOAK=15 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/fuzz_soak_x15.log 2>&1 || { tail -30 $OUT/fuzz_soak_x15.log; exit 1; }
tail -1 $OUT/fuzz_soak_x15.log

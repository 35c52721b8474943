# Round-3 final-tree evidence, part 1: GPU tests + smoke, then rocprof kernel
# traces and WRITE/FETCH_SIZE passes for the BASELINE configs 2-5 (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r3u}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
bash tools/profile_round.sh ${1:-r3u} 2 3 4 5

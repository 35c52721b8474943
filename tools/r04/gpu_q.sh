#!/bin/bash
# Round 4, session q: the whole GPU suite and smoke at the final tree, as the
# driver runs them at round end (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r04q}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
echo smoke ok

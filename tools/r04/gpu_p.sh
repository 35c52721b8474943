#!/bin/bash
# Round 4, session p: 60 seeded persistent-keystream shape draws (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r04p}
mkdir -p $OUT
S3DG_PERSIST_FUZZ=60 timeout -k 10 800 python -u -m pytest tests/test_gpu_ks_persistent.py -m gpu -k fuzz -q --timeout 300 --timeout-method thread > $OUT/persist_fuzz_x60.log 2>&1 || { tail -30 $OUT/persist_fuzz_x60.log; exit 1; }
tail -1 $OUT/persist_fuzz_x60.log

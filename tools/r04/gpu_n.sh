#!/bin/bash
# Round 4, session n: the persistent-keystream tests (with the seeded shape
# fuzz) and a x50 fuzz soak at digest a681e2bdce23fef5 (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r04n}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ks_persistent.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/ks_persistent_tests.log 2>&1 || { tail -30 $OUT/ks_persistent_tests.log; exit 1; }
tail -1 $OUT/ks_persistent_tests.log
S3DG_FUZZ_SOAK=50 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 550 --timeout-method thread > $OUT/fuzz_soak_x50.log 2>&1 || { tail -30 $OUT/fuzz_soak_x50.log; exit 1; }
tail -1 $OUT/fuzz_soak_x50.log

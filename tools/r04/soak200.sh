#!/bin/bash
# Round 4: fuzz soak x200 (5200 seeded cases through every kernel and knob)
# at the final library digest (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r04soak}
mkdir -p $OUT
python -c "import sys; sys.path.insert(0,'.'); from s3dlio_amd import build; print('source digest', build.source_digest())" > $OUT/digest.log
S3DG_FUZZ_SOAK=200 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 850 --timeout-method thread > $OUT/fuzz_soak_x200.log 2>&1 || { tail -30 $OUT/fuzz_soak_x200.log; exit 1; }
tail -1 $OUT/fuzz_soak_x200.log

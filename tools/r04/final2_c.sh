#!/bin/bash
# Round 4, second final evidence: bench lines (with the new digest's traffic)
# of configs 2-17 (tooling).
set -o pipefail
CFGS="2 3 4 5 6 8 9 10 14 15 16 17" bash tools/r04/final_bench.sh r4final2_bench || exit 1

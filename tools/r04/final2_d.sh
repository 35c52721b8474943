#!/bin/bash
# Round 4, second final evidence: bench lines of configs 11-13 and 18-28,
# config 5 with the whole D2H, and the N=8 / N=4 launcher rehearsals (tooling).
set -o pipefail
CFGS="11 12 13 18 19 20 21 22 23 24 25 26 27 28 5full" bash tools/r04/final_bench.sh r4final2_bench2 || exit 1
bash tools/r04/rehearsal.sh r4final2_rehearsal || exit 1

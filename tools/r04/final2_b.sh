#!/bin/bash
# Round 4, second final evidence: traces and PMC passes of configs 8 9 10 14
# 15 16 17, then the bench lines of configs 2-10 (tooling).
set -o pipefail
bash tools/profile_round.sh r4final2_prof_b 8 9 10 14 15 16 17 || exit 1
CFGS="2 3 4 5 6 8 9 10" bash tools/r04/final_bench.sh r4final2_bench_a || exit 1

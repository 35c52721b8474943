#!/bin/bash
# Round 4, second final evidence (persistent keystream, digest a681e2bdce23fef5):
# GPU tests + smoke + fuzz soak x15, then traces and PMC passes of configs
# 2 3 4 5 6 (tooling).
set -o pipefail
bash tools/r04/final_tests.sh r4final2_tests || exit 1
bash tools/profile_round.sh r4final2_prof_a 2 3 4 5 6 || exit 1

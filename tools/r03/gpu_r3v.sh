# Round-3 final-tree evidence, part 2: rocprof traces and PMC traffic for the
# other bench configs (tooling).
set -o pipefail
bash tools/profile_round.sh ${1:-r3v} 6 8 9 10 14 15 16 17

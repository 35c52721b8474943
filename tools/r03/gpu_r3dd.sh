# Round-3 final tree: rocprof traces + WRITE/FETCH_SIZE for every traced
# config (tooling).
set -o pipefail
bash tools/profile_round.sh ${1:-r3dd} 2 3 4 5 6 8 9 10 14 15 16 17

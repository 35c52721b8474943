# A/B bench lines for one knob (tooling; GPU box).
# usage: bash tools/bench_ab.sh <out-subdir> "<configs>" "<flag variants, ';'-separated>" [reps]
set -o pipefail
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT
IFS=';' read -ra VARS <<< "$3"
for r in $(seq 1 ${4:-2}); do
  for c in $2; do
    for i in "${!VARS[@]}"; do
      v=${VARS[$i]}
      timeout -k 10 200 python bench.py --config $c $v --no-cpu-baseline --no-d2h --no-verify --steps 5 > $OUT/c${c}_v${i}_r$r.log 2>&1 || exit 1
      grep '^{' $OUT/c${c}_v${i}_r$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('cfg', '$c', 'rep', '$r', '[$v]', r['achieved'], r['kernel'])"
    done
  done
done

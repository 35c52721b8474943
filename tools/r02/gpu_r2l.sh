# k_keystream per-launch cost lab (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2l}
mkdir -p $OUT
KS_REPS=3 timeout -k 10 400 python -u tools/ks_launch_lab.py > $OUT/ks_launch_lab.log 2>&1 || { tail -20 $OUT/ks_launch_lab.log; exit 1; }
grep '^{' $OUT/ks_launch_lab.log

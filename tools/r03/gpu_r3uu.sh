# Round 3: config-2 launch-time distribution against GFX clock and socket
# power (tools/step_power_lab.py), twice.  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3uu}
mkdir -p $OUT
for k in 1 2; do
  LAB_LAUNCHES=600 timeout -k 10 200 python -u tools/step_power_lab.py > $OUT/step_power_$k.log 2>&1 || { tail -20 $OUT/step_power_$k.log; exit 1; }
  grep '^{' $OUT/step_power_$k.log
done

# DG1/K2 launch-size lab (8 GiB launches vs one launch) and the single-call floor (tooling).
set -o pipefail
OUT=gpurun_out/${1:-r2k}
mkdir -p $OUT
LAB_REPS=3 LAB_GIB=80 LAB_KINDS=dg1c1_8g,dg1c1_all,dg1c2_8g,dg1c2_all,k2_8g,k2_all,one1m,memset1m,ceil1m,one16m \
  timeout -k 10 300 python -u tools/lab_r2.py > $OUT/lab_launch_size.log 2>&1 || { tail -20 $OUT/lab_launch_size.log; exit 1; }
grep '^{' $OUT/lab_launch_size.log

#!/bin/bash
# Round 4, session k: persistent keystream launches (per-XCD unit queues with
# stealing) against the same tree's static grid (-DS3DG_DIAG_KS_STATIC=1) and
# the round-4 final sources, interleaved in one process (p6: the default rule,
# 1-wave workgroups from 6 rounds; p1: from one round); then the DG1 wave
# timelines, static and persistent (trace builds).  First pass (any launch of
# more than one round persistent, as ksp/kss): profiles/r04/k/pass1/.
set -o pipefail
OUT=gpurun_out/${1:-r04k}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ks_persistent.py tests/test_gpu_datagen.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
LAB_AB="r04=013b5e5;p6=.;p1=.:-DS3DG_KS_PERSIST_ROUNDS=1;kss=.:-DS3DG_DIAG_KS_STATIC=1" LAB_POINTS="cfg14;cfg15;cfg16;cfg6;k2_8g;k2_8g_2048;dg1_4g;cfg2" LAB_REPS=6 \
    timeout -k 10 600 python -u tools/r04/lib_ab.py > $OUT/lib_ab.log 2>&1 || { tail -20 $OUT/lib_ab.log; exit 1; }
grep -v "rep " $OUT/lib_ab.log
LAB_LIB=libvariant_trace_static.so timeout -k 10 300 python -u tools/r04/ks_rounds_lab.py > $OUT/ks_rounds_static.log 2>&1 || { tail -20 $OUT/ks_rounds_static.log; exit 1; }
LAB_LIB=libvariant_trace.so timeout -k 10 300 python -u tools/r04/ks_rounds_lab.py > $OUT/ks_rounds_persistent.log 2>&1 || { tail -20 $OUT/ks_rounds_persistent.log; exit 1; }
grep -h '^{' $OUT/ks_rounds_static.log $OUT/ks_rounds_persistent.log | cut -c1-300

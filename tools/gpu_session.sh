#!/bin/bash
# One parameterized GPU-box session (replaces the one-shot tools/r0*/gpu_*.sh
# scripts of rounds 2-4).  Run from the repository root:
#
#   gpurun -- 'bash tools/gpu_session.sh <out-dir> <step> [<step> ...]'
#
# Steps, each under its own time limit; the session stops at the first
# failure (no GPU step runs after a fault, abort or time-out):
#   tests[:EXPR]        pytest -m gpu (optionally -k EXPR), log gpu_tests.log
#   file:PATH           pytest -m gpu on one test file
#   smoke               __graft_entry__.smoke()
#   bench:CFG[:ARGS]    bench.py --config CFG --steps 20 --warmup 5 ARGS (':'-separated)
#   envbench:ENV:CFG    the same with ENV (comma-separated K=V) set
#   driver              bench.py --gpus 1 --steps 20 --warmup 5 (the driver's own command; rounds 2-5 ran bench.py with no flags here, 5 steps)
#   prof:CFG            rocprofv3 --kernel-trace --stats of bench.py --config CFG
#   pmc:CFG:COUNTER     one rocprofv3 --pmc pass (WRITE_SIZE or FETCH_SIZE) of bench.py --config CFG
#   pmcx:SCRIPT:CTRS    one rocprofv3 --pmc pass of per-XCC counters (tools/xcc_counters.yaml) over tools/SCRIPT
#   rehearsal           bench.py N=8 (config 2) / N=4 (config 5, --d2h-full) launcher rehearsals on device 0
#   soak[:N]            tests/test_gpu_fuzz.py with S3DG_FUZZ_SOAK=N (default 15)
#   lab:SCRIPT[:ENV]    python tools/SCRIPT with ENV (comma-separated K=V) set
#   exe:PATH            a native program built in this tree (tools/_native/...)
# Environment: STEPS (bench steps, default 20), WARMUP (default 5).
set -o pipefail
OUT=gpurun_out/${1:?out dir}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
n=0
for step in "$@"; do
    n=$((n + 1))
    IFS=':' read -r kind a b c <<< "$step"
    tag=$(printf '%02d_%s' $n "$kind${a:+_$a}" | tr '/ ,=.' '_____')
    echo "== $step ($tag)"
    case "$kind" in
    tests)
        timeout -k 10 1100 $PYT tests ${a:+-k "$a"} > "$OUT/$tag.log" 2>&1; rc=$?
        tail -3 "$OUT/$tag.log";;
    file)
        timeout -k 10 600 $PYT "$a" > "$OUT/$tag.log" 2>&1; rc=$?
        tail -3 "$OUT/$tag.log";;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/$tag.log" 2>&1; rc=$?
        tail -2 "$OUT/$tag.log";;
    bench)
        extra=$(echo "${b}${c:+:$c}" | tr ':' ' ')
        timeout -k 10 400 python -u bench.py --config "$a" --steps "$STEPS" --warmup "$WARMUP" $extra \
            > "$OUT/$tag.log" 2>&1; rc=$?
        grep '^{' "$OUT/$tag.log" | tail -1 | cut -c1-600;;
    envbench)
        envs=$(echo "$a" | tr ',' ' ')
        timeout -k 10 400 env $envs python -u bench.py --config "$b" --steps "$STEPS" --warmup "$WARMUP" \
            > "$OUT/$tag.log" 2>&1; rc=$?
        grep '^{' "$OUT/$tag.log" | tail -1 | cut -c1-600;;
    driver)
        timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/$tag.log" 2>&1; rc=$?
        grep '^{' "$OUT/$tag.log" | tail -1 | cut -c1-600;;
    prof)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o run --output-format csv \
            -- python3 bench.py --config "$a" --steps "$STEPS" --warmup "$WARMUP" --no-ceiling --no-d2h \
            --no-cpu-baseline > "$OUT/$tag.log" 2>&1; rc=$?
        grep '^{' "$OUT/$tag.log" | tail -1 | cut -c1-300;;
    pmc)
        timeout -s KILL 240 rocprofv3 --pmc "$b" -d "$OUT/$tag" -o run --output-format csv \
            -- python3 bench.py --config "$a" --steps 3 --warmup 1 --no-ceiling --no-d2h --no-cpu-baseline \
            --no-verify > "$OUT/$tag.log" 2>&1; rc=$?
        tail -1 "$OUT/$tag.log";;
    pmcx)           # per-XCC counters (tools/xcc_counters.yaml) over a lab script: pmcx:SCRIPT:C1,C2,...[:ENV]
        ctrs=$(echo "$b" | tr ',' ' ')
        envs=$(echo "$c" | tr ',' ' ')
        for e in $envs; do export "$e"; done
        timeout -s KILL 120 rocprofv3 -E tools/xcc_counters.yaml --pmc $ctrs -d "$OUT/$tag" -o run \
            --output-format csv -- python3 "tools/$a" > "$OUT/$tag.log" 2>&1; rc=$?
        for e in $envs; do unset "${e%%=*}"; done
        tail -1 "$OUT/$tag.log";;
    exe)            # a native program built here (e.g. tools/_native/dispatch_lab)
        timeout -k 10 300 "$a" > "$OUT/$tag.log" 2>&1; rc=$?
        tail -12 "$OUT/$tag.log";;
    rehearsal)      # N=8 / N=4 launcher rehearsals, every rank on device 0 (not a scaling measurement)
        timeout -k 10 300 python bench.py --gpus 8 --device-override 0 --objects 64 --config 2 --steps 3 \
            --warmup 1 --no-ceiling > "$OUT/${tag}_n8_cfg2.log" 2>&1 && \
        timeout -k 10 300 python bench.py --gpus 4 --device-override 0 --objects 400 --config 5 --steps 2 \
            --warmup 1 --d2h-full --no-ceiling > "$OUT/${tag}_n4_cfg5_d2h_full.log" 2>&1; rc=$?
        cat "$OUT/${tag}"_n*.log > "$OUT/$tag.log"
        grep -h '^{' "$OUT/${tag}"_n*.log | cut -c1-300;;
    soak)           # fuzz soak: SOAK x 26 seeded cases through every kernel and knob
        S3DG_FUZZ_SOAK=${a:-15} timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q \
            --timeout 850 --timeout-method thread > "$OUT/$tag.log" 2>&1; rc=$?
        tail -1 "$OUT/$tag.log";;
    lab)
        envs=$(echo "$b" | tr ',' ' ')
        timeout -k 10 900 env $envs python -u "tools/$a" > "$OUT/$tag.log" 2>&1; rc=$?
        grep '^{' "$OUT/$tag.log" | cut -c1-400 | tail -40;;
    *)
        echo "unknown step $step"; rc=2;;
    esac
    if [ $rc -ne 0 ]; then
        echo "step $step failed rc=$rc"; tail -30 "$OUT/$tag.log"; exit $rc
    fi
done
echo "session ok"

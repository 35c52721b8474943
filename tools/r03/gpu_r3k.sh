# Round 3: the binding program against the host-ASan/UBSan build of the
# library (tools/asan_build.sh), with one and three host slots.  Tooling.
set -o pipefail
OUT=gpurun_out/${1:-r3k}
mkdir -p $OUT/a $OUT/b
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
timeout -k 10 300 tools/_build/asan/binding_abi_asan $OUT/a > $OUT/asan_one_slot.log 2>&1 || { tail -40 $OUT/asan_one_slot.log; exit 1; }
tail -2 $OUT/asan_one_slot.log
S3DLIO_GPU_DEVICES=0,0,0 timeout -k 10 300 tools/_build/asan/binding_abi_asan $OUT/b > $OUT/asan_three_slots.log 2>&1 || { tail -40 $OUT/asan_three_slots.log; exit 1; }
tail -2 $OUT/asan_three_slots.log
S3DLIO_GPU_DEVICES=0,0,0 timeout -k 10 300 tools/_build/asan/host_stress_asan 8 3 > $OUT/asan_host_stress.log 2>&1 || { tail -40 $OUT/asan_host_stress.log; exit 1; }
tail -2 $OUT/asan_host_stress.log
rm -rf $OUT/a $OUT/b

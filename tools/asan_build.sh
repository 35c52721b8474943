#!/bin/bash
# Host-side AddressSanitizer + UBSan build of the library and of the binding
# program (tests/capi/binding_abi.c), for a run on the GPU box (tooling).
# Only host code is instrumented (-Xarch_host); device code is the product's.
#   bash tools/asan_build.sh            # here, outputs tools/_build/asan/
#   ASAN_OPTIONS=detect_leaks=0 tools/_build/asan/binding_abi_asan <dir>   # GPU box
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/_build/asan
mkdir -p $OUT
SRCS=$(python3 -c "import sys; sys.path.insert(0, '$ROOT/s3dlio_amd'); import build; print(' '.join(build.SOURCES))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -fvisibility=hidden \
    -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer \
    -mllvm -amdgpu-kernarg-preload-count=16 -I $ROOT/include -I $ROOT/s3dlio_amd/csrc -DS3DG_BUILD \
    -o $OUT/libs3dlio_amd.so $SRCS
python3 -c "import sys; sys.path.insert(0, '$ROOT'); from oracle import oracle_c; oracle_c.build()"
/opt/rocm/lib/llvm/bin/clang -O1 -g -std=c99 -fsanitize=address,undefined -fno-omit-frame-pointer \
    -I $ROOT/include $ROOT/tests/capi/binding_abi.c -L $OUT -ls3dlio_amd $ROOT/oracle/_build/libs3dg_oracle.so \
    -Wl,-rpath,$OUT -Wl,-rpath,$ROOT/oracle/_build -o $OUT/binding_abi_asan
echo "$OUT/binding_abi_asan"
/opt/rocm/lib/llvm/bin/clang -O1 -g -std=c99 -pthread -fsanitize=address,undefined -fno-omit-frame-pointer \
    -I $ROOT/include $ROOT/tests/capi/host_stress.c -L $OUT -ls3dlio_amd $ROOT/oracle/_build/libs3dg_oracle.so \
    -Wl,-rpath,$OUT -Wl,-rpath,$ROOT/oracle/_build -o $OUT/host_stress_asan
echo "$OUT/host_stress_asan"

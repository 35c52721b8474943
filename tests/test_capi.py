"""CPU: the C-ABI library loads, exports every symbol include/s3dlio_gpu.h
declares, and its pure-host helpers agree with the oracle.  No kernel is
launched here (no GPU in this container)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT
from oracle import oracle_py as P

HEADER = os.path.join(ROOT, "include", "s3dlio_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(s3d[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["s3dlio_fill_controlled_data", "s3dlio_fill_controlled_data_seeded",
                 "s3dg_fill_controlled", "s3dg_fill_controlled_stream",
                 "s3dg_fill_controlled_batch", "s3dg_ctx_create", "s3dg_last_error"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    import s3dlio_amd  # noqa: F401  (builds nothing; loads the in-tree .so)
    from s3dlio_amd._lib import LIB_PATH, SIGNATURES
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB_PATH], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    declared = set(declared_functions())
    assert declared <= exported, declared - exported
    # nothing beyond the ABI leaks (internal C++ is hidden)
    assert {e for e in exported if not e.startswith(("s3dg_", "s3dlio_"))} == set()
    assert declared == set(SIGNATURES)


def test_host_helpers_match_oracle():
    from s3dlio_amd import compress_ratio, object_entropy, unique_blocks
    for nb in [1, 2, 3, 5, 16, 2048, 2049, 10**6 + 1]:
        for d in [0, 1, 2, 3, 4, 7, 100, 5000]:
            assert unique_blocks(nb, d) == P.unique_blocks(nb, d)
    for c in [0, 1, 2, 3, 4, 5, 128, 5000]:
        assert compress_ratio(c) == P.compress_ratio(c)
    assert compress_ratio(1.5) == (1, 3) == compress_ratio((3, 2))
    assert compress_ratio(2.0) == (1, 2)
    for j in [0, 1, 999, 2**31]:
        assert object_entropy(0x5EED000000000001, j) == P.object_entropy(0x5EED000000000001, j)


def test_zero_class_rule():
    """The batch kernel's per-launch class: 1 = zero prefix
    ending on a 64-B line (occupancy cap), 2 = >= half a block ending inside a
    line (wall-clock store floor), 0 = neither.  Pure host math."""
    from s3dlio_amd._lib import lib
    from s3dlio_amd import compress_ratio
    cls = lambda c: lib.s3dg_zero_class(*compress_ratio(c))
    assert [cls(c) for c in (1, 2, 4, 8, 16, 32, 64)] == [0, 1, 1, 1, 1, 1, 1]
    assert [cls(c) for c in (3, 5, 6, 7, 9, 100)] == [2, 2, 2, 2, 2, 2]
    assert cls((3, 2)) == 0 and cls((5, 3)) == 0 and cls((4, 3)) == 1 and cls((8, 3)) == 1 and cls((7, 3)) == 2
    assert lib.s3dg_zero_class(0, 1) == 0 and lib.s3dg_zero_class(1, 0) == 0
    for fn, fd in [(1, 2), (3, 4), (2, 3), (1, 3), (2, 5), (1, 4), (4, 5), (63, 64), (127, 128)]:
        prefix = 4096 * fn / fd
        want = 1 if prefix % 64 == 0 else (2 if prefix >= 2048 else 0)
        assert lib.s3dg_zero_class(fn, fd) == want, (fn, fd)


def test_no_gpu_is_an_error_not_a_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import s3dlio_amd as S
    with pytest.raises((RuntimeError, ValueError)):
        S.Context(0)
    with pytest.raises((RuntimeError, ValueError)):
        S.fill_controlled_data(bytearray(4096), 1, 1)


def test_registration_handle_without_gpu():
    """register_host_buffer (s3dg_host_register behind a handle that holds the
    buffer while registered): without a GPU the call raises and
    the handle lets go of the buffer (it can be resized again); an empty buffer
    needs no call; read-only buffers are refused before any call."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import s3dlio_amd as S
    b = bytearray(8192)
    with pytest.raises(RuntimeError, match="hipHostRegister"):
        S.register_host_buffer(b)
    b.extend(b"x")                       # no export left behind
    with S.register_host_buffer(bytearray(0)) as h:
        assert h.nbytes == 0
    with pytest.raises(ValueError, match="writable"):
        S.register_host_buffer(b"\x00" * 16)
    assert S.unregister_host_buffer() == 0


def test_buffer_argument_errors():
    import s3dlio_amd as S
    with pytest.raises(ValueError, match="writable"):
        S.fill_controlled_data(b"\x00" * 16, 1, 1)
    import numpy as np
    a = np.zeros((8, 8), np.uint8)[:, ::2]
    with pytest.raises(ValueError, match="contiguous"):
        S.fill_controlled_data(a, 1, 1)
    S.fill_controlled_data(bytearray(0), 1, 1)   # empty: no-op, no GPU needed


def test_version_string():
    from s3dlio_amd._lib import lib
    assert b"gfx950" in lib.s3dg_version()
    assert isinstance(ctypes.c_char_p(lib.s3dg_last_error()).value, (bytes, type(None)))


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 255, 4096, 8192, 262144 - 4096, 10**6])
def test_host_jump_matches_stepping(n):
    """Jump-ahead polynomial (s3dg_jump.cpp) == n sequential Xoshiro steps."""
    from s3dlio_amd import xoshiro_jump
    st = list(P.Xoshiro256pp.seed_from_u64(12345).s)
    r = P.Xoshiro256pp(st)
    if n <= 300000:
        for _ in range(n):
            r.next_u64()
        assert xoshiro_jump(st, n) == r.s
    else:   # composition: jump(n) == jump(n-a) after jump(a)
        assert xoshiro_jump(xoshiro_jump(st, 4096), n - 4096) == xoshiro_jump(st, n)


def test_optimal_chunk_size_table():
    """tests/test_optimal_chunking.rs:8-19."""
    from s3dlio_amd import optimal_chunk_size
    M = 1024 * 1024
    for n, exp in [(10 * M, 10 * M), (16 * M, 16 * M), (20 * M, 16 * M), (32 * M, 32 * M),
                   (50 * M, 32 * M), (64 * M, 64 * M), (100 * M, 64 * M), (1024 * M, 64 * M)]:
        assert optimal_chunk_size(n) == exp


def test_thread_count_utilities():
    import os
    import s3dlio_amd as S
    assert S.py_total_cpus() == os.cpu_count()
    assert 1 <= S.py_default_data_gen_threads() <= S.py_total_cpus()


def test_dg1_oracles_agree():
    from oracle import oracle_c as C
    for (n, d, fn, fd, s) in [(3 * 2**20 + 5, 1, 0, 1, 7), (2**20 * 5 + 9, 2, 1, 2, 99),
                              (100, 3, 2, 3, 5), (2**20, 1, 0, 1, 2**64 - 1), (7, 0, 1, 3, 1)]:
        assert bytes(C.dgen_fill(n, d, fn, fd, s)) == P.dgen_fill(n, d, fn, fd, s)


def test_generator_config_validation_cpu():
    """Host-side checks happen before any GPU work (block size is fixed by DG1)."""
    import s3dlio_amd as S
    c = S.GeneratorConfig(1000)
    assert (c.dedup_factor, c.compress_factor, c.numa_mode, c.seed) == (1, 1, S.NumaMode.AUTO, None)
    with pytest.raises(ValueError, match="block_size"):
        S.generate_data_from_config(S.GeneratorConfig(10, block_size=4096))


def test_header_is_plain_c_and_links(tmp_path):
    """include/s3dlio_gpu.h is a C header (C99 and C++11 clean), and a C
    program links against the library: host math answers, and with no GPU
    creating a context is an error with a message, not a fallback."""
    import shutil
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not available")
    subprocess.check_call([gcc, "-fsyntax-only", "-x", "c", "-std=c99", "-Wall", "-Wextra", "-pedantic",
                           "-Werror", HEADER])
    subprocess.check_call(["g++", "-fsyntax-only", "-x", "c++", "-std=c++11", "-Wall", "-Werror", HEADER])
    from s3dlio_amd._lib import LIB_PATH
    src = tmp_path / "t.c"
    src.write_text(r'''
#include <stdio.h>
#include "s3dlio_gpu.h"
int main(void) {
    uint32_t fn = 0, fd = 0;
    if (s3dg_unique_blocks(2048, 4) != 512) return 1;
    if (s3dg_compress_ratio(3, &fn, &fd) != 0 || fn != 2 || fd != 3) return 2;
    if (s3dg_object_entropy(1, 2) != 1 + (2ull << 32)) return 3;
    s3dg_ctx *c = 0;
    int r = s3dg_ctx_create(0, &c);
    printf("%d|%s\n", r, r ? s3dg_last_error() : "ok");
    if (r == 0) s3dg_ctx_destroy(c);
    return 0;
}
''')
    exe = tmp_path / "t"
    libdir = os.path.dirname(LIB_PATH)
    subprocess.check_call([gcc, "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HEADER), str(src),
                           "-L", libdir, "-ls3dlio_amd", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out
    code, msg = out.stdout.strip().split("|", 1)
    import torch
    if not torch.cuda.is_available():
        assert int(code) < 0 and msg

"""Build the C-ABI shared library libs3dlio_amd.so in-tree (gfx950 only).

    python s3dlio_amd/build.py          # or __graft_entry__.build()

(run it by path: `python -m` would import the package, i.e. load the old .so)

Plain hipcc, no CMake: two translation units (kernels + C ABI) linked into
one .so that exports exactly the symbols of include/s3dlio_gpu.h.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libs3dlio_amd.so")
SOURCES = [os.path.join(CSRC, "s3dg_kernels.hip"), os.path.join(CSRC, "s3dg_capi.cpp"),
           os.path.join(CSRC, "s3dg_jump.cpp"), os.path.join(CSRC, "s3dg_generator.cpp"),
           os.path.join(CSRC, "s3dg_crc.hip"), os.path.join(CSRC, "s3dg_npz.cpp"),
           os.path.join(CSRC, "s3dg_object.cpp"), os.path.join(CSRC, "s3dg_put.cpp"),
           os.path.join(CSRC, "s3dg_numa.cpp"), os.path.join(CSRC, "s3dg_host.cpp"),
           os.path.join(CSRC, "s3dg_batch.hip")]
HEADERS = [os.path.join(CSRC, "s3dg_internal.h"), os.path.join(CSRC, "s3dg_jump.h"),
           os.path.join(ROOT, "include", "s3dlio_gpu.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


DIGEST_MARK = b"S3DG_BUILD_DIGEST="


def source_digest() -> str:
    """Digest of the library sources (every csrc .hip/.cpp/.h/.c, the public
    header and this build script).  It is compiled into the library
    (s3dg_build_digest()), so a measurement can prove which sources the timed
    binary was built from, and staleness is decided by content, not mtime."""
    import hashlib
    h = hashlib.sha256()
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".cpp", ".h", ".c")):
            with open(os.path.join(CSRC, name), "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    for extra in ("include/s3dlio_gpu.h", "s3dlio_amd/build.py"):
        with open(os.path.join(ROOT, extra), "rb") as f:
            h.update(extra.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def embedded_digest(path: str = LIB) -> str | None:
    """The source digest compiled into a built library (read from the file,
    without loading it), or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    k = data.find(DIGEST_MARK)
    if k < 0:
        return None
    return data[k + len(DIGEST_MARK):k + len(DIGEST_MARK) + 16].decode("ascii", "replace")


def _stale() -> bool:
    return embedded_digest(LIB) != source_digest()


BV_SRC = os.path.join(CSRC, "bytesview.c")


def _bytesview_path() -> str:
    import sysconfig
    return os.path.join(PKG, "_bytesview" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_bytesview(force: bool = False, verbose: bool = False) -> str:
    """The BytesView CPython extension type (gcc against this interpreter's headers)."""
    import sysconfig
    out = _bytesview_path()
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(BV_SRC):
        return out
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-shared", "-fPIC", "-Wall", "-Werror",
           "-I", sysconfig.get_paths()["include"], "-o", out, BV_SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return out


NL_SRC = os.path.join(ROOT, "tools", "native_loop.c")
NL_LIB = os.path.join(ROOT, "tools", "_native", "libnative_loop.so")   # travels to the GPU box (tools/_build does not)


def build_native_loop(force: bool = False, verbose: bool = False) -> str:
    """bench.py's native call loop (tools/native_loop.c; not part of the library)."""
    if not os.path.exists(NL_SRC):
        return ""
    if not force and os.path.exists(NL_LIB) and os.path.getmtime(NL_LIB) >= os.path.getmtime(NL_SRC):
        return NL_LIB
    os.makedirs(os.path.dirname(NL_LIB), exist_ok=True)
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-shared", "-fPIC", "-Wall", "-Werror", "-o", NL_LIB, NL_SRC, "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return NL_LIB


def build(force: bool = False, verbose: bool = False) -> str:
    build_bytesview(force, verbose)
    build_native_loop(force, verbose)
    if not force and not _stale():
        return LIB
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
             # kernel arguments preloaded into SGPRs (gfx950): the first scalar
             # load of every 4 KiB-block workgroup disappears from its critical path
             "-mllvm", "-amdgpu-kernarg-preload-count=16",
             "-I", os.path.join(ROOT, "include"), "-I", CSRC,
             "-DS3DG_BUILD", f"-DS3DG_BUILD_DIGEST=\"{source_digest()}\""]
    # one translation unit per process (no device code crosses units), then link
    import concurrent.futures as cf
    import tempfile
    with tempfile.TemporaryDirectory(prefix="s3dg_obj_") as tmp:
        objs = [os.path.join(tmp, os.path.basename(src) + ".o") for src in SOURCES]

        def compile_one(k):
            cmd = [HIPCC, *flags, "-c", "-o", objs[k], SOURCES[k]]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.check_call(cmd)
        workers = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "0")) or os.cpu_count() or 1))
        with cf.ThreadPoolExecutor(workers) as pool:
            list(pool.map(compile_one, range(len(SOURCES))))
        tmp_lib = LIB + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp_lib] + objs
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(tmp_lib, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))

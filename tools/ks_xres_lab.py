"""Keystream lanes on their XCD's own 4 KiB granules (round 6 lab).  The
keystream is bound by its store pattern at the memory side:
every wave writes 512-B pieces of 64 lane regions.  The fill writes each XCD's
own granules (g = x mod 8).  This lab builds a copy of the library (sources
copied and patched under tools/_lab/src_xres, the product tree untouched)
whose K2 lanes are 512 draws = one 4 KiB granule each, a wave on XCD x taking
the 64 granules = x (mod 8) of one 2 MiB chunk (S3DG_KS_XRES=1), against the
product (4096-draw lanes, XCD groups of 16 waves) and the copy's 512-draw
lanes in the product's order.  Every lane still jumps to its own draw, so
the bytes equal the product's (checked: the buffer's digest after each).
    python tools/ks_xres_lab.py --build     # here: tools/_labso/libks_xres.so
    python tools/ks_xres_lab.py             # GPU box
Tooling only: nothing in the product imports this."""
import ctypes
import json
import os
import re
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "tools", "_lab", "src_xres")
SO = os.path.join(ROOT, "tools", "_labso", "libks_xres.so")
MiB = 1 << 20


def patch(path, old, new):
    s = open(path).read()
    assert old in s, (path, old[:60])
    open(path, "w").write(s.replace(old, new, 1))


def build():
    shutil.rmtree(SRC, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "s3dlio_amd", "csrc"), os.path.join(SRC, "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(SRC, "include"))
    c = os.path.join(SRC, "csrc")
    patch(os.path.join(c, "s3dg_internal.h"), "    uint32_t par;\n", "    uint32_t par;\n    uint32_t xres;          // lab: lanes on their XCD's granules\n")
    patch(os.path.join(c, "s3dg_kernels.hip"), "    const uint64_t gl = (bid * W + w) * 64 + l;",
          "    const uint64_t wi_ = bid * W + w;\n"
          "    const uint64_t gl = A.xres ? (((wi_ >> 3) << lsh) + (wi_ & 7) + 8 * (uint64_t)l) : wi_ * 64 + l;")
    patch(os.path.join(c, "s3dg_kernels.hip"), "        X.xg = xg;", "        X.xg = X.xres ? 1 : xg;")
    patch(os.path.join(c, "s3dg_capi.cpp"), "    A.lpc = lpc;\n    A.span = (uint32_t)span;\n    A.z0 = z0;",
          "    A.lpc = lpc;\n    A.span = (uint32_t)span;\n    A.z0 = z0;\n"
          "    A.xres = getenv(\"S3DG_KS_XRES\") && mode == 0 && lpc == 512 && z0 == 0 ? 1u : 0u;")
    sys.path.insert(0, os.path.join(ROOT, "s3dlio_amd"))
    import build as B
    srcs = [os.path.join(c, os.path.basename(p)) for p in B.SOURCES]
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-fvisibility=hidden", "-DS3DG_BUILD", "-mllvm", "-amdgpu-kernarg-preload-count=16",
                           "-I", os.path.join(SRC, "include"), "-I", c, "-o", SO] + srcs)
    print(SO)


def main():
    if "--build" in sys.argv:
        return build()
    import torch
    libs = {"product": ctypes.CDLL(os.path.join(ROOT, "s3dlio_amd", "libs3dlio_amd.so"), mode=os.RTLD_LOCAL),
            "lab": ctypes.CDLL(SO, mode=os.RTLD_LOCAL)}
    u64 = ctypes.c_uint64
    ctx = {}
    for k, L in libs.items():
        h = ctypes.c_void_p()
        assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
        ctx[k] = h
    # the lab context: 512-draw lanes (min_lane_draws 512)
    assert libs["lab"].s3dg_set_keystream_shape(ctx["lab"], 0, 0, 0, 0, u64(512), -1) == 0
    n, size = 10000, 8 * MiB
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    p = ctypes.c_void_p(buf.data_ptr())

    def k2(k):
        assert libs[k].s3dg_xoshiro_fill(ctx[k], p, u64(n * size), u64(2 * MiB), u64(0), sh) == 0

    def digest():
        w = buf.view(torch.int64)
        return int((w[::4097].sum() ^ w[1::65537].sum()).item())
    cases = [("product", None), ("lab512", "0"), ("lab_xres", "1")]
    with torch.cuda.stream(st):
        ref = None
        for name, xres in cases:   # bytes first
            if xres is None:
                os.environ.pop("S3DG_KS_XRES", None)
            elif xres == "1":
                os.environ["S3DG_KS_XRES"] = "1"
            else:
                os.environ.pop("S3DG_KS_XRES", None)
            buf.fill_(0xAB)
            k2("product" if xres is None else "lab")
            st.synchronize()
            d = digest()
            ref = d if ref is None else ref
            print(json.dumps({"case": name, "digest_equal_product": d == ref}), flush=True)
        reps = int(os.environ.get("LAB_REPS", "10"))
        acc = {}
        for rnd in range(int(os.environ.get("LAB_ROUNDS", "4"))):
            for name, xres in cases:
                if xres == "1":
                    os.environ["S3DG_KS_XRES"] = "1"
                else:
                    os.environ.pop("S3DG_KS_XRES", None)
                lib = "product" if xres is None else "lab"
                k2(lib)
                st.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    k2(lib)
                e1.record(st)
                e1.synchronize()
                gbs = n * size / (e0.elapsed_time(e1) / reps * 1e6)
                print(json.dumps({"round": rnd, "case": name, "GBps": round(gbs, 1)}), flush=True)
                if rnd:
                    acc.setdefault(name, []).append(gbs)
    os.environ.pop("S3DG_KS_XRES", None)
    # DG1 per-object launches (config 14's shape): lane length alone (the
    # copy's mode-1 lanes at 512 draws, product order), 8 GiB objects
    assert libs["lab"].s3dg_set_keystream_shape(ctx["lab"], 1, 0, 0, 0, u64(512), -1) == 0
    obj = 8 << 30
    from s3dlio_amd import object_entropy

    def dg1(k, j):
        assert libs[k].s3dg_dgen_fill(ctx[k], ctypes.c_void_p(buf.data_ptr() + (j % 8) * obj), u64(obj), u64(0),
                                      u64(1 << 40), u64(1), ctypes.c_uint32(0), ctypes.c_uint32(1),
                                      u64(object_entropy(0x5EED000000000001, j)), sh) == 0
    with torch.cuda.stream(st):
        for rnd in range(int(os.environ.get("LAB_ROUNDS", "4"))):
            for name in ("product", "lab"):
                dg1(name, 0)
                st.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for j in range(10):
                    dg1(name, j)
                e1.record(st)
                e1.synchronize()
                gbs = 10 * obj / (e0.elapsed_time(e1) * 1e6)
                print(json.dumps({"round": rnd, "case": "dg1_8g_" + name, "GBps": round(gbs, 1)}), flush=True)
                if rnd:
                    acc.setdefault("dg1_8g_" + name, []).append(gbs)
    for name, v in acc.items():
        print(json.dumps({"summary": name, "GBps_mean": round(sum(v) / len(v), 1), "rounds": len(v)}), flush=True)
    print("ks_xres_lab ok", flush=True)


if __name__ == "__main__":
    main()

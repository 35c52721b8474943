#!/usr/bin/env python3
"""Run tools/ceiling_lab.hip variants interleaved in one process (tooling)."""
import ctypes
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libceiling_lab.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(HERE, "ceiling_lab.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                               "-shared", "-o", SO, src])


def main():
    build()
    if "--build-only" in sys.argv:
        return
    import torch
    L = ctypes.CDLL(SO)
    L.lab_v11.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    gib = float(args[0]) if args else 16
    buf = torch.empty(int(gib * (1 << 30)), dtype=torch.uint8, device="cuda")
    n = buf.numel()
    p = buf.data_ptr()
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    V = {}
    base = torch.randint(0, 255, (4096,), dtype=torch.uint8, device="cuda")
    bp = base.data_ptr()
    V["v4 T=256 C=4096"] = lambda: L.lab_v4(ctypes.c_void_p(p), ctypes.c_uint64(n), ctypes.c_uint64(4096), 256, ctypes.c_void_p(sh))
    V["v8 shared-chain T=256 (1D)"] = lambda: L.lab_v8(ctypes.c_void_p(p), ctypes.c_uint64(n), 256, ctypes.c_void_p(bp), ctypes.c_void_p(sh))
    for nx in (2048, 256, 65536):
        V[f"v9 shared-chain 2D nx={nx}"] = (lambda x=nx: L.lab_v9(ctypes.c_void_p(p), ctypes.c_uint64(n), x, 0, ctypes.c_void_p(bp), ctypes.c_void_p(sh)))
        V[f"v10 ceiling 2D nx={nx}"] = (lambda x=nx: L.lab_v9(ctypes.c_void_p(p), ctypes.c_uint64(n), x, 1, ctypes.c_void_p(bp), ctypes.c_void_p(sh)))
    if "--k2" in sys.argv:   # K2 store-shape study only
        V.clear()
        for R in (32768, 8192, 4096):
            for seg in (128, 256, 512, 1024, 0):
                if seg and R < seg:
                    continue
                name = f"v11 region={R} seg={seg}" if seg else f"v12 wave-seq chunk={64 * R}"
                V[name] = (lambda r=R, g=seg: L.lab_v11(ctypes.c_void_p(p), ctypes.c_uint64(n), r, g, ctypes.c_void_p(sh)))
        L.lab_v11x.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                               ctypes.c_uint32, ctypes.c_void_p]
        for seg in (128, 512):
            for nt in (0, 1):
                for lds in (0, 40 * 1024, 80 * 1024, 150 * 1024):
                    V[f"v11x region=32768 seg={seg} nt={nt} lds={lds}"] = (
                        lambda g=seg, t=nt, d=lds: L.lab_v11x(ctypes.c_void_p(p), ctypes.c_uint64(n), 32768, g, t, d,
                                                            ctypes.c_void_p(sh)))
        V["v10 ceiling 2D nx=2048"] = lambda: L.lab_v9(ctypes.c_void_p(p), ctypes.c_uint64(n), 2048, 1, ctypes.c_void_p(bp), ctypes.c_void_p(sh))
    if "--xcd" in sys.argv:   # K2 store shape, XCD-aware region ownership vs wave-contiguous
        V.clear()
        L.lab_v13.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p]
        for R, seg, pol in [(4096, 512, 2), (4096, 512, 0), (4096, 512, 3), (8192, 512, 2), (4096, 1024, 2),
                            (4096, 256, 2), (16384, 512, 2)]:
            for x in (0, 1):
                V[f"v13 region={R} seg={seg} pol={pol} xcd={x}"] = (
                    lambda r=R, g=seg, q=pol, xx=x: L.lab_v13(ctypes.c_void_p(p), ctypes.c_uint64(n), r, g, xx, q,
                                                             ctypes.c_void_p(sh)))
        V["v10 ceiling 2D nx=2048"] = lambda: L.lab_v9(ctypes.c_void_p(p), ctypes.c_uint64(n), 2048, 1, ctypes.c_void_p(bp), ctypes.c_void_p(sh))
    if "--k2stride" in sys.argv:   # K2 store shape at non-power-of-two region strides (seg 512)
        V.clear()
        for R in (8192, 8704, 9216, 12288, 16384, 16896, 32768, 33280, 5120, 4608):
            V[f"v11 region={R} seg=512"] = (lambda r=R: L.lab_v11(ctypes.c_void_p(p), ctypes.c_uint64(n // r * r // 64 * 64 if False else n), r, 512, ctypes.c_void_p(sh)))
        V["v10 ceiling 2D nx=2048"] = lambda: L.lab_v9(ctypes.c_void_p(p), ctypes.c_uint64(n), 2048, 1, ctypes.c_void_p(bp), ctypes.c_void_p(sh))
    V["torch fill_"] = lambda: buf.fill_(7)
    res = {k: [] for k in V}
    for _ in range(5):
        for k, f in V.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st); f(); e1.record(st)
            torch.cuda.synchronize()
            res[k].append(n / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    for k, v in res.items():
        print(json.dumps({"variant": k, "GBps_median": round(statistics.median(v), 1), "max": round(max(v), 1)}))


if __name__ == "__main__":
    main()

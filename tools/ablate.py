#!/usr/bin/env python3
"""Diagnostic: build the product kernels with parts compiled out
(-DS3DG_ABLATE=k, see s3dg_kernels.hip) and time cfg2-shaped fills of each
variant interleaved in one process.  Tooling only; outputs are wrong by design."""
import ctypes, json, os, statistics, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_build")
VARIANTS = os.environ.get("ABLATE_VARIANTS", "0,1,2,3").split(",")   # S3DG_ABLATE bits (s3dg_kernels.hip)


def build():
    os.makedirs(OUT, exist_ok=True)
    from s3dlio_amd.build import SOURCES
    for k in VARIANTS:
        so = os.path.join(OUT, f"libablate{k}.so")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                               "-shared", f"-DS3DG_ABLATE={k}", "-mllvm", "-amdgpu-kernarg-preload-count=16",
                               "-I", os.path.join(ROOT, "include"),
                               "-I", os.path.join(ROOT, "s3dlio_amd", "csrc"), "-o", so] + SOURCES)


def main():
    if "--build-only" in sys.argv:
        build(); return
    import torch
    libs = {}
    for k in VARIANTS:
        L = ctypes.CDLL(os.path.join(OUT, f"libablate{k}.so"), mode=os.RTLD_LOCAL)
        h = ctypes.c_void_p()
        assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
        libs[k] = (L, h)
    size, n = 8 << 20, 8192
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream(); sh = ctypes.c_void_p(st.cuda_stream)
    u64 = ctypes.c_uint64
    def run(k, d=1, fn=0, fd=1):
        L, h = libs[k]
        r = L.s3dg_fill_controlled_stream(h, ctypes.c_void_p(buf.data_ptr()), u64(size), u64(size), u64(n),
                                          u64(d), ctypes.c_uint32(fn), ctypes.c_uint32(fd), u64(1), u64(0), sh)
        assert r == 0
    shapes = [(2, 14), (2, 12), (2, 10), (2, 8), (1, 16), (1, 12), (1, 8), (4, 4), (4, 6)]
    res = {}
    for _ in range(3):
        for k in VARIANTS:
            for w, cap in shapes:
                L, h = libs[k]
                assert L.s3dg_set_waves_per_block(h, w) == 0
                assert L.s3dg_set_occupancy(h, cap, cap) == 0
                for (d, fn, fd) in [(1, 0, 1)]:
                    run(k, d, fn, fd)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st); run(k, d, fn, fd); e1.record(st); torch.cuda.synchronize()
                    res.setdefault((k, w, cap, d, fd), []).append(buf.numel() / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    for (k, w, cap, d, fd), v in res.items():
        print(json.dumps({"ablate": k, "waves": w, "cap": cap, "dedup": d, "f_den": fd,
                          "GBps": round(statistics.median(v), 1)}))


if __name__ == "__main__":
    main()

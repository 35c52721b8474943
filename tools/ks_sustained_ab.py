#!/usr/bin/env python3
"""Sustained A/B of keystream library variants (tooling): each variant runs
10 x 8 GiB DG1 / K2 launches back to back, 20 times in a row (as bench.py's
timed steps), alternating variants; HIP events around the 20 steps.
    LAB_VARIANTS="tail=;notail=-DS3DG_KS_NOTAIL=1" python tools/variant_lab.py --build-only
    LAB_VARIANTS=... python tools/ks_sustained_ab.py
Nothing in the product imports this."""
import ctypes, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GiB, MiB = 1 << 30, 1 << 20


def main():
    import torch
    from tools.variant_lab import so, variants
    from s3dlio_amd import object_entropy
    n, steps = 10, 20
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    buf = torch.empty(n * 8 * GiB, dtype=torch.uint8, device="cuda")
    libs = {}
    for name in variants():
        L = ctypes.CDLL(so(name), mode=os.RTLD_LOCAL)
        h = ctypes.c_void_p()
        assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
        libs[name] = (L, h)

    def step(L, h, kind):
        for t in range(n):
            q = ctypes.c_void_p(buf.data_ptr() + t * 8 * GiB)
            if kind == "k2_8g":
                r = L.s3dg_xoshiro_fill(h, q, u64(8 * GiB), u64(2 * MiB), u64(t * 4096), sh)
            else:
                d, fn, fd = (2, 1, 2) if kind == "dg1c2_8g" else (1, 0, 1)
                r = L.s3dg_dgen_fill(h, q, u64(8 * GiB), u64(0), u64(1 << 40), u64(d), u32(fn), u32(fd),
                                     u64(object_entropy(0x5EED000000000001, t)), sh)
            assert r == 0
    res = {}
    for rep in range(3):
        for kind in ("dg1_8g", "dg1c2_8g", "k2_8g"):
            for name, (L, h) in libs.items():
                for _ in range(3):
                    step(L, h, kind)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(steps):
                    step(L, h, kind)
                e1.record(st)
                torch.cuda.synchronize()
                res.setdefault((kind, name), []).append(steps * n * 8 * GiB / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        print(f"rep {rep} done", flush=True)
    for (kind, name), v in sorted(res.items()):
        print(json.dumps({"kind": kind, "variant": name, "GBps_median": round(statistics.median(v), 1),
                          "all": [round(x) for x in v]}), flush=True)


if __name__ == "__main__":
    main()

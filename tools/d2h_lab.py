#!/usr/bin/env python3
"""Diagnostic: D2H bandwidth into pinned host memory, A/B interleaved in one
process: torch pin_memory vs s3dg_host_alloc_pinned_local (GPU's NUMA node)
vs plain s3dg_host_alloc_pinned; pure copies of 32 x 8 MiB chunks.
Tooling only."""
import ctypes, json, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import s3dlio_amd as S
    from s3dlio_amd._lib import call
    MiB, GiB = 1 << 20, 1 << 30
    ctx = S.Context(0)
    cb = 256 * MiB
    dev = [torch.empty(cb, dtype=torch.uint8, device="cuda") for _ in range(2)]
    for d in dev:
        ctx.fill_controlled(d, cb, entropy=1)
    kinds = {}
    kinds["torch_pin"] = [int(torch.empty(cb, dtype=torch.uint8, pin_memory=True).data_ptr()) for _ in range(2)]
    keep = [torch.empty(1)]
    tp = [torch.empty(cb, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    kinds["torch_pin"] = [int(t.data_ptr()) for t in tp]
    for name, fn in (("local", "s3dg_host_alloc_pinned_local"), ("default", "s3dg_host_alloc_pinned")):
        ptrs = []
        for _ in range(2):
            p = ctypes.c_void_p()
            if fn.endswith("local"):
                call(fn, 0, cb, ctypes.byref(p))
            else:
                call(fn, cb, ctypes.byref(p))
            ptrs.append(p.value)
        kinds[name] = ptrs
    st = [torch.cuda.Stream() for _ in range(2)]
    res = {}
    for rep in range(5):
        for name, ptrs in kinds.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(16):
                s = k & 1
                call("s3dg_d2h_async", ctx._h, ptrs[s], dev[s].data_ptr(), cb, int(st[s].cuda_stream))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res.setdefault(name, []).append(16 * cb / dt / GiB)
    node = ctypes.c_int(-1)
    call("s3dg_device_numa_node", 0, ctypes.byref(node))
    for name, v in res.items():
        print(json.dumps({"host": name, "numa_node": node.value, "GiBps_median": round(statistics.median(v), 2),
                          "all": [round(x, 1) for x in v]}))
    del keep


if __name__ == "__main__":
    main()

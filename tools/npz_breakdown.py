#!/usr/bin/env python3
"""Where does generate_npz_bytes([6053,6053,1]) spend its time? (tooling)"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def best(f, reps=5):
    f()
    b = 1e9
    for _ in range(reps):
        t = time.perf_counter(); f(); b = min(b, time.perf_counter() - t)
    return b * 1e3


def main():
    import numpy as np
    import torch
    import s3dlio_amd as S
    from s3dlio_amd._lib import call
    from s3dlio_amd.npz import _shape_arr, default_context
    shape, dt, ns = [6053, 6053, 1], "<f4", 1
    arr, nd = _shape_arr(shape)
    total = S.npz_size(shape, dt, ns)
    ctx = default_context()
    build = lambda out: call("s3dg_npz_build", ctx._h, arr, nd, dt.encode(), ns, int(out.ctypes.data), total)
    res = {}
    res["generate_npz_bytes (pooled output, view dropped each call)"] = best(lambda: S.generate_npz_bytes(shape, dt, ns))
    keep = []
    res["generate_npz_bytes (pooled output, views kept -> new mappings)"] = best(
        lambda: keep.append(S.generate_npz_bytes(shape, dt, ns)), reps=3)
    keep.clear()
    res["generate_data 1 GiB (pooled output)"] = best(lambda: S.generate_data(1 << 30), reps=3)
    reuse = np.empty(total, np.uint8); reuse[:] = 0
    res["s3dg_npz_build into a reused, pre-faulted pageable buffer"] = best(lambda: build(reuse))
    pin = torch.empty(total, dtype=torch.uint8, pin_memory=True).numpy()
    res["s3dg_npz_build into a pinned buffer"] = best(lambda: build(pin))
    res["np.empty + first-touch memset (page faults)"] = best(lambda: np.empty(total, np.uint8).fill(0))
    res["memcpy pinned -> reused pageable (numpy copyto)"] = best(lambda: np.copyto(reuse, pin))
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    def d2h_pageable():
        reuse_t = torch.from_numpy(reuse)
        reuse_t.copy_(dev); torch.cuda.synchronize()
    def d2h_pinned():
        torch.from_numpy(pin).copy_(dev); torch.cuda.synchronize()
    res["torch D2H 140 MiB -> pageable"] = best(d2h_pageable)
    res["torch D2H 140 MiB -> pinned"] = best(d2h_pinned)
    for k, v in res.items():
        print(json.dumps({"what": k, "ms": round(v, 2)}))


if __name__ == "__main__":
    main()

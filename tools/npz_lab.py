#!/usr/bin/env python3
"""Where generate_npz_bytes([6053, 6053, 1]) spends its time, by output
buffer kind: the hostbuf pool mapping (MADV_HUGEPAGE), a plain touched numpy
array, the same registered with hipHostRegister, and pinned hipHostMalloc
memory; plus the bare D2H of the same 140 MiB from a device buffer into each.
Tooling only (GPU box)."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import s3dlio_amd as S
    from s3dlio_amd import hostbuf
    from s3dlio_amd._lib import c_u64, call
    from s3dlio_amd.npz import _shape_arr, default_context
    hip = ctypes.CDLL("libamdhip64.so")
    shape = [6053, 6053, 1]
    n = S.npz_size(shape) if hasattr(S, "npz_size") else None
    from s3dlio_amd.npz import npz_size
    n = npz_size(shape)
    arr, nd = _shape_arr(shape)
    ctx = default_context()
    bufs = {}
    bufs["hostbuf"] = hostbuf.empty(n)
    bufs["hostbuf"][:] = 1
    bufs["numpy"] = np.ones(n, np.uint8)
    reg = np.ones(n, np.uint8)
    assert hip.hipHostRegister(ctypes.c_void_p(reg.ctypes.data), ctypes.c_size_t(n), 0) == 0
    bufs["numpy_registered"] = reg
    p = ctypes.c_void_p()
    call("s3dg_host_alloc_pinned", n, ctypes.byref(p))
    pinned = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p.value))
    pinned[:] = 1
    bufs["pinned"] = pinned
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    res = {}
    for rep in range(5):
        for name, b in bufs.items():
            t = time.perf_counter()
            call("s3dg_npz_build", ctx._h, arr, nd, b"<f4", 1, int(b.ctypes.data), n)
            res.setdefault(("npz_build", name), []).append((time.perf_counter() - t) * 1e3)
            torch.cuda.synchronize()
            t = time.perf_counter()
            call("s3dg_d2h_async", ctx._h, int(b.ctypes.data), dev.data_ptr(), n, 0)
            call("s3dg_sync", ctx._h, 0)
            res.setdefault(("d2h_140MiB", name), []).append((time.perf_counter() - t) * 1e3)
    ref = bytes(bufs["pinned"])
    ok = all(bytes(bufs[k]) == ref for k in ("hostbuf", "numpy", "numpy_registered"))
    t = time.perf_counter()
    r2 = np.ones(n, np.uint8)
    t1 = time.perf_counter()
    hip.hipHostRegister(ctypes.c_void_p(r2.ctypes.data), ctypes.c_size_t(n), 0)
    t2 = time.perf_counter()
    hip.hipHostUnregister(ctypes.c_void_p(r2.ctypes.data))
    t3 = time.perf_counter()
    for (what, name), v in sorted(res.items()):
        print(json.dumps({"what": what, "buffer": name, "ms_median": round(statistics.median(v), 3),
                          "ms_all": [round(x, 3) for x in v]}))
    print(json.dumps({"archives_identical": ok, "hipHostRegister_140MiB_ms": round((t2 - t1) * 1e3, 3),
                      "hipHostUnregister_ms": round((t3 - t2) * 1e3, 3)}))


if __name__ == "__main__":
    main()

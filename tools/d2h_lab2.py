#!/usr/bin/env python3
"""Diagnostic: is the D2H rate a property of the stream (the copy engine the
runtime binds it to)?  For each of N fresh streams: 6 timed 256 MiB D2H
copies into a pinned host buffer on the GPU's NUMA node, alone and then with
a fill kernel looping on another stream.  Per-copy rates from HIP events on
the copy stream.  Run once as is and once with HSA_ENABLE_SDMA=0.
Tooling only."""
import ctypes, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import s3dlio_amd as S
    from s3dlio_amd._lib import call
    MiB, GiB = 1 << 20, 1 << 30
    ctx = S.Context(0)
    cb = 256 * MiB
    src = torch.empty(cb, dtype=torch.uint8, device="cuda")
    ctx.fill_controlled(src, cb, entropy=1)
    big = torch.empty(8 * GiB, dtype=torch.uint8, device="cuda")
    host = ctypes.c_void_p()
    call("s3dg_host_alloc_pinned_local", 0, cb, ctypes.byref(host))
    busy = torch.cuda.Stream()
    nst = int(os.environ.get("LAB_STREAMS", "8"))
    for mode in ("alone", "with_fill"):
        for k in range(nst):
            st = torch.cuda.Stream()
            rates = []
            call("s3dg_d2h_async", ctx._h, host.value, src.data_ptr(), cb, int(st.cuda_stream))
            for _ in range(6):
                if mode == "with_fill":
                    ctx.fill_stream(big, obj_size=8 * MiB, n_objs=1024, stream=busy)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                call("s3dg_d2h_async", ctx._h, host.value, src.data_ptr(), cb, int(st.cuda_stream))
                e1.record(st)
                torch.cuda.synchronize()
                rates.append(cb / (e0.elapsed_time(e1) * 1e-3) / GiB)
            print(json.dumps({"mode": mode, "stream": k, "sdma": os.environ.get("HSA_ENABLE_SDMA", "default"),
                              "GiBps_median": round(statistics.median(rates), 1),
                              "all": [round(r, 1) for r in rates]}), flush=True)
    call("s3dg_host_free_pinned", host.value)


if __name__ == "__main__":
    main()

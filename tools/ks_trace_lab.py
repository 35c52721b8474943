#!/usr/bin/env python3
"""k_keystream wave timeline (tooling): a diagnostic build (-DS3DG_KS_TRACE=1)
stamps every wave's start and end with the 100 MHz wall clock; this prints,
per launch, the active-wave profile over time: how long the launch takes to
fill the chip, how long its tail is, and the mean wave duration.

    LAB_VARIANTS="trace=-DS3DG_KS_TRACE=1" python tools/variant_lab.py --build-only   # here
    python tools/ks_trace_lab.py                                                       # GPU box
Nothing in the product imports this."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GiB, MiB = 1 << 30, 1 << 20


def main():
    import torch
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libvariant_trace.so"), mode=os.RTLD_LOCAL)
    h = ctypes.c_void_p()
    assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    tick_ns = 10.0          # s_memrealtime: 100 MHz (span_us is printed beside the event time to check)
    buf = torch.empty(64 * GiB, dtype=torch.uint8, device="cuda")
    trace = torch.zeros(2 * (1 << 22), dtype=torch.int64, device="cuda")
    assert L.s3dg_diag_ks_trace(ctypes.c_void_p(trace.data_ptr())) == 0
    cases = []
    for mode in (0, 1):
        for gib in (8, 64):
            for draws in (1024, 2048):
                cases.append((mode, gib, draws))
    for mode, gib, draws in cases:
        assert L.s3dg_set_keystream_shape(h, mode, 64, 4, 0, u64(draws), -1) == 0
        n = gib * GiB
        p = ctypes.c_void_p(buf.data_ptr())

        def run():
            if mode == 0:
                return L.s3dg_xoshiro_fill(h, p, u64(n), u64(2 * MiB), u64(0), sh)
            return L.s3dg_dgen_fill(h, p, u64(n), u64(0), u64(1 << 40), u64(1), u32(0), u32(1), u64(777), sh)
        assert run() == 0
        trace.zero_()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        assert run() == 0
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        t = trace.view(-1, 2).cpu()
        t = t[t[:, 1] > 0]
        s, e = t[:, 0].double(), t[:, 1].double()
        t0 = s.min()
        s, e = (s - t0) * tick_ns / 1e3, (e - t0) * tick_ns / 1e3      # us from the first wave's start
        T = float(e.max())
        dur = e - s
        # active waves over time, 200 bins
        import numpy as np
        bins = np.linspace(0, T, 201)
        sn, en = s.numpy(), e.numpy()
        active = [int(((sn <= b) & (en > b)).sum()) for b in bins[:-1]]
        full = max(active)
        fill_us = float(bins[next(i for i, a in enumerate(active) if a >= 0.95 * full)])
        tail_start = float(bins[max(i for i, a in enumerate(active) if a >= 0.95 * full)])
        area = float(dur.sum()) / (full * T)
        print(json.dumps({"mode": ["k2", "dg1c1"][mode], "GiB": gib, "draws_per_lane": draws,
                          "event_ms": round(ms, 3), "GBps": round(n / ms / 1e6, 1),
                          "waves": int(len(sn)), "max_active_waves": full,
                          "span_us": round(T, 1), "wave_us_median": round(float(dur.median()), 1),
                          "wave_us_p5_p95": [round(float(dur.quantile(0.05)), 1), round(float(dur.quantile(0.95)), 1)],
                          "first_end_us": round(float(e.min()), 1),
                          "reach_95pct_active_us": round(fill_us, 1), "last_95pct_active_us": round(tail_start, 1),
                          "occupancy_area": round(area, 4),
                          "active_profile_20": [active[i] for i in range(0, 200, 10)]}), flush=True)


if __name__ == "__main__":
    main()

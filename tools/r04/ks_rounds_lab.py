#!/usr/bin/env python3
"""Where DG1's per-object launches lose against one launch (VERDICT r03 weak
#6: configs 14/15 at 0.77 against config 16's 0.83).  A diagnostic build
(-DS3DG_KS_TRACE=1) stamps every keystream wave's start and end with the
100 MHz wall clock.  Ten 8 GiB DG1 c1 launches back to back (config 14's
pattern; each launch overwrites the same trace slots, so the trace keeps the
last one) against one 80 GiB launch (config 16's), default launch shape.
Per launch: the event time, the span of its waves, the waves in flight over
time, and the wave durations by round (waves ranked by start, one round =
the chip's resident waves).

    LAB_VARIANTS="trace=-DS3DG_KS_TRACE=1" python tools/variant_lab.py --build-only   # here
    python tools/r04/ks_rounds_lab.py                                                 # GPU box
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
GiB, MiB = 1 << 30, 1 << 20
TICK_US = 0.01          # s_memrealtime: 100 MHz


def analyse(trace, name, event_ms, nbytes):
    import numpy as np
    t = trace.view(-1, 2).cpu().numpy()
    # XCD of trace slot wi (1-wave workgroups, XCD groups of 16): the remap puts
    # the 16 units of XCD x at bid = 128 * (k >> 4) + 16 * x + (k & 15)
    wi = np.nonzero(t[:, 1] > 0)[0]
    xg = int(os.environ.get("LAB_XG", "16"))
    xcd = (wi // xg) & 7
    t = t[t[:, 1] > 0]
    t0 = t[:, 0].min()
    per_xcd = {}
    for x in range(8):
        sel = t[xcd == x]
        if len(sel):
            per_xcd[x] = {"waves": int(len(sel)), "last_end_us": round(float((sel[:, 1].max() - t0) * TICK_US), 1),
                          "wave_us_mean": round(float(((sel[:, 1] - sel[:, 0]) * TICK_US).mean()), 1)}
    s = (t[:, 0] - t[:, 0].min()) * TICK_US
    e = (t[:, 1] - t[:, 0].min()) * TICK_US
    dur = e - s
    span = float(e.max())
    bins = np.linspace(0, span, 41)
    active = [int(((s <= b) & (e > b)).sum()) for b in bins[:-1]]
    full = max(active)
    order = np.argsort(s, kind="stable")
    rounds = []
    for r in range(0, len(order), full):
        d = dur[order[r:r + full]]
        rounds.append(round(float(np.median(d)), 1))
    area = float(dur.sum()) / (full * span)
    # time the chip is not full at the end: from the last moment >= 95 % busy to the last wave's end
    busy = [i for i, a in enumerate(active) if a >= 0.95 * full]
    tail_us = span - float(bins[busy[-1] + 1]) if busy else None
    # units in flight over the last 200 us, 10-us bins (end of launch)
    tb = np.arange(span - 200.0, span, 10.0)
    end_profile = [int(((s <= b) & (e > b)).sum()) for b in tb]
    # the first unit each resident slot ran vs the rest (ramp cost per unit)
    first = dur[order[:full]]
    rest = dur[order[full:]]
    return {"case": name, "end_profile_10us": end_profile,
            "first_round_us_median": round(float(np.median(first)), 1),
            "later_units_us_median": round(float(np.median(rest)), 1) if len(rest) else None,
            "unit_us_p5_p95": [round(float(np.quantile(dur, 0.05)), 1), round(float(np.quantile(dur, 0.95)), 1)], "event_ms": round(event_ms, 3), "GBps": round(nbytes / event_ms / 1e6, 1),
            "waves": int(len(s)), "resident": full, "span_us": round(span, 1),
            "event_minus_span_us": round(event_ms * 1e3 - span, 1), "occupancy_area": round(area, 4),
            "tail_not_full_us": round(tail_us, 1) if tail_us is not None else None,
            "wave_us_median_by_round": rounds[:12] + (["..."] + rounds[-3:] if len(rounds) > 15 else rounds[12:]),
            "active_profile_40": active, "per_xcd": per_xcd}


def main():
    import torch
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", os.environ.get("LAB_LIB", "libvariant_trace.so")),
                    mode=os.RTLD_LOCAL)
    h = ctypes.c_void_p()
    assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
    if os.environ.get("LAB_TAIL"):      # round 5: tail chunks of half-length units (0: none, so slots do not collide)
        assert L.s3dg_set_keystream_tail(h, ctypes.c_int(int(os.environ["LAB_TAIL"]))) == 0
    if os.environ.get("LAB_XG"):        # units per XCD group of the remap (1: plain round-robin dealing)
        assert L.s3dg_set_keystream_xcd_group(h, 1, ctypes.c_uint32(int(os.environ["LAB_XG"]))) == 0
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    n_obj = 10
    # LAB_SHIFT_MIB: every launch's dst moved up by that many MiB (round 5: do
    # the slow unit groups follow the addresses they write or the XCDs?)
    shift = int(os.environ.get("LAB_SHIFT_MIB", "0")) * MiB
    buf0 = torch.empty(n_obj * 8 * GiB + shift, dtype=torch.uint8, device="cuda")
    buf = buf0[shift:]
    trace = torch.zeros(2 * (n_obj * 8 * GiB // MiB) * 2, dtype=torch.int64, device="cuda")
    assert L.s3dg_diag_ks_trace(ctypes.c_void_p(trace.data_ptr())) == 0
    SEED = 0x5EED000000000001

    def per_object():   # config 14: one s3dg_dgen_fill per 8 GiB object
        for t in range(n_obj):
            q = ctypes.c_void_p(buf.data_ptr() + t * 8 * GiB)
            assert L.s3dg_dgen_fill(h, q, u64(8 * GiB), u64(0), u64(1 << 40), u64(1), u32(0), u32(1),
                                    u64(SEED + t), sh) == 0

    def one_launch():   # config 16: the ten objects in one s3dg_dgen_fill_stream launch
        assert L.s3dg_dgen_fill_stream(h, ctypes.c_void_p(buf.data_ptr()), u64(8 * GiB), u64(8 * GiB), u64(n_obj),
                                       u64(1), u32(0), u32(1), u64(SEED), u64(0), sh) == 0

    for rep in range(int(os.environ.get("LAB_REPS", "3"))):
        for name, fn in (("10 x 8 GiB launches (last one traced)", per_object), ("one 80 GiB launch", one_launch)):
            fn()                      # warm
            torch.cuda.synchronize()
            trace.zero_()
            torch.cuda.synchronize()
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            evs[0].record(st)
            fn()
            evs[1].record(st)
            torch.cuda.synchronize()
            total_ms = evs[0].elapsed_time(evs[1])
            if fn is per_object:
                # the traced (last) launch alone, timed on its own after the same nine
                for t in range(n_obj - 1):
                    q = ctypes.c_void_p(buf.data_ptr() + t * 8 * GiB)
                    assert L.s3dg_dgen_fill(h, q, u64(8 * GiB), u64(0), u64(1 << 40), u64(1), u32(0), u32(1),
                                            u64(SEED + t), sh) == 0
                trace.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                q = ctypes.c_void_p(buf.data_ptr() + (n_obj - 1) * 8 * GiB)
                assert L.s3dg_dgen_fill(h, q, u64(8 * GiB), u64(0), u64(1 << 40), u64(1), u32(0), u32(1),
                                        u64(SEED + n_obj - 1), sh) == 0
                e1.record(st)
                torch.cuda.synchronize()
                res = analyse(trace, name, e0.elapsed_time(e1), 8 * GiB)
            else:
                res = analyse(trace, name, total_ms, n_obj * 8 * GiB)
            res["rep"] = rep
            res["all_ten_objects_GBps"] = round(n_obj * 8 * GiB / total_ms / 1e6, 1)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

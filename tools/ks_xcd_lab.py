#!/usr/bin/env python3
"""Why are half of a keystream launch's units slower (round 5)?  Wave timelines
of the persistent k_keystream (tools/r04/ks_rounds_lab.py) show the units of
queues 1/3/5/7 taking 166-195 us against 145-160 us for queues 0/2/4/6,
whatever 16 MiB address group they write (LAB_SHIFT_MIB=16) and however the
units are grouped (LAB_XG=1).  The trace build (-DS3DG_KS_TRACE=1) now stamps
each unit with the hardware ids of the wave that ran it (HW_ID: wave slot,
SIMD, CU, shader array/engine; XCC_ID), so this groups unit durations by the
XCD that ran them, by the SIMD placement of the CU's resident waves, and by
queue.

    LAB_VARIANTS="trace=-DS3DG_KS_TRACE=1" python tools/variant_lab.py --build-only   # here
    python tools/ks_xcd_lab.py                                                        # GPU box
Tooling only: nothing in the product imports this."""
import collections, ctypes, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GiB, MiB = 1 << 30, 1 << 20
TICK_US = 0.01
M48 = (1 << 48) - 1


def analyse(trace, name, event_ms, nbytes, xg):
    import numpy as np
    t = trace.view(-1, 2).cpu().numpy().astype(np.uint64)
    wi = np.nonzero(t[:, 1] > 0)[0]
    t = t[wi]
    s = (t[:, 0] & M48).astype(np.int64)
    e = (t[:, 1] & M48).astype(np.int64)
    hw = (t[:, 0] >> np.uint64(48)).astype(np.int64)
    xcc = (t[:, 1] >> np.uint64(48)).astype(np.int64) & 15
    t0 = s.min()
    s, e = (s - t0) * TICK_US, (e - t0) * TICK_US
    dur = e - s
    queue = (wi // xg) & 7
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xFF          # CU_ID, SH_ID, SE_ID
    out = {"case": name, "event_ms": round(event_ms, 3), "GBps": round(nbytes / event_ms / 1e6, 1),
           "units": int(len(wi)), "span_us": round(float(e.max()), 1)}
    per_xcc = {}
    for x in range(8):
        m = xcc == x
        if m.any():
            per_xcc[x] = {"units": int(m.sum()), "unit_us_mean": round(float(dur[m].mean()), 1),
                          "last_end_us": round(float(e[m].max()), 1),
                          "cus": int(len(set(cu[m].tolist()))),
                          "queues": dict(collections.Counter(queue[m].tolist()))}
    out["per_xcc"] = per_xcc
    per_q = {}
    for q in range(8):
        m = queue == q
        if m.any():
            per_q[q] = {"unit_us_mean": round(float(dur[m].mean()), 1),
                        "xccs": dict(collections.Counter(xcc[m].tolist()))}
    out["per_queue"] = per_q
    # resident waves per CU and per SIMD: the distinct (SIMD, wave slot) ids seen on a CU
    slots = collections.defaultdict(set)
    for x_, c_, h_ in zip(xcc.tolist(), cu.tolist(), hw.tolist()):
        slots[(x_, c_)].add(h_ & 0xFF)
    per_cu_waves = collections.Counter(len(v) for v in slots.values())
    simd_load = collections.Counter()
    for (x_, c_), v in slots.items():
        k = collections.Counter((h >> 4) & 3 for h in v)
        simd_load[(x_ % 2, tuple(sorted(k.values(), reverse=True)))] += 1
    out["cus_by_resident_waves"] = dict(per_cu_waves)
    out["cus_by_xcc_parity_and_waves_per_simd"] = {f"{a}:{b}": n for (a, b), n in sorted(simd_load.items())}
    # unit duration by how many resident waves share the unit's SIMD
    share = {}
    for (x_, c_), v in slots.items():
        k = collections.Counter((h >> 4) & 3 for h in v)
        for h in v:
            share[(x_, c_, h)] = k[(h >> 4) & 3]
    sh = np.array([share[(x_, c_, h_ & 0xFF)] for x_, c_, h_ in zip(xcc.tolist(), cu.tolist(), hw.tolist())])
    out["unit_us_by_waves_on_simd"] = {int(k): [int((sh == k).sum()), round(float(dur[sh == k].mean()), 1)]
                                       for k in sorted(set(sh.tolist()))}
    return out


def main():
    import torch
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", os.environ.get("LAB_LIB", "libvariant_trace.so")),
                    mode=os.RTLD_LOCAL)
    h = ctypes.c_void_p()
    assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
    assert L.s3dg_set_keystream_tail(h, ctypes.c_int(int(os.environ.get("LAB_TAIL", "0")))) == 0
    xg = int(os.environ.get("LAB_XG", "16"))
    if os.environ.get("LAB_XG"):
        assert L.s3dg_set_keystream_xcd_group(h, 1, ctypes.c_uint32(xg)) == 0
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    n_obj = 10
    buf = torch.empty(n_obj * 8 * GiB, dtype=torch.uint8, device="cuda")
    trace = torch.zeros(2 * (n_obj * 8 * GiB // MiB) * 2, dtype=torch.int64, device="cuda")
    assert L.s3dg_diag_ks_trace(ctypes.c_void_p(trace.data_ptr())) == 0
    SEED = 0x5EED000000000001
    p = buf.data_ptr()

    def one(gib, nobj):
        assert L.s3dg_dgen_fill_stream(h, ctypes.c_void_p(p), u64(gib * GiB), u64(gib * GiB), u64(nobj),
                                       u64(1), u32(0), u32(1), u64(SEED), u64(0), sh) == 0

    for rep in range(int(os.environ.get("LAB_REPS", "2"))):
        for name, gib, nobj in (("one 8 GiB object", 8, 1), ("ten 8 GiB objects, one launch", 8, 10)):
            one(gib, nobj)
            torch.cuda.synchronize()
            trace.zero_()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            one(gib, nobj)
            e1.record(st)
            torch.cuda.synchronize()
            res = analyse(trace, name, e0.elapsed_time(e1), gib * nobj * GiB, xg)
            res["rep"] = rep
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Config 2's slow launches (12.1-12.7 ms against 11.0-11.2 ms on some boxes,
DESIGN.md §5.1.4): do launch settings that run the chip a little below its
1400 W limit avoid them, and what do they cost where there are none?  One
library, one context per setting (s3dg_set_batch_pace: wall-clock store
floor in 10-ns ticks; s3dg_set_occupancy: resident workgroups per CU),
blocks of LAB_BLOCK (20) back-to-back config-2 launches per setting per rep
(as bench.py's steps), settings rotated; every launch timed with HIP events.
Per setting: mean / p10 / p90 ms, the share of launches slower than 1.06 x
the fastest setting's p10, and the amdsmi power, GFX clock and PPT residency
during its blocks.

    python tools/dip_lab.py        # GPU box; LAB_SETTINGS "name=pace/occ;...",
                                   # LAB_POINT cfg2 (default) | cfg3 | cfg4 | cfg5 | cfg8
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, sys, threading, time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
MiB = 1 << 20
DEFAULT = "plain=-1/-1;pace20=20/-1;pace50=50/-1;pace100=100/-1;occ30=-1/30;occ28=-1/28"
# config 5 (d2 c3, the mid-line class): the library default (the tuner's pick
# of floor 100 or plain), each setting forced, and the cap without the floor
DEFAULT_CFG5 = "default=-1/-1;plain=0/-1;pace100=100/-1;pace150=150/-1;pace200=200/-1;cap29=0/29"


def main():
    import torch
    from s3dlio_amd._lib import lib
    from zero_power_lab import smi_handle
    u64, u32, vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p
    n = 10000
    buf = torch.empty(8 * MiB * n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sh = vp(st.cuda_stream)
    p = vp(buf.data_ptr())
    ctxs = {}
    point = os.environ.get("LAB_POINT", "cfg2")
    for item in os.environ.get("LAB_SETTINGS", DEFAULT_CFG5 if point == "cfg5" else DEFAULT).split(";"):
        name, _, spec = item.partition("=")
        pace, occ = (int(x) for x in spec.split("/"))
        h = vp()
        assert lib.s3dg_ctx_create(0, ctypes.byref(h)) == 0
        if pace >= 0:
            assert lib.s3dg_set_batch_pace(h, pace) == 0
        if occ >= 0:
            assert lib.s3dg_set_occupancy(h, -1, occ) == 0
        ctxs[name] = h

    work = 8 * MiB * n
    if point == "cfg4":      # BASELINE config 4: 10 000 log-uniform objects, d2 c1.5, batch API
        from bench import log_uniform_sizes
        from s3dlio_amd._lib import ObjDesc
        sizes = log_uniform_sizes(n)
        arr = (ObjDesc * n)()
        off = 0
        for j, sz in enumerate(sizes):
            arr[j] = ObjDesc(off, sz, 0x5EED000000000001 + (j << 32), 2, 1, 3)
            off += (sz + 4095) // 4096 * 4096
        work = sum(sizes)

    def launch(h):
        if point == "cfg8":  # config 8: 1 000 000 x 64 KiB, stream API
            r = lib.s3dg_fill_controlled_stream(h, p, u64(64 << 10), u64(64 << 10), u64(1000000), u64(1), u32(0),
                                                u32(1), u64(0x5EED000000000001), u64(0), sh)
        elif point == "cfg4":
            r = lib.s3dg_fill_controlled_batch(h, p, arr, u64(n), sh)
        elif point == "cfg5":  # config 5's launch shape: 10 000 x 8 MiB, d2 c3
            r = lib.s3dg_fill_controlled_stream(h, p, u64(8 * MiB), u64(8 * MiB), u64(n), u64(2), u32(2), u32(3),
                                                u64(0x5EED000000000001), u64(0), sh)
        elif point == "cfg3":  # config 3: 10 000 x 8 MiB, d4 c2
            r = lib.s3dg_fill_controlled_stream(h, p, u64(8 * MiB), u64(8 * MiB), u64(n), u64(4), u32(1), u32(2),
                                                u64(0x5EED000000000001), u64(0), sh)
        else:
            r = lib.s3dg_fill_controlled_stream(h, p, u64(8 * MiB), u64(8 * MiB), u64(n), u64(1), u32(0), u32(1),
                                                u64(0x5EED000000000001), u64(0), sh)
        assert r == 0
    smi, sm, bdf = smi_handle()
    rows, on = [], [True]

    def poller():
        while on[0]:
            try:
                m = smi.amdsmi_get_gpu_metrics_info(sm)
                rows.append((time.perf_counter(), m.get("current_gfxclk"), m.get("current_socket_power"),
                             m.get("ppt_residency_acc"), m.get("accumulation_counter"),
                             m.get("temperature_hotspot"), m.get("temperature_mem")))
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.005)
    th = threading.Thread(target=poller, daemon=True)
    th.start()
    block = int(os.environ.get("LAB_BLOCK", "20"))
    reps = int(os.environ.get("LAB_REPS", "15"))
    per, seg = {}, {}
    names = list(ctxs)
    for rep in range(reps):
        order = names[rep % len(names):] + names[:rep % len(names)]
        for name in order:
            h = ctxs[name]
            launch(h)
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(block)]
            t0 = time.perf_counter()
            for e0, e1 in evs:
                e0.record(st)
                launch(h)
                e1.record(st)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            per.setdefault(name, []).extend(a.elapsed_time(b) for a, b in evs)
            seg.setdefault(name, []).append((t0, t1))
        print(f"rep {rep} done", flush=True)
    on[0] = False
    fastest = min(sorted(v)[len(v) // 10] for v in per.values())
    for name in names:
        v = sorted(per[name])
        sel = [r for r in rows if any(a < r[0] <= b for a, b in seg[name])]
        num = lambda i: [r[i] for r in sel if isinstance(r[i], (int, float))]  # noqa: E731
        mean = sum(v) / len(v)
        print(json.dumps({"setting": name, "point": point, "n": len(v), "ms_mean": round(mean, 4),
                          "GBps_mean": round(work / (mean * 1e-3) / 1e9, 1),
                          "frac": round(work / (mean * 1e-3) / 8e12, 4),
                          "ms_p10": round(v[len(v) // 10], 4), "ms_p50": round(v[len(v) // 2], 4),
                          "ms_p90": round(v[9 * len(v) // 10], 4), "ms_max": round(v[-1], 4),
                          "slow_share": round(sum(x > 1.06 * fastest for x in v) / len(v), 4),
                          "power_med": statistics.median(num(2)) if num(2) else None,
                          "gfxclk_med": statistics.median(num(1)) if num(1) else None,
                          "gfxclk_min": min(num(1)) if num(1) else None,
                          "hotspot_C_max": max(num(5)) if num(5) else None,
                          "hbm_C_max": max(num(6)) if num(6) else None}), flush=True)


if __name__ == "__main__":
    main()

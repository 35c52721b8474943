#!/usr/bin/env python3
"""Diagnostic (round 3): are config 2's occasional slow launches (11.9-12.9 ms
against 11.1-11.3 ms, seen on some boxes) power-limit transients?  Runs
config-2 launches back to back through the product library, times each one
with HIP events, polls the amdsmi GPU metrics every ~5 ms in a thread, and
reports the GFX clock, socket power and PPT residency seen during slow and
normal launches.

    python tools/step_power_lab.py        # GPU box; LAB_LAUNCHES (default 300)
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, sys, threading, time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from zero_power_lab import smi_handle  # noqa: E402

MiB = 1 << 20


def main():
    import torch
    from s3dlio_amd._lib import lib
    n = 10000
    launches = int(os.environ.get("LAB_LAUNCHES", "300"))
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    h = ctypes.c_void_p()
    assert lib.s3dg_ctx_create(0, ctypes.byref(h)) == 0
    buf = torch.empty(8 * MiB * n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    p = ctypes.c_void_p(buf.data_ptr())
    smi, sm, bdf = smi_handle()

    def launch():
        assert lib.s3dg_fill_controlled_stream(h, p, u64(8 * MiB), u64(8 * MiB), u64(n), u64(1), u32(0), u32(1),
                                               u64(0x5EED000000000001), u64(0), sh) == 0

    rows, on = [], [True]

    def poller():
        while on[0]:
            try:
                m = smi.amdsmi_get_gpu_metrics_info(sm)
                rows.append((time.perf_counter(), m.get("current_gfxclk"), m.get("current_socket_power"),
                             m.get("ppt_residency_acc"), m.get("accumulation_counter"), m.get("temperature_mem")))
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.005)

    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    th = threading.Thread(target=poller)
    th.start()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    t_host = []
    for e0, e1 in evs:
        e0.record(st)
        launch()
        e1.record(st)
    # host timestamps of each launch's end: wait event by event
    for e0, e1 in evs:
        e1.synchronize()
        t_host.append(time.perf_counter())
    on[0] = False
    th.join()
    ms = [e0.elapsed_time(e1) for e0, e1 in evs]
    med = statistics.median(ms)
    slow = [i for i, x in enumerate(ms) if x > 1.03 * med]

    def during(i):
        # samples taken while launch i ran: (end of i-1, end of i]; host stamps lag by the sync latency
        t1 = t_host[i]
        t0 = t_host[i - 1] if i else t1 - ms[i] / 1e3
        return [r for r in rows if t0 < r[0] <= t1]

    def summary(ids):
        clk = [r[1] for i in ids for r in during(i) if isinstance(r[1], (int, float))]
        pw = [r[2] for i in ids for r in during(i) if isinstance(r[2], (int, float))]
        return {"launches": len(ids), "ms_med": round(statistics.median([ms[i] for i in ids]), 3) if ids else None,
                "gfxclk_med": statistics.median(clk) if clk else None, "gfxclk_min": min(clk) if clk else None,
                "power_med": statistics.median(pw) if pw else None, "samples": len(clk)}
    normal = [i for i in range(launches) if i not in slow]
    acc = [(r[3], r[4]) for r in rows if isinstance(r[3], (int, float)) and isinstance(r[4], (int, float))]
    ppt = (acc[-1][0] - acc[0][0]) / max(1, acc[-1][1] - acc[0][1]) if len(acc) > 1 else None
    print(json.dumps({"smi_device": bdf, "launches": launches, "ms_median": round(med, 3),
                      "ms_p10_p90_max": [round(sorted(ms)[launches // 10], 3), round(sorted(ms)[9 * launches // 10], 3),
                                         round(max(ms), 3)],
                      "slow_over_3pct": len(slow), "slow_indices": slow[:40],
                      "GBps_median": round(8 * MiB * n / (med * 1e-3) / 1e9, 1),
                      "GBps_mean": round(8 * MiB * n * launches / (sum(ms) * 1e-3) / 1e9, 1),
                      "ppt_residency": round(ppt, 3) if ppt is not None else None,
                      "normal": summary(normal), "slow": summary(slow)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Power and rate of the fill's on-chip data movement (tools/reg_fill_lab.hip):
config 2's product fill against kernels that store the same random 4 KiB
base block into every granule of the same 78 GiB buffer, (a) loaded from L2
per granule, (b) through an LDS image, (c) from registers held by a
persistent grid (R workgroups, optional s_sleep pacing).  Each variant runs
back to back for LAB_SECONDS (default 1.5) per segment, segments interleaved
over LAB_REPS rounds; per launch HIP events give the rate, amdsmi (polled
every ~5 ms) the socket power, GFX clock and PPT residency during the
segment.

    python tools/reg_fill_lab.py --build    # here
    python tools/reg_fill_lab.py            # GPU box
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, subprocess, sys, threading, time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
OUT = os.path.join(ROOT, "tools", "_build")
LIB = os.path.join(OUT, "libreglab.so")
MiB = 1 << 20


def build():
    os.makedirs(OUT, exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-o", LIB, os.path.join(ROOT, "tools", "reg_fill_lab.hip")])


def main():
    if "--build" in sys.argv:
        build()
        return
    import torch
    from s3dlio_amd._lib import lib
    from zero_power_lab import smi_handle
    L = ctypes.CDLL(LIB)
    u64, u32, vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p
    L.lab_store_l2.argtypes = [vp, vp, u64, u32, vp]
    L.lab_store_lds.argtypes = [vp, vp, u64, u32, vp]
    L.lab_store_reg.argtypes = [vp, vp, u64, u32, u32, u32, vp]
    n = 10000
    nblk = 8 * MiB * n // 4096
    buf = torch.empty(8 * MiB * n, dtype=torch.uint8, device="cuda")
    g = torch.Generator().manual_seed(7)
    base = torch.randint(0, 256, (4096,), dtype=torch.uint8, generator=g).cuda()
    st = torch.cuda.current_stream()
    sh = vp(st.cuda_stream)
    h = vp()
    assert lib.s3dg_ctx_create(0, ctypes.byref(h)) == 0
    p, bp = vp(buf.data_ptr()), vp(base.data_ptr())
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    variants = {
        "fill_cfg2": lambda: lib.s3dg_fill_controlled_stream(h, p, u64(8 * MiB), u64(8 * MiB), u64(n), u64(1),
                                                             u32(0), u32(1), u64(0x5EED000000000001), u64(0), sh),
        "store_l2": lambda: L.lab_store_l2(p, bp, nblk, 0, sh),
        "store_lds": lambda: L.lab_store_lds(p, bp, nblk, 0, sh),
    }
    for wpc in [int(x) for x in os.environ.get("LAB_REG_WPC", "32,16,8").split(",")]:
        for spin in [int(x) for x in os.environ.get("LAB_REG_SPIN", "0,2").split(",")]:
            variants[f"reg_{wpc}pcu_s{spin}"] = (lambda wpc=wpc, spin=spin:
                                                 L.lab_store_reg(p, bp, nblk, cus * wpc, 0, spin, sh))
    smi, sm, bdf = smi_handle()
    rows, on = [], [True]

    def poller():
        while on[0]:
            try:
                m = smi.amdsmi_get_gpu_metrics_info(sm)
                rows.append((time.perf_counter(), m.get("current_gfxclk"), m.get("current_socket_power"),
                             m.get("ppt_residency_acc"), m.get("accumulation_counter")))
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.005)
    th = threading.Thread(target=poller, daemon=True)
    th.start()
    secs = float(os.environ.get("LAB_SECONDS", "1.5"))
    res = {}
    for rep in range(int(os.environ.get("LAB_REPS", "3"))):
        names = list(variants)
        names = names[rep % len(names):] + names[:rep % len(names)]
        for name in names:
            f = variants[name]
            assert f() == 0
            torch.cuda.synchronize()
            k = max(4, int(secs / 0.012))
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
            t0 = time.perf_counter()
            for e0, e1 in evs:
                e0.record(st)
                assert f() == 0
                e1.record(st)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ms = [a.elapsed_time(b) for a, b in evs]
            seg = [r for r in rows if t0 + 0.2 * (t1 - t0) < r[0] <= t1]
            clk = [r[1] for r in seg if isinstance(r[1], (int, float))]
            pw = [r[2] for r in seg if isinstance(r[2], (int, float))]
            acc = [(r[3], r[4]) for r in seg if isinstance(r[3], (int, float)) and isinstance(r[4], (int, float))]
            ppt = (acc[-1][0] - acc[0][0]) / max(1, acc[-1][1] - acc[0][1]) if len(acc) > 1 else None
            res.setdefault(name, []).append({"ms_mean": sum(ms) / len(ms), "ms_max": max(ms),
                                             "gfxclk": statistics.median(clk) if clk else None,
                                             "power": statistics.median(pw) if pw else None, "ppt": ppt})
        print(f"rep {rep} done", flush=True)
    on[0] = False
    for name, v in res.items():
        ms = statistics.median([x["ms_mean"] for x in v])
        print(json.dumps({"variant": name, "GBps": round(8 * MiB * n / (ms * 1e-3) / 1e9, 1),
                          "frac": round(8 * MiB * n / (ms * 1e-3) / 8e12, 4), "ms_mean_med": round(ms, 3),
                          "power_W": [x["power"] for x in v], "gfxclk_MHz": [x["gfxclk"] for x in v],
                          "ppt_residency": [round(x["ppt"], 3) if x["ppt"] is not None else None for x in v],
                          "ms_max": [round(x["ms_max"], 3) for x in v]}), flush=True)


if __name__ == "__main__":
    main()

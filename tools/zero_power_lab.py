#!/usr/bin/env python3
"""Diagnostic (round 3, config 3): does the zero-prefix data change the GPU's
power, clocks or throttling?  Runs config-3-shaped streams (and config 2 /
d1 c4 as controls) back to back for a few seconds per segment through two
builds of the product library -- `base` and `zconst` (zero-prefix pieces
store 0x5A5A5A5A: same instructions, other data; tools/variant_lab.py) --
and reads the amdsmi GPU metrics / violation accumulators around each
segment, polling clocks, power and temperatures in between.

    LAB_VARIANTS="base=;zconst=-DS3DG_DIAG_ZERO=1" python tools/variant_lab.py --build-only   # here
    python tools/zero_power_lab.py                                                          # GPU box
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, sys, threading, time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import variant_lab  # noqa: E402  (library paths only)

MiB = 1 << 20
POINTS = {"cfg3": (4, 1, 2), "cfg2": (1, 0, 1), "d1c4": (1, 3, 4), "cfg5": (2, 2, 3), "d1c3": (1, 2, 3),
          "d1c2": (1, 1, 2), "d4c1": (4, 0, 1), "d2c15": (2, 1, 3), "d1c8": (1, 7, 8), "d1c15": (1, 1, 3)}


def points():
    """LAB_POINTS="cfg3,cfg2,cfg3@28,cfg5@0%100": name[@batch workgroups per CU
    cap][%batch store floor in wall-clock ticks]; omitted = library default."""
    out = []
    for item in os.environ.get("LAB_POINTS", "cfg3,cfg2,d1c4").split(","):
        head, _, pace = item.partition("%")
        name, _, occ = head.partition("@")
        out.append((item, name, int(occ) if occ else -1, int(pace) if pace else -1))
    return out


def smi_handle():
    import amdsmi
    import torch
    amdsmi.amdsmi_init()
    want = None
    try:
        p = torch.cuda.get_device_properties(0)
        want = (getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
    except Exception:
        pass
    hs = amdsmi.amdsmi_get_processor_handles()
    for h in hs:
        try:
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)   # "dddd:bb:dd.f"
            dom, bus, rest = bdf.split(":")
            if want and int(bus, 16) == want[1] and int(rest.split(".")[0], 16) == want[2]:
                return amdsmi, h, bdf
        except Exception:
            continue
    return amdsmi, hs[0], "first-of-%d" % len(hs)


def metrics(smi, h):
    m = smi.amdsmi_get_gpu_metrics_info(h)
    try:
        v = smi.amdsmi_get_violation_status(h)
    except Exception:
        v = {}
    return m, v


def num(x):
    return x if isinstance(x, (int, float)) else None


def main():
    import torch
    n = int(os.environ.get("LAB_N", "10000"))
    seg_s = float(os.environ.get("LAB_SEG_S", "2.5"))
    reps = int(os.environ.get("LAB_REPS", "3"))
    names = [v for v in os.environ.get("LAB_NAMES", "base,zconst").split(",")]
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    libs = {}
    for name in names:
        L = ctypes.CDLL(variant_lab.so(name), mode=os.RTLD_LOCAL)
        hd = ctypes.c_void_p()
        assert L.s3dg_ctx_create(0, ctypes.byref(hd)) == 0
        libs[name] = (L, hd)
    buf = torch.empty(8 * MiB * n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    p = ctypes.c_void_p(buf.data_ptr())
    smi, h, bdf = smi_handle()
    print(json.dumps({"smi_device": bdf}), flush=True)

    def launch(L, hd, point):
        name = point[1]
        if name == "k2":                               # npz keystream, 2 MiB chunks, one launch
            assert L.s3dg_xoshiro_fill(hd, p, u64(8 * MiB * n), u64(2 * MiB), u64(0), sh) == 0
            return
        if name in ("dg1", "dg1c2"):                   # DG1, one launch over the whole buffer
            d, fn, fd = (2, 1, 2) if name == "dg1c2" else (1, 0, 1)
            assert L.s3dg_dgen_fill(hd, p, u64(8 * MiB * n), u64(0), u64(1 << 40), u64(d), u32(fn), u32(fd),
                                    u64(777), sh) == 0
            return
        if name.startswith("f") and "x" in name:      # "f<f_num>x<f_den>": dedup 1, any compress
            d, (fn, fd) = 1, map(int, name[1:].split("x"))
        else:
            d, fn, fd = POINTS[name]
        r = L.s3dg_fill_controlled_stream(hd, p, u64(8 * MiB), u64(8 * MiB), u64(n), u64(d), u32(fn), u32(fd),
                                          u64(0x5EED000000000001), u64(0), sh)
        assert r == 0

    poll = {"on": False, "rows": []}

    def poller():
        while poll["on"]:
            try:
                m = smi.amdsmi_get_gpu_metrics_info(h)
                poll["rows"].append({k: m.get(k) for k in ("current_uclk", "current_gfxclk", "current_socket_power",
                                                           "temperature_hbm", "temperature_hotspot",
                                                           "temperature_mem", "average_umc_activity",
                                                           "throttle_status", "indep_throttle_status", "current_socclk",
                                                           "voltage_gfx", "voltage_soc", "voltage_mem")})
            except Exception as e:  # noqa: BLE001
                poll["rows"].append({"error": str(e)})
            time.sleep(0.05)

    for name, (L, hd) in libs.items():        # warm both builds
        launch(L, hd, ("cfg2", "cfg2", -1, -1))
    torch.cuda.synchronize()
    for rep in range(reps):
        for point in points():
            for name, (L, hd) in libs.items():
                assert L.s3dg_set_occupancy(hd, -1, point[2]) == 0
                if hasattr(L, "s3dg_set_batch_pace"):
                    assert L.s3dg_set_batch_pace(hd, point[3]) == 0
                m0, v0 = metrics(smi, h)
                poll["on"], poll["rows"] = True, []
                th = threading.Thread(target=poller)
                th.start()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record(st)
                k = 0
                while time.perf_counter() - t0 < seg_s:
                    for _ in range(8):
                        launch(L, hd, point)
                        k += 1
                    torch.cuda.synchronize()
                e1.record(st)
                torch.cuda.synchronize()
                poll["on"] = False
                th.join()
                m1, v1 = metrics(smi, h)
                dt = e0.elapsed_time(e1) * 1e-3
                out = {"rep": rep, "point": point[0], "variant": name, "launches": k,
                       "GBps": round(k * 8 * MiB * n / dt / 1e9, 1), "seconds": round(dt, 3)}
                e_a, e_b = num(m0.get("energy_accumulator")), num(m1.get("energy_accumulator"))
                c_a, c_b = num(m0.get("system_clock_counter")), num(m1.get("system_clock_counter"))
                out["energy_acc_delta"] = (e_b - e_a) if e_a is not None and e_b is not None else None
                out["sys_clock_delta"] = (c_b - c_a) if c_a is not None and c_b is not None else None
                for key in ("ppt_residency_acc", "socket_thm_residency_acc", "prochot_residency_acc",
                            "vr_thm_residency_acc", "accumulation_counter", "mem_activity_acc", "gfx_activity_acc"):
                    a, b = num(m0.get(key)), num(m1.get(key))
                    out[key + "_delta"] = (b - a) if a is not None and b is not None else None
                for key in ("acc_counter", "acc_ppt_pwr", "acc_socket_thrm", "acc_hbm_thrm", "acc_vr_thrm",
                            "acc_prochot_thrm", "acc_gfx_clk_below_host_limit"):
                    a, b = num(v0.get(key)), num(v1.get(key))
                    out["viol_" + key + "_delta"] = (b - a) if a is not None and b is not None else None
                rows = [r for r in poll["rows"] if "error" not in r]
                for key in ("current_uclk", "current_gfxclk", "current_socket_power", "temperature_hbm",
                            "temperature_hotspot", "temperature_mem", "average_umc_activity", "current_socclk",
                            "voltage_gfx", "voltage_soc", "voltage_mem"):
                    vals = [r[key] for r in rows if isinstance(r.get(key), (int, float))]
                    out[key + "_med"] = statistics.median(vals) if vals else None
                    out[key + "_max"] = max(vals) if vals else None
                out["throttle_status_set"] = sorted({str(r.get("throttle_status")) for r in rows})
                out["indep_throttle_status_set"] = sorted({str(r.get("indep_throttle_status")) for r in rows})[:6]
                out["poll_samples"] = len(rows)
                print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

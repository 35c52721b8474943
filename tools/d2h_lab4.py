#!/usr/bin/env python3
"""Diagnostic: D2H copy rate over time in one process (60 x 256 MiB copies,
each timed with HIP events on its stream) next to the GPU's PCIe DPM state
(/sys/class/drm/card*/device/pp_dpm_pcie and current_link_speed, read before,
during and after).  Tooling only."""
import ctypes, glob, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pcie_state():
    out = {}
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        st = {}
        for f in ("pp_dpm_pcie", "current_link_speed", "current_link_width", "pp_dpm_fclk"):
            try:
                st[f] = open(os.path.join(d, f)).read().strip().replace("\n", " | ")
            except Exception:
                pass
        if st:
            out[d] = st
    return out


def main():
    import torch
    import s3dlio_amd as S
    from s3dlio_amd._lib import call
    GiB, MiB = 1 << 30, 1 << 20
    ctx = S.Context(0)
    cb = 256 * MiB
    src = torch.empty(cb, dtype=torch.uint8, device="cuda")
    ctx.fill_controlled(src, cb, entropy=1)
    host = ctypes.c_void_p()
    call("s3dg_host_alloc_pinned_local", 0, cb, ctypes.byref(host))
    st = torch.cuda.Stream()
    print(json.dumps({"t": "before", "pcie": pcie_state()}), flush=True)
    t0 = time.perf_counter()
    rates = []
    for k in range(int(os.environ.get("LAB_COPIES", "60"))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        call("s3dg_d2h_async", ctx._h, host.value, src.data_ptr(), cb, int(st.cuda_stream))
        e1.record(st)
        torch.cuda.synchronize()
        rates.append(round(cb / (e0.elapsed_time(e1) * 1e-3) / GiB, 1))
        if k in (2, 30):
            print(json.dumps({"t": f"after copy {k}", "pcie": pcie_state()}), flush=True)
    print(json.dumps({"rates_GiBps": rates, "seconds": round(time.perf_counter() - t0, 2)}), flush=True)
    time.sleep(2)
    print(json.dumps({"t": "idle 2 s", "pcie": pcie_state()}), flush=True)
    call("s3dg_host_free_pinned", host.value)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Diagnostic: D2H copy rate vs the GPU's PCIe link state over time.

    python tools/pcie_lab.py          # GPU box

Copies 256 MiB device chunks into a pinned host ring (the bench's D2H sample
shape) in bursts separated by idle gaps, timing every copy with HIP events,
while a thread samples the link's sysfs state (current_link_speed /
current_link_width of the GPU's PCI function and of its upstream bridges, and
the driver's pp_dpm_pcie level, when readable) every LAB_POLL_MS.  Prints one
JSON line per burst: copy rates in order, and the link states seen during it.
Tooling only: nothing in the product imports this."""
import ctypes, json, os, sys, threading, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MiB, GiB = 1 << 20, 1 << 30


def pci_paths(bdf):
    """The GPU function's sysfs dir and its upstream bridges (nearest first)."""
    dev = os.path.realpath(f"/sys/bus/pci/devices/{bdf}")
    out, p = [], dev
    while os.path.basename(p).count(":") == 2:
        out.append(p)
        p = os.path.dirname(p)
    return out


def peers_below(paths):
    """For each bridge above the GPU: the other AMD GPUs (class 0x03xxxx or
    0x12xxxx, vendor 0x1002, function 0) below it, i.e. sharing its uplink."""
    gpus = []
    for d in os.listdir("/sys/bus/pci/devices"):
        cls, ven = read(f"/sys/bus/pci/devices/{d}/class"), read(f"/sys/bus/pci/devices/{d}/vendor")
        if ven == "0x1002" and cls and cls[:4] in ("0x03", "0x12") and d.endswith(".0"):
            gpus.append(os.path.realpath(f"/sys/bus/pci/devices/{d}"))
    me = paths[0] if paths else None
    return {os.path.basename(b): sorted(os.path.basename(g) for g in gpus if g != me and g.startswith(b + "/"))
            for b in paths[1:]}


def read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def link_state(paths):
    st = {}
    for i, p in enumerate(paths[:4]):
        sp, wd = read(p + "/current_link_speed"), read(p + "/current_link_width")
        if sp is not None:
            st[f"l{i}"] = f"{sp} x{wd}"
    dpm = read(paths[0] + "/pp_dpm_pcie") if paths else None
    if dpm:
        cur = [ln for ln in dpm.splitlines() if ln.rstrip().endswith("*")]
        st["dpm"] = cur[0] if cur else dpm.replace("\n", " | ")
    return st


def main():
    import torch
    from s3dlio_amd import Context
    from s3dlio_amd._lib import call
    dev = 0
    ctx = Context(dev)
    props = torch.cuda.get_device_properties(dev)
    bdf = "%04x:%02x:%02x.0" % (getattr(props, "pci_domain_id", 0), props.pci_bus_id, props.pci_device_id)
    paths = pci_paths(bdf)
    print(json.dumps({"bdf": bdf, "paths": paths, "max": [read(p + "/max_link_speed") for p in paths[:4]],
                      "dpm_levels": read(paths[0] + "/pp_dpm_pcie") if paths else None,
                      "gpus_sharing_bridge": peers_below(paths)}), flush=True)
    cb = 256 * MiB
    src = torch.empty(cb, dtype=torch.uint8, device=f"cuda:{dev}")
    src.fill_(7)
    host = []
    for _ in range(2):
        p = ctypes.c_void_p()
        call("s3dg_host_alloc_pinned_local", dev, cb, ctypes.byref(p))
        host.append(p.value)
    cpy = torch.cuda.Stream(device=dev)
    poll = float(os.environ.get("LAB_POLL_MS", "5")) / 1e3
    samples, stop = [], threading.Event()

    def poller():
        while not stop.is_set():
            samples.append((time.perf_counter(), json.dumps(link_state(paths), sort_keys=True)))
            time.sleep(poll)
    th = threading.Thread(target=poller, daemon=True)
    th.start()
    try:
        for gap in [float(x) for x in os.environ.get("LAB_GAPS", "0,0.5,2,0,5,0").split(",")]:
            time.sleep(gap)
            n = int(os.environ.get("LAB_COPIES", "48"))
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
            t0 = time.perf_counter()
            for k in range(n):
                ev[k][0].record(cpy)
                call("s3dg_d2h_async", ctx._h, host[k & 1], int(src.data_ptr()), cb, int(cpy.cuda_stream))
                ev[k][1].record(cpy)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rates = [round(cb / (a.elapsed_time(b) * 1e-3) / GiB, 1) for a, b in ev]
            seen = {}
            for t, s in samples:
                if t0 - 0.05 <= t <= t1:
                    seen[s] = seen.get(s, 0) + 1
            before = [s for t, s in samples if t < t0][-1:] or [None]
            print(json.dumps({"gap_s": gap, "seconds": round(t1 - t0, 4), "GiBps": rates,
                              "link_before": before[0], "link_during": seen}), flush=True)
    finally:
        stop.set()
        th.join()
        torch.cuda.synchronize()
        for p in host:
            call("s3dg_host_free_pinned", p)


if __name__ == "__main__":
    main()

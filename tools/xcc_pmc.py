"""Per-XCC write-path counters of the fill and the keystream in ONE process
(VERDICT r05 next #1a).  Run under rocprofv3 with the per-XCC derived
counters of tools/xcc_counters.yaml:

    rocprofv3 -E tools/xcc_counters.yaml --pmc X0_TCC_EA0_WRREQ ... -- python3 tools/xcc_pmc.py

Launches, interleaved, through the product library (s3dlio_amd): the fill
as config 2 (10 000 x 8 MiB, one k_fill_batch launch), K2 as config 6 (the
same bytes as 2 MiB Xoshiro256++ chunks, one persistent k_keystream launch)
and DG1 c1 as config 14 (one 8 GiB object per launch).  LAB_ROUNDS rounds
(default 2).  Bytes are not checked here (the product's own tests do).

LAB_SMI=1 (no profiler): each kind LAB_REPS (default 10) times back to back,
HIP-event rate, and the amdsmi GFX clock / socket power polled every ~5 ms
over those launches: one JSON line per kind with GB/s, clock, power and the
write rate per GFX cycle (64-B requests per cycle per XCD)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MiB, GiB = 1 << 20, 1 << 30


def main():
    import torch
    from s3dlio_amd import Context, object_entropy
    from s3dlio_amd._lib import call
    dev = 0
    torch.cuda.set_device(dev)
    ctx = Context(dev, base_seed=0xBA5EB10C00000000)
    n, size = 10000, 8 * MiB
    ring = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    p = int(ring.data_ptr())
    sh = int(torch.cuda.current_stream().cuda_stream)
    sb = 0x5EED000000000001

    def fill():
        call("s3dg_fill_controlled_stream", ctx._h, p, size, size, n, 1, 0, 1, sb, 0, sh)

    def k2():
        call("s3dg_xoshiro_fill", ctx._h, p, n * size, 2 * MiB, 0, sh)

    def dg1():
        for j in range(2):
            call("s3dg_dgen_fill", ctx._h, p + j * 8 * GiB, 8 * GiB, 0, 1 << 40, 1, 0, 1,
                 object_entropy(sb, j), sh)
    if os.environ.get("LAB_KIND") == "cfg5":
        # config 5's launch shape (d2 c3) with the store floor forced to
        # LAB_PACE ticks (0: plain): LAB_N launches, to compare the counters
        # of the slow launches (12.1-12.8 ms) with the fast ones (11.0-11.3)
        ctx.set_batch_pace(int(os.environ.get("LAB_PACE", "0")))
        for k in range(int(os.environ.get("LAB_N", "16"))):
            call("s3dg_fill_controlled_stream", ctx._h, p, size, size, n, 2, 2, 3, sb, 0, sh)
            torch.cuda.synchronize()
        print("xcc_pmc ok", flush=True)
        return
    if os.environ.get("LAB_SMI") == "1":
        return smi_mode(torch, {"fill": (fill, n * size), "k2": (k2, n * size), "dg1": (dg1, 16 * GiB)})
    for r in range(int(os.environ.get("LAB_ROUNDS", "2"))):
        for name, f in (("fill", fill), ("k2", k2), ("dg1", dg1)):
            f()
            torch.cuda.synchronize()
            print(f"round {r} {name} done", flush=True)
    print("xcc_pmc ok", flush=True)


def smi_mode(torch, kinds):
    import json
    import threading
    import time
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from zero_power_lab import smi_handle
    smi, sm, bdf = smi_handle()
    rows, on = [], [True]

    def poller():
        while on[0]:
            try:
                m = smi.amdsmi_get_gpu_metrics_info(sm)
                rows.append((time.perf_counter(), m.get("current_gfxclk"), m.get("current_socket_power")))
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.005)
    th = threading.Thread(target=poller, daemon=True)
    th.start()
    reps = int(os.environ.get("LAB_REPS", "10"))
    st = torch.cuda.current_stream()
    for rnd in range(int(os.environ.get("LAB_ROUNDS", "2"))):
        for name, (f, nbytes) in kinds.items():
            f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(st)
            for _ in range(reps):
                f()
            e1.record(st)
            e1.synchronize()
            t1 = time.perf_counter()
            ms = e0.elapsed_time(e1) / reps
            sel = [r for r in rows if t0 + 0.2 * (t1 - t0) <= r[0] <= t1]
            clk = sum(r[1] for r in sel if r[1]) / max(1, sum(1 for r in sel if r[1]))
            pw = sum(r[2] for r in sel if r[2]) / max(1, sum(1 for r in sel if r[2]))
            gbs = nbytes / (ms * 1e6)
            print(json.dumps({"round": rnd, "kind": name, "GBps": round(gbs, 1), "gfxclk_MHz": round(clk, 1),
                              "socket_W": round(pw, 1), "samples": len(sel),
                              "wrreq_per_cycle_per_xcd": round(gbs * 1e9 / 64 / 8 / (clk * 1e6), 3) if clk else None}),
                  flush=True)
    on[0] = False
    th.join()
    print("xcc_pmc ok", flush=True)


if __name__ == "__main__":
    main()

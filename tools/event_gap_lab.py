#!/usr/bin/env python3
"""Do HIP events between launches cost time? (tooling)  10 x 8 GiB DG1 /
K2 launches back to back, timed (a) with two events around all of them and
(b) with an event pair around every launch, as bench.py records them.
Nothing in the product imports this."""
import json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GiB, MiB = 1 << 30, 1 << 20


def main():
    import torch
    from s3dlio_amd import Context, object_entropy
    from s3dlio_amd._lib import call
    ctx = Context(0)
    st = torch.cuda.current_stream()
    sh = int(st.cuda_stream)
    n = 10
    buf = torch.empty(n * 8 * GiB, dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    kinds = {
        "dg1c1_bench_seeds": lambda t: call("s3dg_dgen_fill", ctx._h, base + t * 8 * GiB, 8 * GiB, 0, 1 << 40, 1, 0, 1,
                                            object_entropy(0x5EED000000000001, t), sh),
        "dg1c1_small_seeds": lambda t: call("s3dg_dgen_fill", ctx._h, base + t * 8 * GiB, 8 * GiB, 0, 1 << 40, 1, 0, 1,
                                            777 + t, sh),
        "k2": lambda t: call("s3dg_xoshiro_fill", ctx._h, base + t * 8 * GiB, 8 * GiB, 2 * MiB, t * 4096, sh),
    }
    res = {}
    for rep in range(3):
        for k, f in kinds.items():
            for mode in ("outer", "per_launch"):
                for t in range(n):
                    f(t)
                torch.cuda.synchronize()
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for t in range(n):
                    if mode == "per_launch":
                        evs[2 * t].record(st)
                    f(t)
                    if mode == "per_launch":
                        evs[2 * t + 1].record(st)
                e1.record(st)
                torch.cuda.synchronize()
                tot = e0.elapsed_time(e1)
                r = res.setdefault((k, mode), {"GBps": [], "sum_launch_ms": []})
                r["GBps"].append(n * 8 * GiB / (tot * 1e-3) / 1e9)
                if mode == "per_launch":
                    r["sum_launch_ms"].append(sum(evs[2 * t].elapsed_time(evs[2 * t + 1]) for t in range(n)))
        print(f"rep {rep} done", flush=True)
    for (k, mode), r in res.items():
        print(json.dumps({"kind": k, "events": mode, "GBps_median": round(statistics.median(r["GBps"]), 1),
                          "sum_launch_ms_median": round(statistics.median(r["sum_launch_ms"]), 3)
                          if r["sum_launch_ms"] else None}), flush=True)


if __name__ == "__main__":
    main()

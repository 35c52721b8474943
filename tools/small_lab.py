#!/usr/bin/env python3
"""Diagnostic: device time of small-object batches without the host
preparation.  Run under `rocprofv3 --kernel-trace`: before each timed batch
call the lab launches a one-element torch add as a marker, and
tools/small_lab_trace.py sums the batch kernels between markers.  Points
vary the batch launch knobs.  (A host-gated stream does not work here: the
batch call paces itself on its sub-batches' events, so it would wait on the
gate it is queued behind.)

    LAB_POINTS="size:waves:occ:pf:store:tile;..." rocprofv3 --kernel-trace ... -- python tools/small_lab.py
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ("20485:0:-1:-1:-1:0;20485:0:-1:-1:-1:1;20485:0:-1:-1:-1:8;20485:2:14:-1:3:1;20485:1:24:-1:-1:1;"
           "20485:1:-1:0:-1:1;20485:1:-1:64:-1:1;20485:2:-1:-1:-1:1;65536:0:-1:-1:-1:0;65536:0:-1:-1:-1:1")


def main():
    import torch
    from s3dlio_amd import Context
    from s3dlio_amd._lib import ObjDesc, call
    ctx = Context(0)
    GiB = 1 << 30
    buf = torch.empty(int(float(os.environ.get("LAB_GIB", "52")) * GiB), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sh = int(st.cuda_stream)
    marker = torch.zeros(1, device="cuda")
    arrs = {}
    res = {}
    pts = [tuple(int(x) for x in p.split(":")) for p in os.environ.get("LAB_POINTS", DEFAULT).split(";")]
    for rep in range(int(os.environ.get("LAB_REPS", "3"))):
        for p in pts:
            size, waves, occ, pf, sp, tile = p
            if size not in arrs:
                stride = (size + 4095) // 4096 * 4096
                n = min(buf.numel() // stride, 2500000)
                a = (ObjDesc * n)()
                for j in range(n):
                    a[j] = ObjDesc(j * stride, size, 0x5EED + (j << 32), 1, 0, 1)
                arrs[size] = (a, n)
            a, n = arrs[size]
            ctx.set_waves_per_block(waves)
            ctx.set_occupancy(occ, occ)
            ctx.set_batch_prefetch(pf if pf >= 0 else -1)
            ctx.set_store_policy(sp, sp)
            ctx.set_batch_tile(tile)
            call("s3dg_fill_controlled_batch", ctx._h, buf.data_ptr(), a, n, sh)     # warm
            torch.cuda.synchronize()
            marker.add_(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            call("s3dg_fill_controlled_batch", ctx._h, buf.data_ptr(), a, n, sh)
            e1.record(st)
            torch.cuda.synchronize()
            res.setdefault(p, []).append(size * n / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        print(f"rep {rep} done", flush=True)
    for p, v in res.items():
        print(json.dumps({"size": p[0], "waves": p[1], "occ": p[2], "pf": p[3], "store": p[4], "tile": p[5],
                          "GBps_events_median": round(statistics.median(v), 1), "max": round(max(v), 1)}), flush=True)


if __name__ == "__main__":
    main()

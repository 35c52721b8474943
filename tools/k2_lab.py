#!/usr/bin/env python3
"""Diagnostic: k_keystream launch-shape sweep on the product library (K2 npz
keystream and DG1 dgen mode), interleaved in one process.

    LAB_POINTS="16:4:0:2048;64:1:0:2048" python tools/k2_lab.py     # GPU box
Point = draws-per-stage : waves-per-workgroup : workgroups-per-CU cap : min draws per lane
        [: store policy (-1 default, 0 plain, 1 nt, 2 sc1)].
Tooling only: nothing in the product imports this."""
import json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ("16:4:0:2048;16:2:0:2048;16:1:0:2048;32:4:0:2048;32:2:0:2048;32:1:0:2048;"
           "64:4:0:2048;64:2:0:2048;64:1:0:2048;16:4:3:2048;16:4:2:2048;32:2:4:2048;"
           "64:1:3:2048;64:1:2:2048;16:4:0:4096;64:1:0:4096;64:1:0:1024;64:2:0:4096")


def main():
    import torch
    from s3dlio_amd import Context
    from s3dlio_amd._lib import call
    MiB, GiB = 1 << 20, 1 << 30
    n = int(float(os.environ.get("LAB_GIB", "40")) * GiB)
    ctx = Context(0)
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sh = int(st.cuda_stream)
    pts = [tuple(int(x) for x in p.split(":")) for p in os.environ.get("LAB_POINTS", DEFAULT).split(";")]
    pts = [p if len(p) == 5 else p + (-1,) for p in pts]

    def run(kind):
        if kind == "k2":
            call("s3dg_xoshiro_fill", ctx._h, buf.data_ptr(), n, 2 * MiB, 0, sh)
        elif kind == "dg1":   # DG1: one object, 1 MiB blocks, dedup 1, compress 2
            call("s3dg_dgen_fill", ctx._h, buf.data_ptr(), n, 0, 1 << 40, 1, 1, 2, 12345, sh)
        else:                 # DG1 at compress 1 (no zero prefix)
            call("s3dg_dgen_fill", ctx._h, buf.data_ptr(), n, 0, 1 << 40, 1, 0, 1, 12345, sh)
    res, occ = {}, {}
    for rep in range(int(os.environ.get("LAB_REPS", "3"))):
        for p in pts:
            ctx.set_keystream_shape(0, *p)
            ctx.set_keystream_shape(1, *p)
            occ[p] = ctx.query_keystream_occupancy(0)
            for kind in os.environ.get("LAB_K2KINDS", "k2,dg1").split(","):
                run(kind)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st); run(kind); e1.record(st); torch.cuda.synchronize()
                res.setdefault((p, kind), []).append(n / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        print(f"rep {rep} done", flush=True)
    for (p, kind), v in res.items():
        print(json.dumps({"kind": kind, "draws": p[0], "waves": p[1], "cap": p[2], "min_draws": p[3], "store": p[4],
                          "wgs_per_cu": occ[p], "GBps_median": round(statistics.median(v), 1),
                          "max": round(max(v), 1)}), flush=True)


if __name__ == "__main__":
    main()

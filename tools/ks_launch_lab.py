#!/usr/bin/env python3
"""k_keystream per-launch cost lab (tooling): the same 64 GiB of K2 / DG1 c1
bytes as launches of 1..64 GiB, and 8 GiB launches at several launch shapes.
A fixed cost per launch (ramp + tail) shows as t = a + b * bytes.

    KS_REPS=3 python tools/ks_launch_lab.py
Nothing in the product imports this."""
import json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GiB, MiB = 1 << 30, 1 << 20


def main():
    import torch
    from s3dlio_amd import Context
    from s3dlio_amd._lib import call
    ctx = Context(0)
    st = torch.cuda.current_stream()
    sh = int(st.cuda_stream)
    total = 64 * GiB
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    reps = int(os.environ.get("KS_REPS", "3"))

    def launches(mode, per):
        n = total // per
        if mode == 0:
            return lambda: [call("s3dg_xoshiro_fill", ctx._h, base + t * per, per, 2 * MiB, t * (per // (2 * MiB)), sh)
                            for t in range(n)]
        return lambda: [call("s3dg_dgen_fill", ctx._h, base + t * per, per, 0, 1 << 40, 1, 0, 1, 777 + t, sh)
                        for t in range(n)]

    W = {}
    sizes = [int(x) for x in os.environ.get("KS_SIZES", "1,2,4,8,16,64").split(",")]
    for mode, nm in ((0, "k2"), (1, "dg1c1")):
        for g in sizes:
            W[f"{nm}_{g}g"] = (launches(mode, g * GiB), None)
        # launch shapes at 8 GiB: (draws, waves, wgs_per_cu, min_lane_draws)
        for shp in ((64, 2, 0, 1024), (64, 1, 0, 1024), (64, 4, 0, 512), (32, 4, 0, 512), (64, 4, 0, 2048)):
            W[f"{nm}_8g_shape{shp}"] = (launches(mode, 8 * GiB), (mode, shp))
    res = {}
    for rep in range(reps):
        for k, (fn, shp) in W.items():
            if shp:
                ctx.set_keystream_shape(shp[0], *shp[1])
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            torch.cuda.synchronize()
            if shp:
                ctx.set_keystream_shape(shp[0])
            res.setdefault(k, []).append(total / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        print(f"rep {rep} done", flush=True)
    for k, r in res.items():
        print(json.dumps({"kind": k, "GBps_median": round(statistics.median(r), 1), "max": round(max(r), 1)}),
              flush=True)


if __name__ == "__main__":
    main()

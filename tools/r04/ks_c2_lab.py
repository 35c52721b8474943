#!/usr/bin/env python3
"""DG1 with a zero prefix (configs 15 / 17: d2 c2) under the launch shapes the
persistent grid makes possible: the default (4-wave workgroups, XCD groups of
32 waves, static grid), 4-wave persistent, and 1-wave workgroups static and
persistent with XCD groups of 16 or 32 waves.  One process, the product
library, shapes interleaved and rotated every round; GB/s of ten 8 GiB
launches (config 15) and of one 80 GiB launch (config 17).

    python tools/r04/ks_c2_lab.py      # GPU box
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
GiB = 1 << 30


def main():
    import torch
    import s3dlio_amd as S
    from s3dlio_amd._lib import call
    ctx = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    h = ctx._h
    st = torch.cuda.current_stream()
    sh = int(st.cuda_stream)
    buf = torch.empty(10 * 8 * GiB, dtype=torch.uint8, device="cuda")
    G8 = 8 * GiB
    # name: (waves, xcd group waves, persist rounds)
    shapes = {"w4_static(default)": (0, 0, -1), "w4_persist": (4, 32, 1),
              "w1_static_x16": (1, 16, 0), "w1_persist_x16": (1, 16, 1),
              "w1_static_x32": (1, 32, 0), "w1_persist_x32": (1, 32, 1)}
    seed = 0x5EED000000000001

    def setup(w, xg, pr):
        call("s3dg_set_keystream_shape", h, 1, 0, w, 0, 0, -1)
        call("s3dg_set_keystream_xcd_group", h, 1, xg)
        call("s3dg_set_keystream_persist", h, pr)

    def cfg15():
        for t in range(10):
            call("s3dg_dgen_fill", h, buf.data_ptr() + t * G8, G8, 0, 1 << 40, 2, 1, 2, seed + t, sh)

    def cfg17():
        call("s3dg_dgen_fill_stream", h, buf.data_ptr(), G8, G8, 10, 2, 1, 2, seed, 0, sh)

    res, digests = {}, {}
    names = list(shapes)
    reps = int(os.environ.get("LAB_REPS", "6"))
    for rep in range(reps):
        order = names[rep % len(names):] + names[:rep % len(names)]
        for pt, fn in (("cfg15", cfg15), ("cfg17", cfg17)):
            for name in order:
                setup(*shapes[name])
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                fn()
                fn()
                e1.record(st)
                torch.cuda.synchronize()
                res.setdefault((pt, name), []).append(2 * 10 * G8 / (e0.elapsed_time(e1) * 1e-3) / 1e9)
                if rep == 0:
                    digests.setdefault(pt, set()).add(int(buf[:: 1 << 20].to(torch.int64).sum().item()))
        print(f"rep {rep} done", flush=True)
    for pt in ("cfg15", "cfg17"):
        print(json.dumps({"point": pt, "outputs_identical": len(digests[pt]) == 1}), flush=True)
        for name in names:
            v = res[(pt, name)]
            print(json.dumps({"point": pt, "shape": name, "GBps_median": round(statistics.median(v), 1),
                              "min": round(min(v), 1), "max": round(max(v), 1)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Interleaved A/B sweep of the fill kernel knobs vs write-only ceilings, in
one process (cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per
variant with the median / min over rounds.

    python tools/sweep.py [--gib 16] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--dedup", type=int, default=1)
    ap.add_argument("--compress", type=int, default=1)
    a = ap.parse_args()
    import torch
    import s3dlio_amd as S
    size = 8 << 20
    n = int(a.gib * (1 << 30)) // size
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    ctx = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    st = torch.cuda.current_stream()

    variants = {}
    for nt in (True, False):
        for occ in (1, 2, 3, 4, 8):
            def f(nt=nt, occ=occ):
                ctx.set_nontemporal(nt); ctx.set_occupancy(occ)
                ctx.fill_stream(buf, obj_size=size, n_objs=n, dedup=a.dedup, compress=a.compress,
                                seed_base=1)
            variants[f"fill nt={int(nt)} wg/cu={occ}"] = f
            def g(nt=nt, occ=occ):
                ctx.set_nontemporal(nt); ctx.set_occupancy(occ)
                ctx.write_ceiling(buf)
            variants[f"ceiling nt={int(nt)} wg/cu={occ}"] = g
    variants["torch zero_"] = lambda: buf.zero_()
    variants["torch fill_(7)"] = lambda: buf.fill_(7)

    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, f in variants.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st); f(); e1.record(st)
            torch.cuda.synchronize()
            res[k].append(buf.numel() / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    for k, v in res.items():
        print(json.dumps({"variant": k, "GBps_median": round(statistics.median(v), 1),
                          "GBps_max": round(max(v), 1), "bytes": buf.numel()}))


if __name__ == "__main__":
    main()

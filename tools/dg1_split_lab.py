#!/usr/bin/env python3
"""DG1 with a zero prefix: one keystream launch vs the zero-prefix + tail
split (s3dg_set_dgen_zero_split), and the zero launch's occupancy cap and
store policy.  One context per setting, interleaved, order rotated per rep;
each sample one step of bench.py's configs 14/15 (ten 8 GiB objects, one
s3dg_dgen_fill each; dedup 1/2) or 16/17 (the ten in one
s3dg_dgen_fill_stream launch) at the given compress (default 1 for 14/16, 2
for 15/17), timed with HIP events; mean GB/s over the samples.

    python tools/dg1_split_lab.py          # GPU box
LAB_SETTINGS: "name=chunks/waves/occ/store/overlap[/xcd_group[/lane_draws[/tail]]];..." (default
below), LAB_POINTS: "cfg15@2;cfg17@2;cfg15@3" (@compress; cfg6:
config 6's K2 launch, 84 GB as 2 MiB Xoshiro256++ chunks), LAB_REPS (default 6).
Tooling only: nothing in the product imports this."""
import json, os, statistics, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GiB = 1 << 30
DEFAULT = ("one=0/-1/-1/-1/0;w1=-1/1/0/3/0;w4o4=-1/4/4/2/0;w4o8=-1/4/8/3/0;w4o4_ov=-1/4/4/2/1;"
           "w1_ov=-1/1/0/3/1;w1o14_ov=-1/1/14/3/1")


def main():
    import torch
    import s3dlio_amd as S
    sets = {}
    for item in os.environ.get("LAB_SETTINGS", DEFAULT).split(";"):
        name, _, spec = item.partition("=")
        f = [int(x) for x in spec.split("/")]
        ch, w, occ, st, ov = f[:5]
        c = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
        c.set_dgen_zero_split(ch, w, occ, st, ov)
        if len(f) > 5 and f[5]:          # DG1 keystream XCD group (waves) for the tails
            c.set_keystream_xcd_group(1, f[5])
        if len(f) > 6 and f[6]:          # DG1 keystream draws per lane (tails: lanes of a 64-lane wave)
            c.set_keystream_shape(1, 0, 0, 0, f[6], -1)
        if len(f) > 7:                   # one-object launches' half-lane tail blocks (s3dg_set_keystream_tail)
            c.set_keystream_tail(f[7])
        sets[name] = c
    pts = os.environ.get("LAB_POINTS", "cfg15@2;cfg17@2;cfg15@3;cfg17@3").split(";")
    reps = int(os.environ.get("LAB_REPS", "6"))
    buf = torch.empty(10 * 8 * GiB, dtype=torch.uint8, device="cuda")
    G8 = 8 * GiB

    def run(c, kind, comp):
        if kind == "cfg6":                                  # config 6: 10 000 x 8 MiB as 2 MiB keystream chunks
            c.xoshiro_fill(buf, 10000 * 8 * (1 << 20), 2 << 20, 0x5EED)
            return
        d = 2 if kind in ("cfg15", "cfg17") else 1          # configs 14 / 16: dedup 1
        if kind in ("cfg14", "cfg15"):                      # one launch per 8 GiB object
            for t in range(10):
                c.dgen_fill(buf[t * G8:(t + 1) * G8], G8, dedup=d, compress=comp, seed=0x5EED + t)
        else:                                               # the ten in one launch
            c.dgen_fill_stream(buf, G8, 10, dedup=d, compress=comp, seed_base=0x5EED)
    res, digest = {}, {}
    names = list(sets)
    for rep in range(reps):
        for p in pts:
            kind, _, comp = p.partition("@")
            comp = (tuple(int(x) for x in comp.split("/")) if "/" in comp
                    else int(comp or (1 if kind in ("cfg14", "cfg16") else 2)))
            order = names[rep % len(names):] + names[:rep % len(names)]
            if rep % 2:
                order.reverse()
            for n in order:
                run(sets[n], kind, comp)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(sets[n], kind, comp)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((n, p), []).append(e0.elapsed_time(e1))
                if rep == 0:
                    digest.setdefault(p, {})[n] = int(buf[::4099].to(torch.int64).sum().item())
        print(f"rep {rep} done", flush=True)
    for p in pts:
        print(json.dumps({"point": p, "outputs_identical": len(set(digest[p].values())) == 1}), flush=True)
        for n in names:
            ms = res[(n, p)]
            mean = sum(ms) / len(ms)
            nb = 10000 * 8 * (1 << 20) if p.startswith("cfg6") else 80 * GiB
            print(json.dumps({"setting": n, "point": p, "GBps_mean": round(nb / (mean * 1e-3) / 1e9, 1),
                              "frac": round(nb / (mean * 1e-3) / 8e12, 4),
                              "ms_mean": round(mean, 3), "ms_min": round(min(ms), 3),
                              "ms_median": round(statistics.median(ms), 3), "n": len(ms)}), flush=True)


if __name__ == "__main__":
    main()

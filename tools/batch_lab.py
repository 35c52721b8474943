#!/usr/bin/env python3
"""Diagnostic: fill-kernel launch-shape study on the product library.
Sweeps the runtime knobs (waves per block, resident-workgroup cap per CU,
batch tile-record prefetch distance, store cache policy) over cfg4 (log-uniform sizes, batch),
cfg7 (uniform 8 MiB, batch) and cfg2 (uniform 8 MiB, stream), interleaved in
one process, and prints GB/s per point.

    python tools/batch_lab.py            # on the GPU box
Tooling only: nothing in the product imports this."""
import ctypes, itertools, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def points():
    spec = os.environ.get("LAB_POINTS")
    if spec:     # "kind:waves:occ:pf[:store[:tile]];..."  store: -1 default, 0 plain, 1 nt, 2 sc1
        for p in spec.split(";"):
            k, w, o, f, *rest = p.split(":")
            rest = [int(x) for x in rest] + [-1, 0][len(rest):]
            yield k, int(w), int(o), int(f), rest[0], rest[1]
        return
    for w, o, f in itertools.product([1], [0, 28, 24, 20, 16], [0, 128]):
        for k in ("cfg4", "cfg7"):
            yield k, w, o, f, -1, 0
    for w, o in [(2, 0), (2, 14), (2, 12)]:
        for k in ("cfg4", "cfg7"):
            yield k, w, o, 0, -1, 0
    for w, o in [(2, 0), (2, 14), (2, 12), (1, 0), (1, 24), (1, 20), (1, 16)]:
        yield "stream2", w, o, 0, -1, 0


def main():
    import torch
    from bench import log_uniform_sizes, SEED_BASE
    from s3dlio_amd import Context
    from s3dlio_amd._lib import ObjDesc, call
    MiB = 1 << 20
    n = int(os.environ.get("LAB_N", "10000"))
    bs = os.environ.get("LAB_BASE_SEED")      # e.g. bench.py's 0xBA5EB10C00000000
    ctx = Context(0, base_seed=int(bs, 0)) if bs else Context(0)
    pts = list(points())

    def table(sizes, d, fn, fd, align=4096):
        arr = (ObjDesc * len(sizes))()
        off = 0
        for j, sz in enumerate(sizes):
            arr[j] = ObjDesc(off, sz, SEED_BASE + (j << 32), d, fn, fd)
            off += (sz + align - 1) // align * align
        return arr, off, sum(sizes)
    descs = {}
    for name, sizes, d, fn, fd in [("cfg4", log_uniform_sizes(n), 2, 1, 3),
                                   # cfg4 sizes rounded up to whole 64-block tiles: no dead slots
                                   ("cfg4r", [(s + (1 << 18) - 1) >> 18 << 18 for s in log_uniform_sizes(n)], 2, 1, 3),
                                   ("cfg7", [8 * MiB] * n, 1, 0, 1),
                                   ("small", log_uniform_sizes(10 * n, 5, 4096, MiB), 1, 0, 1),
                                   ("mid", [MiB + 123] * (5 * n), 3, 2, 3),
                                   ("kb64", [64 << 10] * (10 * n), 1, 0, 1),
                                   ("kb20", [(20 << 10) + 5] * (20 * n), 1, 0, 1)]:
        descs[name] = table(sizes, d, fn, fd)
    # generic uniform batches: "u<size>x<dedup>x<f_num>x<f_den>[x<align>]", ~52 GB each
    for k in {p[0] for p in pts if p[0].startswith("u")}:
        sz, d, fn, fd, *al = (int(x) for x in k[1:].split("x"))
        al = al[0] if al else 4096
        descs[k] = table([sz] * min(5 * n * MiB // sz, 52 * 10**9 // ((sz + al - 1) // al * al)), d, fn, fd, al)
    # generic uniform streams: "s<size>x<dedup>x<f_num>x<f_den>[x<align>]" (k_fill_stream);
    # "t<size>x..." the same through the tiled path (s3dg_set_stream_tiles 1, as bench.py)
    for k in {p[0] for p in pts if p[0][:1] in ("s", "t") and p[0][1:2].isdigit()}:
        sz, d, fn, fd, *al = (int(x) for x in k[1:].split("x"))
        al = al[0] if al else 4096
        stride = (sz + al - 1) // al * al
        cnt = min(5 * n * MiB // sz, 52 * 10**9 // stride)
        descs[k] = (("gs", sz, stride, cnt, d, fn, fd), stride * cnt, sz * cnt)
    descs["stream2"] = (None, 8 * MiB * n, 8 * MiB * n)
    descs["stream3"] = ("s3", 8 * MiB * n, 8 * MiB * n)        # cfg3: dedup 4, compress 2
    descs["stream5"] = ("s5", 8 * MiB * n, 8 * MiB * n)        # cfg5: dedup 2, compress 3
    descs["stream2t"], descs["stream3t"], descs["stream5t"] = descs["stream2"], descs["stream3"], descs["stream5"]
    descs["ceiling"] = ("c", 8 * MiB * n, 8 * MiB * n)         # store-only kernel, fill shapes
    dst_off = int(os.environ.get("LAB_DST_OFF", "0"))      # generic s/u kinds: destination offset
    buf = torch.empty(max(v[1] for v in descs.values()) + dst_off, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sh = int(st.cuda_stream)

    def run(name):
        arr = descs[name][0]
        name = name.rstrip("t") if name.startswith("stream") else name
        if name == "ceiling":
            call("s3dg_write_ceiling", ctx._h, buf.data_ptr(), 8 * MiB * n, 0xA5A5A5A5, sh)
            return
        if isinstance(arr, tuple):
            _, sz, stride, cnt, d, fn, fd = arr
            call("s3dg_fill_controlled_stream", ctx._h, buf.data_ptr() + dst_off, sz, stride, cnt, d, fn, fd,
                 SEED_BASE, 0, sh)
            return
        if arr is None or arr in ("s3", "s5"):
            d, fn, fd = {None: (1, 0, 1), "s3": (4, 1, 2), "s5": (2, 2, 3)}[arr]
            call("s3dg_fill_controlled_stream", ctx._h, buf.data_ptr(), 8 * MiB, 8 * MiB, n, d, fn, fd,
                 SEED_BASE, 0, sh)
        else:
            call("s3dg_fill_controlled_batch", ctx._h, buf.data_ptr() + dst_off, arr, len(arr), sh)

    res, occ = {}, {}
    for rep in range(int(os.environ.get("LAB_REPS", "3"))):
        for p in pts:
            k, w, o, f, sp, _ = p
            ctx.set_store_policy(sp, sp)
            ctx.set_waves_per_block(w)
            ctx.set_occupancy(o, o)
            ctx.set_batch_prefetch(f)
            ctx.set_batch_tile(p[5])
            ctx.set_stream_tiles(1 if k in ("stream2t", "stream3t", "stream5t") or k[:1] == "t" else 0)
            occ[p] = ctx.query_occupancy(batch=not k.startswith(("stream", "ceiling")) and not k[1:2].isdigit()
                                         or k.startswith("u"))
            run(k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st); run(k); e1.record(st); torch.cuda.synchronize()
            res.setdefault(p, []).append(descs[k][2] / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        print(f"rep {rep} done", flush=True)
    for p, v in res.items():
        k, w, o, f, sp, tb = p
        print(json.dumps({"cfg": k, "waves": w, "occ_cap": o, "wgs_per_cu": occ[p], "pf": f, "store": sp, "tile": tb,
                          "GBps_median": round(statistics.median(v), 1), "max": round(max(v), 1)}), flush=True)


if __name__ == "__main__":
    main()

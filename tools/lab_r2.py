#!/usr/bin/env python3
"""Diagnostic lab (round 2): named workloads on the product library, each timed
with HIP events on the launch stream (device time) and perf_counter around the
call alone (host enqueue time), so small-object and secondary-kernel costs can
be split into host preparation and device work.  Runs unchanged under
`rocprofv3 --kernel-trace --stats` and `--pmc` passes.

    LAB_KINDS="s64k,b64k,b20k,cfg2,ceil_tiled,crc,dg1c1,dg1c2,k2,one1m" python tools/lab_r2.py
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MiB, GiB = 1 << 20, 1 << 30
SEED = 0x5EED000000000001


def main():
    import torch
    from s3dlio_amd import Context
    from s3dlio_amd._lib import ObjDesc, call
    ctx = Context(0)
    st = torch.cuda.current_stream()
    sh = int(st.cuda_stream)
    kinds = os.environ.get("LAB_KINDS", "s64k,b64k,b20k,cfg2,ceil_tiled,crc,dg1c1,dg1c2,k2,one1m,one4m,one16m")
    kinds = [k for k in kinds.split(",") if k]
    reps = int(os.environ.get("LAB_REPS", "3"))
    buf = torch.empty(int(float(os.environ.get("LAB_GIB", "80")) * GiB), dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    cap = buf.numel()

    def batch(sizes, d, fn, fd):
        arr = (ObjDesc * len(sizes))()
        off = 0
        for j, sz in enumerate(sizes):
            arr[j] = ObjDesc(off, sz, SEED + (j << 32), d, fn, fd)
            off += (sz + 4095) // 4096 * 4096
        assert off <= cap
        return arr

    W = {}
    n64 = min(1000000, cap // (64 << 10))
    W["s64k"] = (lambda: call("s3dg_fill_controlled_stream", ctx._h, base, 64 << 10, 64 << 10, n64, 1, 0, 1,
                              SEED, 0, sh), n64 * (64 << 10), 1)
    a64 = None
    if any(k.startswith("b64k") for k in kinds):
        a64 = batch([64 << 10] * n64, 1, 0, 1)
        W["b64k"] = (lambda: call("s3dg_fill_controlled_batch", ctx._h, base, a64, n64, sh), n64 * (64 << 10), 1)
    if any(k.startswith("b20k") for k in kinds):
        sz = (20 << 10) + 5
        n20 = min(2000000, cap // (24 << 10))
        a20 = batch([sz] * n20, 1, 0, 1)
        W["b20k"] = (lambda a20=a20, n20=n20: call("s3dg_fill_controlled_batch", ctx._h, base, a20, n20, sh),
                     n20 * sz, 1)
    if "s20k" in kinds:
        sz = (20 << 10) + 5
        n20 = min(2000000, cap // (24 << 10))
        W["s20k"] = (lambda sz=sz, n20=n20: call("s3dg_fill_controlled_stream", ctx._h, base, sz, 24 << 10, n20,
                                                 1, 0, 1, SEED, 0, sh), n20 * sz, 1)
    n8 = min(10000, cap // (8 * MiB))
    W["cfg2"] = (lambda: call("s3dg_fill_controlled_stream", ctx._h, base, 8 * MiB, 8 * MiB, n8, 1, 0, 1,
                              SEED, 0, sh), n8 * 8 * MiB, 1)
    W["cfg3"] = (lambda: call("s3dg_fill_controlled_stream", ctx._h, base, 8 * MiB, 8 * MiB, n8, 4, 1, 2,
                              SEED, 0, sh), n8 * 8 * MiB, 1)
    cb = n8 * 8 * MiB
    W["ceil_tiled"] = (lambda: call("s3dg_write_ceiling_tiled", ctx._h, base, cb, 0xA5A5A5A5, sh), cb, 1)
    W["ceil"] = (lambda: call("s3dg_write_ceiling", ctx._h, base, cb, 0xA5A5A5A5, sh), cb, 1)
    W["ceil_fill"] = (lambda: call("s3dg_write_ceiling_fill", ctx._h, base, cb, 0, sh), cb, 1)
    for pace in (1, 2, 3, 4, 6, 8, 12, 16):
        W[f"ceil_fill_p{pace}"] = (lambda pace=pace: call("s3dg_write_ceiling_fill", ctx._h, base, cb, pace, sh), cb, 1)
    crc_n = min(16 * GiB, cap)
    out = ctypes.c_uint32()
    if any(k.startswith("crcr") for k in kinds):   # CRC over random bytes (the keystream)
        call("s3dg_xoshiro_fill", ctx._h, base, crc_n, 2 * MiB, 99, sh)
        torch.cuda.synchronize()
        W["crcr"] = (lambda: call("s3dg_crc32", ctx._h, base, crc_n, sh, ctypes.byref(out)), crc_n, 1)
    W["crc"] = (lambda: call("s3dg_crc32", ctx._h, base, crc_n, sh, ctypes.byref(out)), crc_n, 1)
    dn = min(40 * GiB, cap)
    W["dg1c1"] = (lambda: call("s3dg_dgen_fill", ctx._h, base, dn, 0, 1 << 40, 1, 0, 1, 12345, sh), dn, 1)
    W["dg1c2"] = (lambda: call("s3dg_dgen_fill", ctx._h, base, dn, 0, 1 << 40, 2, 1, 2, 12345, sh), dn, 1)
    W["k2"] = (lambda: call("s3dg_xoshiro_fill", ctx._h, base, dn, 2 * MiB, 0, sh), dn, 1)
    # launch size: the same bytes as 8 GiB launches (bench configs 14/15) or one launch
    nbig = cap // (8 * GiB)
    for nm, d_, fn_, fd_ in (("dg1c1", 1, 0, 1), ("dg1c2", 2, 1, 2)):
        W[nm + "_8g"] = (lambda d_=d_, fn_=fn_, fd_=fd_: [call("s3dg_dgen_fill", ctx._h, base + t * 8 * GiB, 8 * GiB,
                                                               0, 1 << 40, d_, fn_, fd_, 12345 + t, sh)
                                                          for t in range(nbig)], nbig * 8 * GiB, 1)
        W[nm + "_all"] = (lambda d_=d_, fn_=fn_, fd_=fd_: call("s3dg_dgen_fill", ctx._h, base, nbig * 8 * GiB, 0,
                                                               1 << 40, d_, fn_, fd_, 12345, sh), nbig * 8 * GiB, 1)
    W["k2_8g"] = (lambda: [call("s3dg_xoshiro_fill", ctx._h, base + t * 8 * GiB, 8 * GiB, 2 * MiB, t * 4096, sh)
                           for t in range(nbig)], nbig * 8 * GiB, 1)
    W["k2_all"] = (lambda: call("s3dg_xoshiro_fill", ctx._h, base, nbig * 8 * GiB, 2 * MiB, 0, sh),
                   nbig * 8 * GiB, 1)
    # the reference's criterion shape (benches/performance_microbenchmarks.rs:43-64): one
    # fill_controlled_data call on one buffer, back to back
    for nm, sz in (("one1m", MiB), ("one4m", 4 * MiB), ("one16m", 16 * MiB)):
        W[nm] = (lambda sz=sz: call("s3dg_fill_controlled", ctx._h, base, sz, 1, 0, 1, 7, sh), sz, 200)

    # the floor of a back-to-back 1 MiB launch: a store-only kernel and hipMemsetD32Async
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    W["memset1m"] = (lambda: hip.hipMemsetD32Async(base, 0x5A5A5A5A, MiB // 4, sh), MiB, 200)
    W["ceil1m"] = (lambda: call("s3dg_write_ceiling", ctx._h, base, MiB, 0xA5A5A5A5, sh), MiB, 200)

    # "<kind>@<tile>": the same workload with s3dg_set_batch_tile(tile) (1 = dense)
    for k in list(kinds):
        if "@" in k:
            kk, tile = k.split("@")
            fn0, nb0, inner0 = W[kk]
            W[k] = ((lambda fn0=fn0, tile=int(tile): (ctx.set_batch_tile(tile), fn0(), ctx.set_batch_tile(0))),
                    nb0, inner0)
    res = {}
    for rep in range(reps):
        for k in kinds:
            fn, nbytes, inner = W[k]
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            t0 = time.perf_counter()
            for _ in range(inner):
                fn()
            th = time.perf_counter() - t0
            e1.record(st)
            torch.cuda.synchronize()
            tw = time.perf_counter() - t0
            r = res.setdefault(k, {"dev": [], "host": [], "wall": []})
            r["dev"].append(nbytes * inner / (e0.elapsed_time(e1) * 1e-3) / 1e9)
            r["host"].append(th / inner * 1e3)
            r["wall"].append(nbytes * inner / tw / 1e9)
        print(f"rep {rep} done", flush=True)
    for k, r in res.items():
        print(json.dumps({"kind": k, "bytes": W[k][1], "calls": W[k][2],
                          "GBps_dev_median": round(statistics.median(r["dev"]), 1),
                          "GBps_dev_max": round(max(r["dev"]), 1),
                          "host_ms_per_call_median": round(statistics.median(r["host"]), 3),
                          "GBps_wall_median": round(statistics.median(r["wall"]), 1)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Device CRC-32 rate on random (keystream) and constant buffers, for the
kernel chosen by S3DG_CRC_KERNEL (0 = conflict-free single-bank tables,
default; 1 = round-2 k_crc32_regions).  HIP events around s3dg_crc32 (the
kernel plus its small region-result copy and host fold).  Tooling only."""
import ctypes, json, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import s3dlio_amd as S
    from s3dlio_amd._lib import call, c_u32
    GiB = 1 << 30
    n = int(float(os.environ.get("CRC_GIB", "16")) * GiB)
    ctx = S.Context(0)
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    for kind in ("random", "constant"):
        if kind == "random":
            ctx.xoshiro_fill(buf, n, 2 << 20, seed_base=11)
        else:
            buf.fill_(0x5A)
        torch.cuda.synchronize()
        vals, rates = set(), []
        for rep in range(6):
            v = c_u32()
            t = time.perf_counter()
            call("s3dg_crc32", ctx._h, buf.data_ptr(), n, 0, ctypes.byref(v))
            dt = time.perf_counter() - t
            vals.add(v.value)
            if rep:
                rates.append(n / dt / 1e9)
        out[kind] = {"GBps_median": round(statistics.median(rates), 1), "max": round(max(rates), 1),
                     "crc": sorted(vals)}
    print(json.dumps({"kernel": os.environ.get("S3DG_CRC_KERNEL", "0"), "GiB": n / GiB, **out}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Throughput of the secondary surfaces (not the headline metric):
host-buffer drop-ins (generate + D2H), streaming Generator, NPZ build, device CRC.
Prints one JSON line per measurement."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(f, reps=3):
    f()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter(); f(); best = min(best, time.perf_counter() - t)
    return best


def main():
    import numpy as np
    import torch
    import s3dlio_amd as S
    GiB, MiB = 1 << 30, 1 << 20
    out = []
    # host-buffer drop-ins (pageable numpy buffer / pinned torch buffer)
    for label, size in [("1 GiB", GiB), ("64 MiB", 64 * MiB), ("8 MiB", 8 * MiB)]:
        buf = np.empty(size, np.uint8); buf[:] = 1
        t = timeit(lambda: S.fill_controlled_data_seeded(buf, 1, 1, entropy=1))
        out.append({"what": f"fill_controlled_data_seeded -> pageable host {label}", "GiBps": size / t / GiB})
        t = timeit(lambda: S.generate_into_buffer(buf))
        out.append({"what": f"generate_into_buffer -> pageable host {label}", "GiBps": size / t / GiB})
        pin = torch.empty(size, dtype=torch.uint8, pin_memory=True)
        t = timeit(lambda: S.generate_into_buffer(pin.numpy()))
        out.append({"what": f"generate_into_buffer -> pinned host {label}", "GiBps": size / t / GiB})
    g = S.Generator(16 * GiB, seed=1, chunk_size=64 * MiB)
    b = np.empty(64 * MiB, np.uint8); b[:] = 0
    t = time.perf_counter(); n = 0
    while not g.is_complete():
        n += g.fill_chunk(b)
    out.append({"what": "Generator 16 GiB, 64 MiB chunks -> pageable host", "GiBps": n / (time.perf_counter() - t) / GiB})
    t = timeit(lambda: S.generate_npz_bytes([6053, 6053, 1]))
    out.append({"what": "generate_npz_bytes([6053,6053,1]) 140 MiB, host bytes", "ms": t * 1e3,
                "GiBps": S.npz_size([6053, 6053, 1]) / t / GiB,
                "reference": "~20 ms (28-core, docs/Changelog.md:847-852)"})
    ctx = S.Context(0)
    d = torch.empty(16 * GiB, dtype=torch.uint8, device="cuda")
    ctx.xoshiro_fill(d)
    torch.cuda.synchronize()
    t = timeit(lambda: S.crc32_device(ctx, d))
    out.append({"what": "device CRC-32 over 16 GiB (read-bound)", "GBps": 16 * GiB / t / 1e9})
    for o in out:
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in o.items()}))


if __name__ == "__main__":
    main()

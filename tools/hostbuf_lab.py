#!/usr/bin/env python3
"""Owned-result host buffers (generate_data / generate_npz_bytes /
generate_object outputs): pageable pooled mappings (hostbuf.py) vs pinned
memory.  Times s3dg_generate_data into each buffer kind at 1, 8 and 64 MiB
(warm buffers), and the cost of obtaining a FRESH buffer of each kind (mmap +
first-touch faults during the copy, vs hipHostMalloc).  Tooling only."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import s3dlio_amd as S
    from s3dlio_amd import hostbuf
    from s3dlio_amd._lib import call
    MiB = 1 << 20
    out = []
    for size in (1 * MiB, 8 * MiB, 64 * MiB):
        warm = {"hostbuf": hostbuf.empty(size), "numpy": np.ones(size, np.uint8)}
        p = ctypes.c_void_p()
        call("s3dg_host_alloc_pinned", size, ctypes.byref(p))
        warm["pinned"] = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(p.value))
        for b in warm.values():
            call("s3dg_generate_data", int(b.ctypes.data), size, 1, 1, 0, 0)
        reps = max(5, (256 * MiB) // size)
        for name, b in warm.items():
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                call("s3dg_generate_data", int(b.ctypes.data), size, 1, 1, 0, 0)
                ts.append(time.perf_counter() - t)
            out.append({"what": "generate_data into a warm buffer", "buffer": name, "MiB": size // MiB,
                        "us_median": round(statistics.median(ts) * 1e6, 1),
                        "GiBps": round(size / statistics.median(ts) / 2**30, 2)})
        # fresh buffers: a new anonymous mapping (faults during the copy) vs hipHostMalloc + free
        ts_map, ts_pin = [], []
        for _ in range(5):
            import mmap
            t = time.perf_counter()
            mm = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            a = np.frombuffer(mm, np.uint8)
            call("s3dg_generate_data", int(a.ctypes.data), size, 1, 1, 0, 0)
            ts_map.append(time.perf_counter() - t)
            del a
            mm.close()
            t = time.perf_counter()
            q = ctypes.c_void_p()
            call("s3dg_host_alloc_pinned", size, ctypes.byref(q))
            call("s3dg_generate_data", q.value, size, 1, 1, 0, 0)
            call("s3dg_host_free_pinned", q.value)
            ts_pin.append(time.perf_counter() - t)
        out.append({"what": "fresh buffer + generate_data (+ free)", "MiB": size // MiB,
                    "mmap_first_touch_us": round(statistics.median(ts_map) * 1e6, 1),
                    "hipHostMalloc_us": round(statistics.median(ts_pin) * 1e6, 1)})
        call("s3dg_host_free_pinned", p.value)
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()

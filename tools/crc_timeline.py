#!/usr/bin/env python3
"""CRC overlap evidence.

    rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o t --output-format csv -- python3 tools/crc_timeline.py run
    python3 tools/crc_timeline.py summarize DIR

`run`: 5 x generate_npz_bytes([6053, 6053, 1]) (the unet3d-size 140 MiB
archive, src/python_api/python_datagen_api.rs:395) and one file:// PUT of
1024 x 8 MiB (s3dg_put_objects_multi, one GPU).  `summarize`: for every
k_crc32_regions dispatch, how much of its time overlaps a D2H copy, and each
phase's span.  Tooling only."""
import csv
import glob
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MiB = 1 << 20


def run():
    import s3dlio_amd as S
    marks = {}
    for k in range(5):
        t = time.time_ns()
        v = S.generate_npz_bytes([6053, 6053, 1])
        marks[f"npz{k}"] = (t, time.time_ns(), len(v))
    root = tempfile.mkdtemp(prefix="crc_tl_", dir=os.environ.get("PUT_DIR", "/tmp"))
    try:
        t = time.time_ns()
        r = S.put_objects([f"file://{root}/o{j}" for j in range(1024)], 8 * MiB, 16, seed=5,
                          payload="controlled", devices=[0])
        marks["put"] = (t, time.time_ns(), r.bytes)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    print(json.dumps(marks))


def summarize(d):
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    mf = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)[0]
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(kf))]
    cps = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", ""), int(r.get("Bytes", 0) or 0))
           for r in csv.DictReader(open(mf))]
    # D2H copies: SDMA copies in the memory-copy trace, or (HIP's default for
    # these copies on gfx950) blit kernels in the kernel trace
    d2h = sorted([(a, b) for a, b, dr, n in cps if "DEVICE_TO_HOST" in dr.upper()] +
                 [(a, b) for a, b, n in kern if "copyBuffer" in n and b - a > 100_000])
    crc = [(a, b) for a, b, n in kern if "crc32" in n]
    tot = hidden = 0
    for a, b in crc:
        tot += b - a
        for c0, c1 in d2h:
            lo, hi = max(a, c0), min(b, c1)
            if hi > lo:
                hidden += hi - lo
    out = {"crc_dispatches": len(crc), "crc_time_us": round(tot / 1e3, 1),
           "crc_time_under_d2h_us": round(hidden / 1e3, 1),
           "fraction_hidden": round(hidden / tot, 4) if tot else None,
           "d2h_copies": len(d2h), "d2h_time_us": round(sum(b - a for a, b in d2h) / 1e3, 1)}
    # per phase: the NPZ builds (first 5 CRC dispatches of 140 MiB) and the PUT
    npz = [(a, b) for a, b in crc[:5]]
    out["npz_crc_us_each"] = [round((b - a) / 1e3, 1) for a, b in npz]
    big = [(a, b) for a, b in d2h if b - a > 1_000_000][:5]
    out["npz_d2h_us_each"] = [round((b - a) / 1e3, 1) for a, b in big]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2])

#!/usr/bin/env python3
"""Throughput of the PUT pipeline (s3dg_put_objects) to file:// objects, next to
the file-system write ceiling of the same box (the same bytes written from one
host buffer by 16 Python threads).  One JSON line per measurement."""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MiB, GiB = 1 << 20, 1 << 30


def fs_ceiling(root, n, size, threads=16):
    import numpy as np
    buf = np.random.default_rng(1).integers(0, 256, size, dtype=np.uint8).tobytes()
    d = os.path.join(root, "ceiling")
    os.makedirs(d, exist_ok=True)
    idx = iter(range(n))
    lock = threading.Lock()

    def work():
        while True:
            with lock:
                j = next(idx, None)
            if j is None:
                return
            with open(os.path.join(d, f"o{j}"), "wb") as f:
                f.write(buf)

    t = time.perf_counter()
    ts = [threading.Thread(target=work) for _ in range(threads)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    dt = time.perf_counter() - t
    shutil.rmtree(d)
    return n * size / dt / GiB


def main():
    import s3dlio_amd as S
    root = tempfile.mkdtemp(prefix="s3dg_put_", dir=os.environ.get("PUT_DIR", "/tmp"))
    try:
        print(subprocess.run(["df", "-h", root], capture_output=True, text=True).stdout.strip(),
              file=sys.stderr)
        n, size = int(os.environ.get("PUT_N", "1024")), 8 * MiB
        S.put_objects([f"file://{root}/warm/o{j}" for j in range(64)], size, 16, seed=1,
                      payload="controlled")
        shutil.rmtree(f"{root}/warm")
        out = [{"what": f"fs write ceiling: {n} x 8 MiB from one host buffer, 16 threads",
                "GiBps": fs_ceiling(root, n, size)}]
        lanes = [int(x) for x in os.environ.get("PUT_LANES", "1").split(",")]
        for kind, d, c in [("controlled", 1, 1), ("random", 1, 1), ("dgen", 2, 3)]:
            for mif in (16, 64):
                for nl in lanes:
                    uris = [f"file://{root}/p/o{j}" for j in range(n)]
                    cfg = S.Config.new_with_defaults("RAW", 1, size, d, c)
                    r = S.put_objects(uris, size, mif, cfg, seed=3, payload=kind, devices=[0] * nl)
                    out.append({"what": f"put_objects {n} x 8 MiB {kind} d{d} c{c}, max_in_flight={mif}, "
                                        f"{nl} lane(s) on GPU 0",
                                "GiBps": r.bytes / r.seconds / GiB, "seconds": r.seconds,
                                "gpu_wait_seconds": r.gpu_seconds})
                    shutil.rmtree(f"{root}/p")
        for o in out:
            print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in o.items()}))
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Diagnose multi-object DG1 put payloads vs the oracle (tooling)."""
import os
import sys
import tempfile
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import s3dlio_amd as S
    from oracle import oracle_c as O
    from oracle import format_oracle as F
    print("lib:", S._lib.LIB_PATH)
    MiB = 1 << 20
    for kind, t, n, size, d, c in [("dgen", "RAW", 5, 2 * MiB + 17, 2, 2), ("dgen", "RAW", 5, 2 * MiB + 17, 1, 1),
                                   ("dgen", "RAW", 3, 3 * MiB, 1, 1), ("dgen", "NPZ", 5, 2 * MiB + 17, 2, 2)]:
        root = tempfile.mkdtemp()
        uris = [f"file://{root}/o{j}" for j in range(n)]
        cfg = S.Config.new_with_defaults(t, 1, size, d, c)
        seed = 0x1234 + n
        r = S.put_objects(uris, size, 16, cfg, seed=seed, payload=kind)
        fn, fd = S.compress_ratio(max(1, c))
        for j in range(n):
            got = open(f"{root}/o{j}", "rb").read()
            pay = O.dgen_fill(size, d, fn, fd, O.object_entropy(seed, j)).tobytes()
            exp = F.build_npz(1, pay) if t == "NPZ" else pay
            gp = np.frombuffer(got, np.uint8); ep = np.frombuffer(exp, np.uint8)
            diff = np.nonzero(gp != ep)[0] if len(gp) == len(ep) else [-1]
            print(kind, t, n, size, d, c, "obj", j, "ndiff", len(diff), "first", diff[:3] if len(diff) else None,
                  "crc_ok", r.checksums[j] == zlib.crc32(got))


if __name__ == "__main__":
    main()

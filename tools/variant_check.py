#!/usr/bin/env python3
"""Diagnostic: byte-check a compile-time variant library (tools/variant_lab.py
builds) on the K2 keystream and the fill paths against the C oracle before
its timings are trusted.  LAB_VARIANTS as for variant_lab.py.  Tooling only."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from variant_lab import variants, so
    from oracle import oracle_c as OC
    from oracle import oracle_py as P
    u64 = ctypes.c_uint64
    MiB = 1 << 20
    bad = 0
    for name in variants():
        L = ctypes.CDLL(so(name), mode=os.RTLD_LOCAL)
        h = ctypes.c_void_p()
        assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
        base = np.zeros(4096, np.uint8)
        assert L.s3dg_get_base_block(h, base.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == 0
        for n, chunk, sb in [(5242893, 2 * MiB, 0), (64 * MiB + 77, 2 * MiB, 9), (3 * MiB, 65536, 5)]:
            t = torch.empty(n, dtype=torch.uint8, device="cuda")
            assert L.s3dg_xoshiro_fill(h, ctypes.c_void_p(t.data_ptr()), u64(n), u64(chunk), u64(sb), None) == 0
            torch.cuda.synchronize()
            ok = np.array_equal(t.cpu().numpy(), OC.xoshiro_chunks(n, chunk, sb))
            bad += not ok
            print(name, "k2", n, chunk, "ok" if ok else "MISMATCH", flush=True)
        size, cnt = 8 * MiB, 12
        t = torch.empty(size * cnt, dtype=torch.uint8, device="cuda")
        assert L.s3dg_fill_controlled_stream(h, ctypes.c_void_p(t.data_ptr()), u64(size), u64(size), u64(cnt),
                                             u64(2), ctypes.c_uint32(2), ctypes.c_uint32(3), u64(77), u64(0),
                                             None) == 0
        torch.cuda.synchronize()
        ok = np.array_equal(t.cpu().numpy(), OC.fill_stream(size, cnt, 2, 2, 3, 77, 0, base, threads=8))
        bad += not ok
        print(name, "stream", "ok" if ok else "MISMATCH", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

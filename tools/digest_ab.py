"""Two builds of the library in one process, config 2's fill launch (10 000 x
8 MiB, one launch) interleaved in blocks (LAB_REPS launches, LAB_ROUNDS
rounds): does a host-only change between two digests move the device rate?
    python tools/digest_ab.py tools/_labso/lib_<old>.so     # GPU box
Tooling only."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MiB = 1 << 20


def main():
    import torch
    libs = {"tree": os.path.join(ROOT, "s3dlio_amd", "libs3dlio_amd.so"), "other": sys.argv[1]}
    L, H = {}, {}
    for k, path in libs.items():
        L[k] = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
        L[k].s3dg_build_digest.restype = ctypes.c_char_p
        h = ctypes.c_void_p()
        assert L[k].s3dg_ctx_create(0, ctypes.byref(h)) == 0
        H[k] = h
        print(json.dumps({"lib": k, "digest": L[k].s3dg_build_digest().decode()}), flush=True)
    n, size = 10000, 8 * MiB
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    sh, p = ctypes.c_void_p(st.cuda_stream), ctypes.c_void_p(buf.data_ptr())
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32

    def fill(k):
        assert L[k].s3dg_fill_controlled_stream(H[k], p, u64(size), u64(size), u64(n), u64(1), u32(0), u32(1),
                                                u64(0x5EED000000000001), u64(0), sh) == 0
    reps, acc = int(os.environ.get("LAB_REPS", "10")), {}
    with torch.cuda.stream(st):
        for rnd in range(int(os.environ.get("LAB_ROUNDS", "6"))):
            for k in (("tree", "other") if rnd % 2 else ("other", "tree")):
                fill(k)
                st.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
                for a, b in ev:
                    a.record(st)
                    fill(k)
                    b.record(st)
                st.synchronize()
                ms = [a.elapsed_time(b) for a, b in ev]
                gbs = n * size / (sum(ms) / len(ms) * 1e6)
                print(json.dumps({"round": rnd, "lib": k, "GBps": round(gbs, 1), "ms_min": round(min(ms), 4),
                                  "ms_max": round(max(ms), 4)}), flush=True)
                if rnd:
                    acc.setdefault(k, []).append(gbs)
    for k, v in acc.items():
        print(json.dumps({"summary": k, "GBps_mean": round(sum(v) / len(v), 1)}), flush=True)
    print("digest_ab ok", flush=True)


if __name__ == "__main__":
    main()

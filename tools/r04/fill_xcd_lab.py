#!/usr/bin/env python3
"""Do the fill's XCDs finish together?  (The keystream's do not: DESIGN.md
§5.2, round 4.)  A diagnostic copy of the library (sources copied to
tools/_build/src_filltrace; the product tree is not touched) stamps the
wall-clock end of every live k_fill_batch workgroup, indexed by its block's
4 KiB granule in the buffer and bounds-checked against the trace length.
Slots are XCD-aligned, so granule g is written by XCD g mod 8.  Per XCD: when
its last workgroup ended, and how many workgroups it completed in the
launch's last 2 % / 5 %.

    python tools/r04/fill_xcd_lab.py --build    # here
    python tools/r04/fill_xcd_lab.py            # GPU box
Tooling only: nothing in the product imports this."""
import ctypes, json, os, shutil, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_build")
SRC = os.path.join(OUT, "src_filltrace")
LIB = os.path.join(OUT, "libfilltrace.so")
MiB = 1 << 20
TICK_US = 0.01


def build():
    from s3dlio_amd.build import SOURCES, CSRC
    if os.path.isdir(SRC):
        shutil.rmtree(SRC)
    shutil.copytree(CSRC, os.path.join(SRC, "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(SRC, "include"))
    k = os.path.join(SRC, "csrc", "s3dg_kernels.hip")
    s = open(k).read()
    s = s.replace("__device__ uint64_t *g_ks_trace;",
                  "__device__ uint64_t *g_ks_trace;\n__device__ uint64_t *g_fill_trace;\n"
                  "__device__ uint64_t g_fill_trace_n;", 1)
    anchor = "\n}\n\n// Prefix parameters of one object on the device"
    assert s.count(anchor) == 1, "k_fill_batch end not found"
    s = s.replace(anchor, "\n    if (!ABL && t == 0 && g_fill_trace) {\n"
                  "        const uint64_t gi = (e.dst_off >> 12) + (uint64_t)ib;\n"
                  "        if (gi < g_fill_trace_n) g_fill_trace[gi] = wall_clock64();\n    }" + anchor, 1)
    s += ("\n#if S3DG_KS_TRACE\nextern \"C\" __attribute__((visibility(\"default\"))) int s3dg_diag_fill_trace("
          "void *buf, uint64_t n) {\n"
          "    int r = (int)hipMemcpyToSymbol(HIP_SYMBOL(s3dg::g_fill_trace_n), &n, sizeof(n));\n"
          "    if (r) return r;\n"
          "    return (int)hipMemcpyToSymbol(HIP_SYMBOL(s3dg::g_fill_trace), &buf, sizeof(buf));\n}\n#endif\n")
    open(k, "w").write(s)
    srcs = [os.path.join(SRC, "csrc", os.path.basename(p)) for p in SOURCES]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fvisibility=hidden", "-mllvm", "-amdgpu-kernarg-preload-count=16", "-I", os.path.join(SRC, "include"),
           "-I", os.path.join(SRC, "csrc"), "-DS3DG_BUILD", "-DS3DG_KS_TRACE=1", "-o", LIB] + srcs
    subprocess.check_call(cmd)


def main():
    if "--build" in sys.argv:
        build()
        return
    import numpy as np
    import torch
    L = ctypes.CDLL(LIB, mode=os.RTLD_LOCAL)
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    L.s3dg_diag_fill_trace.argtypes = [ctypes.c_void_p, u64]
    h = ctypes.c_void_p()
    assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    n = 10000
    buf = torch.empty(8 * MiB * n, dtype=torch.uint8, device="cuda")
    nblk = 8 * MiB * n // 4096
    trace = torch.zeros(nblk, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    print(json.dumps({"buf_granule_mod8": (buf.data_ptr() >> 12) & 7, "nblk": nblk}), flush=True)
    assert L.s3dg_diag_fill_trace(ctypes.c_void_p(trace.data_ptr()), u64(nblk)) == 0
    p = ctypes.c_void_p(buf.data_ptr())
    cases = {"cfg2 (d1 c1)": (1, 0, 1), "cfg3 (d4 c2)": (4, 1, 2), "cfg5 (d2 c3)": (2, 2, 3)}
    for rep in range(int(os.environ.get("LAB_REPS", "2"))):
        for name, (d, fn, fd) in cases.items():
            def run():
                assert L.s3dg_fill_controlled_stream(h, p, u64(8 * MiB), u64(8 * MiB), u64(n), u64(d), u32(fn),
                                                     u32(fd), u64(0x5EED000000000001), u64(0), sh) == 0
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            trace.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            t = trace.cpu().numpy()
            g = np.nonzero(t)[0]
            e = t[g].astype(np.float64)
            e = (e - e.min()) * TICK_US
            span = float(e.max())
            x = g & 7
            per = {}
            for k in range(8):
                ek = e[x == k]
                per[k] = {"wgs": int(len(ek)), "last_end_us": round(float(ek.max()), 1),
                          "ended_in_last_2pct": int((ek > 0.98 * span).sum()),
                          "ended_in_last_5pct": int((ek > 0.95 * span).sum())}
            lasts = sorted(v["last_end_us"] for v in per.values())
            print(json.dumps({"case": name, "rep": rep, "event_ms": round(ms, 3),
                              "GBps": round(8 * MiB * n / ms / 1e6, 1), "traced_wgs": int(len(g)),
                              "span_us": round(span, 1), "xcd_last_end_spread_us": round(lasts[-1] - lasts[0], 1),
                              "per_xcd": per}), flush=True)


if __name__ == "__main__":
    main()

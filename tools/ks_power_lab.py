"""Is the keystream power-bound?    The per-XCC
counters (profiles/r06/xcc/) put K2's write rate per GFX cycle at the fill's
and its clock ~5 % lower; the cause proposed is the power its PRNG draws under
the 1400 W limit.  This lab times config 6's K2 launch (10 000 x 8 MiB as
2 MiB chunks, one persistent k_keystream launch) from the product library and
from a diagnostic build with the Xoshiro steps replaced by adds
(-DS3DG_ABLATE=32: same LDS stages, same stores, same launch; wrong bytes by
design), blocks of LAB_REPS launches alternating, with the amdsmi GFX clock
and socket power polled every ~5 ms.  Also the fill (config 2) for reference.

    python tools/ks_power_lab.py --build     # here: tools/_labso/libks_ablate32.so
    python tools/ks_power_lab.py             # GPU box
Tooling only: nothing in the product imports this."""
import ctypes
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
OUT = os.path.join(ROOT, "tools", "_labso")
MiB = 1 << 20


def build():
    os.makedirs(OUT, exist_ok=True)
    from s3dlio_amd.build import SOURCES
    so = os.path.join(OUT, "libks_ablate32.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-fvisibility=hidden", "-DS3DG_BUILD", "-DS3DG_ABLATE=32",
                           "-mllvm", "-amdgpu-kernarg-preload-count=16",
                           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "s3dlio_amd", "csrc"),
                           "-o", so] + SOURCES)
    print(so)


def main():
    if "--build" in sys.argv:
        return build()
    import torch
    from zero_power_lab import smi_handle
    libs = {"product": ctypes.CDLL(os.path.join(ROOT, "s3dlio_amd", "libs3dlio_amd.so"), mode=os.RTLD_LOCAL),
            "ablate32": ctypes.CDLL(os.path.join(OUT, "libks_ablate32.so"), mode=os.RTLD_LOCAL)}
    ctx = {}
    for k, L in libs.items():
        h = ctypes.c_void_p()
        assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
        ctx[k] = h
    n, size = 10000, 8 * MiB
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    p = ctypes.c_void_p(buf.data_ptr())
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32

    def k2(k):
        assert libs[k].s3dg_xoshiro_fill(ctx[k], p, u64(n * size), u64(2 * MiB), u64(0), sh) == 0

    def fill(k):
        assert libs[k].s3dg_fill_controlled_stream(ctx[k], p, u64(size), u64(size), u64(n), u64(1), u32(0), u32(1),
                                                   u64(0x5EED000000000001), u64(0), sh) == 0
    smi, sm, bdf = smi_handle()
    rows, on = [], [True]

    def poller():
        while on[0]:
            try:
                m = smi.amdsmi_get_gpu_metrics_info(sm)
                rows.append((time.perf_counter(), m.get("current_gfxclk"), m.get("current_socket_power")))
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.005)
    th = threading.Thread(target=poller, daemon=True)
    th.start()
    reps = int(os.environ.get("LAB_REPS", "12"))
    cases = [("k2", "product", k2), ("k2", "ablate32", k2), ("fill", "product", fill)]
    acc = {}
    with torch.cuda.stream(st):
        for rnd in range(int(os.environ.get("LAB_ROUNDS", "4"))):
            for name, lib, f in cases:
                f(lib)
                st.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record(st)
                for _ in range(reps):
                    f(lib)
                e1.record(st)
                e1.synchronize()
                t1 = time.perf_counter()
                ms = e0.elapsed_time(e1) / reps
                sel = [r for r in rows if t0 + 0.2 * (t1 - t0) <= r[0] <= t1]
                clk = [r[1] for r in sel if r[1]]
                pw = [r[2] for r in sel if r[2]]
                rec = {"round": rnd, "kernel": name, "library": lib, "GBps": round(n * size / (ms * 1e6), 1),
                       "gfxclk_MHz": round(sum(clk) / len(clk), 1) if clk else None,
                       "socket_W": round(sum(pw) / len(pw), 1) if pw else None, "samples": len(sel)}
                print(json.dumps(rec), flush=True)
                if rnd > 0:
                    acc.setdefault((name, lib), []).append(rec)
    on[0] = False
    th.join()
    for (name, lib), v in acc.items():
        def mean(key):
            xs = [r[key] for r in v if r[key] is not None]
            return round(sum(xs) / len(xs), 1) if xs else None
        print(json.dumps({"summary": f"{name}/{lib}", "GBps": mean("GBps"), "gfxclk_MHz": mean("gfxclk_MHz"),
                          "socket_W": mean("socket_W"), "rounds": len(v)}), flush=True)
    print("ks_power_lab ok", flush=True)


if __name__ == "__main__":
    main()

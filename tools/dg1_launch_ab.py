#!/usr/bin/env python3
"""Why do bench.py's per-object DG1 launches (config 14) run slower than the
variant lab's?  (tooling)  10 x 8 GiB DG1 c1 launches, interleaved in one
process, through (a) the product's Context + call() as bench.py does, with
its per-launch events, (b) the product library through raw ctypes, (c) the
lab build (tools/_build/libvariant_cur.so) as tools/variant_lab.py calls it,
and (d) bench.py's own step: its ring, seeds and per-launch events.
Nothing in the product imports this."""
import ctypes, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GiB, MiB = 1 << 30, 1 << 20
SEED = 0x5EED000000000001


def main():
    import torch
    from s3dlio_amd import Context, object_entropy
    from s3dlio_amd._lib import call, lib
    n = 10
    ctx = Context(0, base_seed=0xBA5EB10C00000000)
    st = torch.cuda.current_stream()
    sh = int(st.cuda_stream)
    buf = torch.empty(n * 8 * GiB, dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    V = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libvariant_cur.so"), mode=os.RTLD_LOCAL)
    vh = ctypes.c_void_p()
    assert V.s3dg_ctx_create(0, ctypes.byref(vh)) == 0
    vsh = ctypes.c_void_p(sh)

    def a():   # bench.py: Context + call(), event pair per launch
        evs = []
        for t in range(n):
            evs.append(torch.cuda.Event(enable_timing=True)); evs[-1].record(st)
            call("s3dg_dgen_fill", ctx._h, base + t * 8 * GiB, 8 * GiB, 0, 1 << 40, 1, 0, 1,
                 object_entropy(SEED, t), sh)
            evs.append(torch.cuda.Event(enable_timing=True)); evs[-1].record(st)

    def b():   # product library, raw ctypes with the variant lab's argument objects
        for t in range(n):
            assert lib.s3dg_dgen_fill(ctx._h, base + t * 8 * GiB, 8 * GiB, 0, 1 << 40, 1, 0, 1, 777 + t, sh) == 0

    def c():   # lab build, as tools/variant_lab.py
        for t in range(n):
            q = ctypes.c_void_p(base + t * 8 * GiB)
            assert V.s3dg_dgen_fill(vh, q, u64(8 * GiB), u64(0), u64(1 << 40), u64(1), u32(0), u32(1),
                                    u64(777 + t), vsh) == 0

    def d():   # product library, the lab's seeds, through call()
        for t in range(n):
            call("s3dg_dgen_fill", ctx._h, base + t * 8 * GiB, 8 * GiB, 0, 1 << 40, 1, 0, 1, 777 + t, sh)

    def e():   # lab build with bench seeds
        for t in range(n):
            q = ctypes.c_void_p(base + t * 8 * GiB)
            assert V.s3dg_dgen_fill(vh, q, u64(8 * GiB), u64(0), u64(1 << 40), u64(1), u32(0), u32(1),
                                    u64(object_entropy(SEED, t)), vsh) == 0

    W = {"a_bench_style": a, "b_product_raw": b, "c_lab_build": c, "d_product_lab_seeds": d, "e_lab_build_bench_seeds": e}
    res = {}
    for rep in range(4):
        for k, f in W.items():
            f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(3):
                f()
            e1.record(st)
            torch.cuda.synchronize()
            res.setdefault(k, []).append(3 * n * 8 * GiB / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        print(f"rep {rep} done", flush=True)
    for k, r in res.items():
        print(json.dumps({"kind": k, "GBps_median": round(statistics.median(r), 1), "all": [round(x) for x in r]}),
              flush=True)


if __name__ == "__main__":
    main()

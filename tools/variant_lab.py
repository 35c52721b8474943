#!/usr/bin/env python3
"""Diagnostic: A/B of compile-time kernel variants on the same workloads,
interleaved in one process.  Each variant is the product library built with
extra -D flags (LAB_VARIANTS="name=-DFOO=1 -DBAR=2;name2=").  Points as in
tools/batch_lab.py: "kind:waves:occ:pf:store[:tile];..." with kind in
stream2 (cfg2 stream), stream3 (cfg3 stream), cfg4 (log-uniform batch),
cfg7 (uniform 8 MiB batch), small (log-uniform 4 KiB-1 MiB batch), mid
(uniform 1 MiB + 123 B batch), ceiling (store-only kernel), crc (s3dg_crc32),
k2 (2 MiB keystream chunks; fields waves:wgs_per_cu:min_lane_draws:store[:xcd_waves]).

    LAB_VARIANTS=... python tools/variant_lab.py --build-only   # here
    LAB_VARIANTS=... LAB_POINTS=... python tools/variant_lab.py # GPU box
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_build")


def variants():
    spec = os.environ.get("LAB_VARIANTS", "base=")
    out = {}
    for item in spec.split(";"):
        name, _, flags = item.partition("=")
        out[name.strip()] = flags.split()
    return out


def so(name):
    return os.path.join(OUT, f"libvariant_{name}.so")


def build():
    from s3dlio_amd.build import SOURCES, CSRC
    os.makedirs(OUT, exist_ok=True)
    procs = []
    for name, flags in variants().items():
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-mllvm", "-amdgpu-kernarg-preload-count=16", "-I", os.path.join(ROOT, "include"),
               "-I", CSRC, "-DS3DG_BUILD", *flags, "-o", so(name)] + SOURCES
        procs.append(subprocess.Popen(cmd))
        if len(procs) >= 4:
            assert procs.pop(0).wait() == 0
    for p in procs:
        assert p.wait() == 0


def main():
    if "--build-only" in sys.argv:
        build()
        return
    import torch
    from bench import log_uniform_sizes, SEED_BASE
    from s3dlio_amd._lib import ObjDesc
    MiB = 1 << 20
    n = int(os.environ.get("LAB_N", "10000"))
    nsmall = int(os.environ.get("LAB_NSMALL", str(20 * n)))   # objects of the kb20* kinds
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    libs = {}
    for name in variants():
        L = ctypes.CDLL(so(name), mode=os.RTLD_LOCAL)
        h = ctypes.c_void_p()
        assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
        libs[name] = (L, h)
    descs = {}
    for kind, sizes, d, fn, fd in [("cfg4", log_uniform_sizes(n), 2, 1, 3), ("cfg7", [8 * MiB] * n, 1, 0, 1),
                                   ("cfg4d1", log_uniform_sizes(n), 1, 0, 1), ("cfg4c1", log_uniform_sizes(n), 2, 0, 1),
                                   # config 4's sizes rounded up to whole 64-block tiles (256 KiB): no dead slots
                                   ("cfg4r", [(x + (256 << 10) - 1) // (256 << 10) * (256 << 10) for x in log_uniform_sizes(n)],
                                    1, 0, 1),
                                   # config 4's sizes, largest first / smallest first
                                   ("cfg4desc", sorted(log_uniform_sizes(n), reverse=True), 1, 0, 1),
                                   ("small", log_uniform_sizes(10 * n, 5, 4096, MiB), 1, 0, 1),
                                   ("mid", [MiB + 123] * (5 * n), 3, 2, 3),
                                   ("kb64", [64 << 10] * (10 * n), 1, 0, 1),
                                   ("kb20", [(20 << 10) + 5] * nsmall, 1, 0, 1),
                                   ("kb20n", [20 << 10] * nsmall, 1, 0, 1),      # 5 blocks, packed
                                   ("kb20g", [20 << 10] * nsmall, 1, 0, 1)]:     # 5 blocks, 24 KiB stride
        gap = 4096 if kind == "kb20g" else 0
        arr = (ObjDesc * len(sizes))()
        off = 0
        for j, sz in enumerate(sizes):
            arr[j] = ObjDesc(off, sz, SEED_BASE + (j << 32), d, fn, fd)
            off += (sz + 4095) // 4096 * 4096 + gap
        descs[kind] = (arr, sum(sizes), off)
    crcs = {}
    work = {"stream2": 8 * MiB * n, "k2": 8 * MiB * n, "k2_8g": 8 * MiB * n, "dg1": 8 * MiB * n,
            "dg1_8g": 8 * MiB * n, "dg1c2_8g": 8 * MiB * n, "stream3": 8 * MiB * n, "stream5": 8 * MiB * n, "ceiling": 8 * MiB * n, "crc": 8 * MiB * n,
            **{k: v[1] for k, v in descs.items()}}
    buf = torch.empty(max([8 * MiB * n] + [v[2] for v in descs.values()]), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    p = ctypes.c_void_p(buf.data_ptr())

    def stream_params(kind):
        if kind in ("stream2", "stream3", "stream5"):
            return {"stream2": (1, 0, 1), "stream3": (4, 1, 2), "stream5": (2, 2, 3)}[kind]
        if kind.startswith("sd") and kind.count("x") == 2:   # "sd<dedup>x<f_num>x<f_den>": any stream
            d, fn, fd = kind[2:].split("x")
            return int(d), int(fn), int(fd)
        return None

    for k in os.environ.get("LAB_POINTS", "").split(";"):
        if stream_params(k.split(":")[0]):
            work[k.split(":")[0]] = 8 * MiB * n

    def run(L, h, kind):
        if stream_params(kind):
            d, fn, fd = stream_params(kind)
            r = L.s3dg_fill_controlled_stream(h, p, u64(8 * MiB), u64(8 * MiB), u64(n), u64(d), u32(fn), u32(fd),
                                              u64(SEED_BASE), u64(0), sh)
        elif kind == "k2":                   # xoshiro keystream, 2 MiB chunks
            r = L.s3dg_xoshiro_fill(h, p, u64(8 * MiB * n), u64(2 * MiB), u64(0), sh)
        elif kind in ("k2_8g", "dg1", "dg1_8g", "dg1c2_8g"):   # keystream / DG1 launches of 8 GiB or one
            per = 8 << 30 if kind.endswith("_8g") else 8 * MiB * n
            r = 0
            for t in range((8 * MiB * n) // per):
                q = ctypes.c_void_p(buf.data_ptr() + t * per)
                if kind == "k2_8g":
                    r |= L.s3dg_xoshiro_fill(h, q, u64(per), u64(2 * MiB), u64(t * (per // (2 * MiB))), sh)
                else:
                    d, fn, fd = (2, 1, 2) if kind == "dg1c2_8g" else (1, 0, 1)
                    r |= L.s3dg_dgen_fill(h, q, u64(per), u64(0), u64(1 << 40), u64(d), u32(fn), u32(fd),
                                          u64(777 + t), sh)
        elif kind == "ceiling":
            r = L.s3dg_write_ceiling(h, p, u64(8 * MiB * n), u32(0xA5A5A5A5), sh)
        elif kind == "crc":                  # synchronous: device regions + host fold
            out = u32()
            r = L.s3dg_crc32(h, p, u64(8 * MiB * n), sh, ctypes.byref(out))
            crcs.setdefault(L, set()).add(out.value)
        else:
            r = L.s3dg_fill_controlled_batch(h, p, descs[kind][0], u64(len(descs[kind][0])), sh)
        assert r == 0
    pts = []
    for item in os.environ.get("LAB_POINTS", "stream2:2:-1:128:-1;cfg4:1:-1:128:-1").split(";"):
        k, w, o, f, sp, *tb = item.split(":")
        pts.append((k, int(w), int(o), int(f), int(sp), int(tb[0]) if tb else 0))
    res = {}
    for rep in range(int(os.environ.get("LAB_REPS", "4"))):
        for pt in pts:
            order = list(libs.items())
            if os.environ.get("LAB_ALTERNATE") and rep % 2:   # reverse the variant order on odd rounds
                order.reverse()
            for name, (L, h) in order:
                k, w, o, f, sp, tb = pt
                assert L.s3dg_set_waves_per_block(h, w) == 0
                assert L.s3dg_set_occupancy(h, o, o) == 0
                assert L.s3dg_set_batch_prefetch(h, u32(f)) == 0
                assert L.s3dg_set_store_policy(h, sp, sp) == 0
                if not (k.startswith("k2") or k.startswith("dg1")):
                    assert L.s3dg_set_batch_tile(h, u32(tb)) == 0
                ksd = int(k.split("@")[1]) if "@" in k else 64   # "k2@32": 32 draws per stage
                if k.startswith("k2"):         # k2 / dg1: waves, wgs/CU, min lane draws, store
                    assert L.s3dg_set_keystream_shape(h, 0, ksd, w, o, u64(f), sp) == 0
                if k.startswith("dg1"):
                    assert L.s3dg_set_keystream_shape(h, 1, ksd, w, o, u64(f), sp) == 0
                if (k.startswith("k2") or k.startswith("dg1")) and hasattr(L, "s3dg_set_keystream_xcd_group"):
                    for md in (0, 1):           # 6th field: waves per XCD group (0 = default)
                        assert L.s3dg_set_keystream_xcd_group(h, md, u32(tb)) == 0
                run(L, h, k.split("@")[0])
                torch.cuda.synchronize()
                if k == "crc":
                    import time
                    t0 = time.perf_counter(); run(L, h, k); dt = time.perf_counter() - t0
                else:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st); run(L, h, k.split("@")[0]); e1.record(st); torch.cuda.synchronize()
                    dt = e0.elapsed_time(e1) * 1e-3
                res.setdefault((name, pt), []).append(work[k.split("@")[0]] / dt / 1e9)
        print(f"rep {rep} done", flush=True)
    if crcs:
        print(json.dumps({"crc_values_per_variant": {n: sorted(crcs.get(libs[n][0], [])) for n in libs}}))
    for (name, pt), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        print(json.dumps({"variant": name, "point": ":".join(map(str, pt)),
                          "GBps_median": round(statistics.median(v), 1), "max": round(max(v), 1)}), flush=True)


if __name__ == "__main__":
    main()

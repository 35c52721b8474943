#!/usr/bin/env python3
"""Library A/B in one process: whole product libraries
(another commit's sources, or this tree with diagnostic -D flags) loaded side
by side, each with its own context, and timed on the same workloads with the
library defaults, interleaved, variant order rotated every round.

    python tools/lib_ab.py --build        # here: builds tools/_build/libab_<name>.so
    python tools/lib_ab.py                # GPU box: runs LAB_POINTS x variants

Variants (LAB_AB, "name=git-ref|.[:-Dflag ...];..."): git-ref = the sources
of that commit (git archive), "." = this tree.  Default: r02 final (aa93058),
r03 final (dedd5d0), this tree (the first session also ran this tree with the
batch floor compiled out and with round 2's 2^22-workgroup grid cap, flags
since removed or kept as diagnostics: profiles/r04/lib_ab/).
Points: cfg2 / cfg3 / cfg5 (10 000 x 8 MiB streams, d1 c1 / d4 c2 / d2 c3),
cfg4 (10 000 log-uniform objects, d2 c1.5, batch), cfg10 (2 000 000 x
(20 KiB + 5 B) at a 24 KiB stride, batch, dense layout), kb20g (2 000 000 x
20 KiB at a 24 KiB stride: a dead gap slot per object); keystream points
cfg14 / cfg15 (ten 8 GiB DG1 launches, d1 c1 / d2 c2), cfg16 (the ten in one
launch), cfg6 (K2, 10 000 x 8 MiB as 2 MiB chunks, one launch), k2_8g (the
same keystream as 8 GiB launches; k2_8g_2048 with 2048-draw lanes), dg1_4g
(twenty 4 GiB DG1 c1 launches).  Each sample is LAB_LAUNCHES
back-to-back launches between two HIP events on one stream.

Per-launch mode (the driver scores the MEAN, and a
median hides a slow mode): LAB_BLOCK=B times every launch with its own event
pair, B launches back to back per variant per rep (as bench.py's steps run),
and reports per variant the mean, p10/p50/p90/max and the share of launches
slower than LAB_SLOW x the fastest variant's p10 (default 1.06); LAB_SMI=1
polls the GPU's GFX clock and socket power (amdsmi, every ~5 ms) and gives
the medians seen during the slow and the normal launches of each variant.
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, subprocess, sys, tarfile, io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_build")
DEFAULT = "r02=aa93058;r03=dedd5d0;head=."
SRC_NAMES = ["s3dg_kernels.hip", "s3dg_capi.cpp", "s3dg_jump.cpp", "s3dg_generator.cpp", "s3dg_crc.hip",
             "s3dg_npz.cpp", "s3dg_object.cpp", "s3dg_put.cpp", "s3dg_numa.cpp", "s3dg_host.cpp", "s3dg_batch.hip"]


def variants():
    out = {}
    for item in os.environ.get("LAB_AB", DEFAULT).split(";"):
        name, _, spec = item.partition("=")
        ref, _, flags = spec.partition(":")
        out[name.strip()] = (ref.strip(), flags.split())
    return out


def so(name):
    return os.path.join(OUT, f"libab_{name}.so")


def sources(ref):
    """(include dir, csrc dir) of a git ref's sources, or of this tree."""
    if ref == ".":
        return os.path.join(ROOT, "include"), os.path.join(ROOT, "s3dlio_amd", "csrc")
    dst = os.path.join(OUT, f"src_{ref}")
    if not os.path.isdir(dst):
        blob = subprocess.check_output(["git", "-C", ROOT, "archive", ref, "include", "s3dlio_amd/csrc"])
        with tarfile.open(fileobj=io.BytesIO(blob)) as t:
            t.extractall(dst)
    return os.path.join(dst, "include"), os.path.join(dst, "s3dlio_amd", "csrc")


def build():
    os.makedirs(OUT, exist_ok=True)
    procs = []
    for name, (ref, flags) in variants().items():
        inc, csrc = sources(ref)
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-fvisibility=hidden", "-Wno-unused-function", "-mllvm", "-amdgpu-kernarg-preload-count=16",
               "-I", inc, "-I", csrc, "-DS3DG_BUILD", *flags, "-o", so(name)] + [
                   os.path.join(csrc, s) for s in SRC_NAMES if os.path.exists(os.path.join(csrc, s))]
        procs.append(subprocess.Popen(cmd))
        if len(procs) >= 3:
            assert procs.pop(0).wait() == 0
    for p in procs:
        assert p.wait() == 0


def main():
    if "--build" in sys.argv:
        build()
        return
    import torch
    from bench import log_uniform_sizes, SEED_BASE

    class ObjDesc(ctypes.Structure):
        _fields_ = [("dst_off", ctypes.c_uint64), ("size", ctypes.c_uint64), ("entropy", ctypes.c_uint64),
                    ("dedup", ctypes.c_uint64), ("f_num", ctypes.c_uint32), ("f_den", ctypes.c_uint32)]
    MiB = 1 << 20
    n = int(os.environ.get("LAB_N", "10000"))
    launches = int(os.environ.get("LAB_LAUNCHES", "3"))
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    libs = {}
    for name in variants():
        L = ctypes.CDLL(so(name), mode=os.RTLD_LOCAL)
        L.s3dg_fill_controlled_stream.argtypes = [ctypes.c_void_p] * 2 + [u64] * 4 + [u32] * 2 + [u64] * 2 + [
            ctypes.c_void_p]
        L.s3dg_fill_controlled_batch.argtypes = [ctypes.c_void_p] * 3 + [u64, ctypes.c_void_p]
        L.s3dg_dgen_fill.argtypes = [ctypes.c_void_p] * 2 + [u64] * 4 + [u32] * 2 + [u64, ctypes.c_void_p]
        L.s3dg_dgen_fill_stream.argtypes = [ctypes.c_void_p] * 2 + [u64] * 4 + [u32] * 2 + [u64] * 2 + [
            ctypes.c_void_p]
        L.s3dg_xoshiro_fill.argtypes = [ctypes.c_void_p] * 2 + [u64] * 3 + [ctypes.c_void_p]
        h = ctypes.c_void_p()
        assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
        libs[name] = (L, h)
    sizes = log_uniform_sizes(n)
    arr = (ObjDesc * n)()
    off = 0
    for j, sz in enumerate(sizes):
        arr[j] = ObjDesc(off, sz, SEED_BASE + (j << 32), 2, 1, 3)
        off += (sz + 4095) // 4096 * 4096
    # config 10's objects: 2 000 000 x (20 KiB + 5 B) at a 24 KiB stride, d1 c1 (dense layout)
    n10 = int(os.environ.get("LAB_N10", "2000000"))
    arr10 = (ObjDesc * n10)()
    for j in range(n10):
        arr10[j] = ObjDesc(j * 24576, 20 * 1024 + 5, SEED_BASE + (j << 32), 1, 0, 1)
    # "kb20g": config 10's count of 20 KiB objects at a 24 KiB stride (a dead gap slot per object)
    arr20g = (ObjDesc * n10)()
    for j in range(n10):
        arr20g[j] = ObjDesc(j * 24576, 20 * 1024, SEED_BASE + (j << 32), 1, 0, 1)
    buf = torch.empty(max(8 * MiB * n, off, n10 * 24576, 10 << 33), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    p = ctypes.c_void_p(buf.data_ptr())
    streams = {"cfg2": (1, 0, 1), "cfg3": (4, 1, 2), "cfg5": (2, 2, 3)}
    work = {k: 8 * MiB * n for k in streams}
    work["cfg4"] = sum(sizes)
    work["cfg10"] = n10 * (20 * 1024 + 5)
    work["kb20g"] = n10 * 20 * 1024

    G8 = 8 << 30
    ks_pts = {"cfg14": (1, 0, 1), "cfg15": (2, 1, 2)}   # DG1 d, f_num, f_den: ten 8 GiB launches
    for k in ("cfg14", "cfg15", "cfg16", "cfg6", "k2_8g", "k2_8g_2048", "dg1_4g"):
        work[k] = 10 * G8 if k != "cfg6" else 8 * MiB * n

    def run(L, h, kind):
        kind, _, split = kind.partition("@")      # "cfg4@64": s3dg_set_batch_split(64) for this point
        if hasattr(L, "s3dg_set_batch_split"):
            assert L.s3dg_set_batch_split(h, int(split) if split else -1) == 0
        if kind in ks_pts:                        # configs 14/15: one s3dg_dgen_fill per 8 GiB object
            d, fn, fd = ks_pts[kind]
            for t in range(10):
                assert L.s3dg_dgen_fill(h, ctypes.c_void_p(buf.data_ptr() + t * G8), u64(G8), u64(0), u64(1 << 40),
                                        u64(d), u32(fn), u32(fd), u64(SEED_BASE + t), sh) == 0
            return
        if kind == "cfg16":                       # ten 8 GiB DG1 objects in one launch
            assert L.s3dg_dgen_fill_stream(h, p, u64(G8), u64(G8), u64(10), u64(1), u32(0), u32(1),
                                           u64(SEED_BASE), u64(0), sh) == 0
            return
        if kind == "cfg6":                        # K2: 10 000 x 8 MiB as 2 MiB chunks, one launch
            assert L.s3dg_xoshiro_fill(h, p, u64(8 * MiB * n), u64(2 * MiB), u64(0), sh) == 0
            return
        if kind == "dg1_4g":                      # twenty 4 GiB DG1 c1 launches (4 rounds each)
            for t in range(20):
                assert L.s3dg_dgen_fill(h, ctypes.c_void_p(buf.data_ptr() + t * (G8 // 2)), u64(G8 // 2), u64(0),
                                        u64(1 << 40), u64(1), u32(0), u32(1), u64(SEED_BASE + t), sh) == 0
            return
        if kind in ("k2_8g", "k2_8g_2048"):       # the same keystream as 8 GiB launches
            if kind == "k2_8g_2048":              # 2048-draw lanes (8 rounds) instead of 4096 (4)
                assert L.s3dg_set_keystream_shape(h, 0, 0, 0, 0, u64(2048), -1) == 0
            for t in range(10):
                assert L.s3dg_xoshiro_fill(h, ctypes.c_void_p(buf.data_ptr() + t * G8), u64(G8), u64(2 * MiB),
                                           u64(t * (G8 // (2 * MiB))), sh) == 0
            if kind == "k2_8g_2048":
                assert L.s3dg_set_keystream_shape(h, 0, 0, 0, 0, u64(0), -1) == 0
            return
        if kind in streams:
            d, fn, fd = streams[kind]
            r = L.s3dg_fill_controlled_stream(h, p, 8 * MiB, 8 * MiB, n, d, fn, fd, SEED_BASE, 0, sh)
        elif kind == "cfg10":
            r = L.s3dg_fill_controlled_batch(h, p, arr10, n10, sh)
        elif kind == "kb20g":
            r = L.s3dg_fill_controlled_batch(h, p, arr20g, n10, sh)
        else:
            r = L.s3dg_fill_controlled_batch(h, p, arr, n, sh)
        assert r == 0, (kind, r)

    pts = os.environ.get("LAB_POINTS", "cfg2;cfg3;cfg5;cfg4").split(";")
    names = list(libs)
    res = {}
    digests = {}
    reps = int(os.environ.get("LAB_REPS", "8"))
    block = int(os.environ.get("LAB_BLOCK", "0"))   # > 0: per-launch events, B launches per variant per rep
    per = {}                                        # (variant, point) -> [(ms, t_start_host, t_end_host)]
    rows, on, th = [], [True], None
    if block and os.environ.get("LAB_SMI") == "1":
        import threading, time
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from zero_power_lab import smi_handle
        smi, sm, bdf = smi_handle()
        print(json.dumps({"smi_device": bdf}), flush=True)

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
    import time
    for rep in range(reps):
        for k in pts:
            order = names[rep % len(names):] + names[:rep % len(names)]
            if rep % 2:
                order.reverse()
            for name in order:
                L, h = libs[name]
                run(L, h, k)
                torch.cuda.synchronize()
                if block:
                    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                           for _ in range(block)]
                    for e0, e1 in evs:
                        e0.record(st)
                        run(L, h, k)
                        e1.record(st)
                    t_end = []
                    for _, e1 in evs:       # host stamp of each launch's end (lags by the sync latency)
                        e1.synchronize()
                        t_end.append(time.perf_counter())
                    for q, (e0, e1) in enumerate(evs):
                        ms = e0.elapsed_time(e1)
                        per.setdefault((name, k), []).append((ms, t_end[q - 1] if q else t_end[q] - ms / 1e3,
                                                              t_end[q]))
                        res.setdefault((name, k), []).append(work[k.partition("@")[0]] / (ms * 1e-3) / 1e9)
                else:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(launches):
                        run(L, h, k)
                    e1.record(st)
                    torch.cuda.synchronize()
                    res.setdefault((name, k), []).append(launches * work[k.partition("@")[0]] /
                                                        (e0.elapsed_time(e1) * 1e-3) / 1e9)
                if rep == 0:   # every variant writes the same bytes
                    digests.setdefault(k, {})[name] = int(buf[:64 * MiB].to(torch.int64).sum().item())
        print(f"rep {rep} done", flush=True)
    on[0] = False
    if th:
        th.join()
    slow_x = float(os.environ.get("LAB_SLOW", "1.06"))

    def pct(v, q):
        v = sorted(v)
        return v[min(len(v) - 1, int(q * len(v)))]
    for k in pts:
        same = len(set(digests[k].values())) == 1
        print(json.dumps({"point": k, "outputs_identical": same}), flush=True)
        if block:
            fastest = min(pct([m for m, _, _ in per[(n_, k)]], 0.1) for n_ in names)
            thr = slow_x * fastest
        for name in names:
            v = res[(name, k)]
            out = {"variant": name, "point": k, "GBps_median": round(statistics.median(v), 1),
                   "min": round(min(v), 1), "max": round(max(v), 1), "n": len(v)}
            if block:
                ms = [m for m, _, _ in per[(name, k)]]
                mean_ms = sum(ms) / len(ms)
                slow = [i for i, m in enumerate(ms) if m > thr]
                # where the slow launches sit: (rep, position in its block, ms)
                out["slow_launches"] = [(i // block, i % block, round(ms[i], 3)) for i in slow][:40]
                out["slow_share_first_in_block"] = round(sum(1 for i in slow if i % block == 0) / len(ms), 4)
                out.update({"GBps_mean": round(work[k.partition("@")[0]] / (mean_ms * 1e-3) / 1e9, 1),
                            "ms_mean": round(mean_ms, 4), "ms_p10": round(pct(ms, 0.1), 4),
                            "ms_p50": round(pct(ms, 0.5), 4), "ms_p90": round(pct(ms, 0.9), 4),
                            "ms_max": round(max(ms), 4), "slow_threshold_ms": round(thr, 4),
                            "slow_share": round(len(slow) / len(ms), 4)})
                if rows:
                    def during(ids):
                        clk, pw = [], []
                        for i in ids:
                            _, a, b = per[(name, k)][i]
                            for r in rows:
                                if a < r[0] <= b:
                                    if isinstance(r[1], (int, float)):
                                        clk.append(r[1])
                                    if isinstance(r[2], (int, float)):
                                        pw.append(r[2])
                        return {"launches": len(ids), "gfxclk_med": statistics.median(clk) if clk else None,
                                "gfxclk_min": min(clk) if clk else None,
                                "power_med": statistics.median(pw) if pw else None, "samples": len(clk)}
                    fast = [i for i in range(len(ms)) if i not in set(slow)]
                    out["smi_normal"] = during(fast)
                    out["smi_slow"] = during(slow)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

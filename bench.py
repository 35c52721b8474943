#!/usr/bin/env python3
"""bench.py — device-resident synthetic-payload GiB/s (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]

A "step" is one pass of the hot path over one batch: every object of the
configuration generated once into HBM by the gfx950 kernel (src/data_gen.rs
fill_controlled_data semantics, one payload per object).  Default workload =
BASELINE config 2: 10 000 x 8 MiB objects, dedup=1, compress=1 per GPU.
N>1: launched by torch.distributed.run, one rank per GPU; each rank owns its
own object-index range (weak scaling, no data-path collective; a gloo
control plane does the barrier and the max over ranks).

Prints ONE JSON line on rank 0 (contract in the task statement), including
`roofline` (kernel-event timing vs the 8 TB/s HBM peak) and `cpu_baseline`
(the C oracle, multi-threaded, on this host — rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MiB = 1 << 20
GiB = 1 << 30
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
SEED_BASE = 0x5EED000000000001
BASE_SEED = 0xBA5EB10C00000000
METRIC = "device-resident synthetic-payload GiB/s, 8 MiB objects, 1/2/4/8 MI355X"

CONFIGS = {
    2: dict(name="cfg2: 10000 x 8 MiB, dedup=1 compress=1 (pure fill)", n=10000,
            size=8 * MiB, dedup=1, compress=1, scaling="weak"),
    3: dict(name="cfg3: 10000 x 8 MiB, dedup=4 compress=2", n=10000, size=8 * MiB,
            dedup=4, compress=2, scaling="weak"),
    4: dict(name="cfg4: 10000 x log-uniform 4 KiB..64 MiB, dedup=2 compress=1.5", n=10000,
            size=None, dedup=2, compress=(3, 2), scaling="weak"),
    5: dict(name="cfg5: 100000 x 8 MiB, dedup=2 compress=3 (total over all GPUs)", n=100000,
            size=8 * MiB, dedup=2, compress=3, scaling="strong"),
    # not a BASELINE config: the K2 keystream (npz x-fill, npz.rs:376-383) over the cfg2 footprint
    7: dict(name="diag: cfg2 objects (10000 x 8 MiB, d1 c1) through the batch API", n=10000,
            size=None, dedup=1, compress=1, scaling="weak", uniform=8 * MiB),
    6: dict(name="k2: keystream fill, 10000 x 8 MiB as 2 MiB Xoshiro256++ chunks", n=10000,
            size=8 * MiB, dedup=1, compress=1, scaling="weak", keystream=True),
}


def log_uniform_sizes(n: int, seed: int = 4, lo: int = 4096, hi: int = 64 * MiB) -> list[int]:
    """cfg4 sizes: floor(exp(U(ln lo, ln hi))), U from SplitMix64(seed)."""
    x, out = seed, []
    a, b = math.log(lo), math.log(hi)
    for _ in range(n):
        x = (x + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        z ^= z >> 31
        u = (z >> 11) * (1.0 / (1 << 53))
        out.append(min(hi, max(lo, int(math.floor(math.exp(a + u * (b - a)))))))
    return out


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    p.add_argument("--objects", type=int, default=None, help="override object count per rank")
    p.add_argument("--ring-gib", type=float, default=80.0,
                   help="device output ring per GPU (objects wrap when the step exceeds it)")
    p.add_argument("--waves-per-block", type=int, default=None, help="1, 2 or 4 (default 2)")
    p.add_argument("--stream-tiles", type=int, default=-1,
                   help="1: uniform streams through the tiled batch kernel, 0: 2D stream kernel, -1: library default")
    p.add_argument("--store", choices=["default", "plain", "nt", "sc1", "ntsc1"], default="default",
                   help="fill-kernel store cache policy (default: library's, nt sc1 stream / sc1 batch)")
    p.add_argument("--occupancy", type=int, default=None,
                   help="resident fill workgroups per CU cap (default: library's, 14 stream / none batch)")
    p.add_argument("--prefetch", type=int, default=None,
                   help="batch tile-record prefetch distance in 64-block units (default: library's, 256)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-d2h", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--device-override", type=int, default=None,
                   help="rehearsal only: put every rank on this device (e.g. 2 ranks on a 1-GPU box)")
    return p.parse_args()


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def launch_ranks(n: int) -> int:
    """`--gpus N` outside torch.distributed.run: start the N ranks as a child
    torch.distributed.run (one process per GPU) and return its exit code.
    Nothing here has touched the GPU."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main() -> int:
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus)
    import torch
    from s3dlio_amd import Context, compress_ratio, object_entropy
    from s3dlio_amd._lib import ObjDesc, lib, call
    from s3dlio_amd.shard import ControlPlane, object_range

    cp = ControlPlane()
    rank, world = cp.rank, cp.world
    dev = cp.local_rank if args.device_override is None else args.device_override
    torch.cuda.set_device(dev)
    cfg = CONFIGS[args.config]
    ctx = Context(dev, base_seed=BASE_SEED, waves_per_block=args.waves_per_block)
    store = {"default": -1, "plain": 0, "nt": 1, "sc1": 2, "ntsc1": 3}[args.store]
    ctx.set_store_policy(store, store)
    ctx.set_stream_tiles(args.stream_tiles)
    if args.occupancy is not None:
        ctx.set_occupancy(args.occupancy, args.occupancy)
    if args.prefetch is not None:
        ctx.set_batch_prefetch(args.prefetch)
    stream = torch.cuda.current_stream()
    sh = int(stream.cuda_stream)
    fn, fd = compress_ratio(cfg["compress"])

    # ---- this rank's objects -------------------------------------------------------
    if cfg["scaling"] == "strong":
        n_total = args.objects or cfg["n"]
        lo, hi = object_range(n_total, rank, world)
    else:
        n_rank = args.objects or cfg["n"]
        lo, hi = rank * n_rank, (rank + 1) * n_rank
    n_rank = hi - lo
    ring_cap = int(args.ring_gib * GiB)

    launches = []      # (kind, args...) executed per step, all on `sh`
    slot_obj = {}      # ring slot -> (obj index, size, dst_off) of the last write, for verification
    if cfg["size"] is not None:
        size = cfg["size"]
        stride = (size + 4095) // 4096 * 4096
        ring_objs = max(1, min(n_rank, ring_cap // stride))
        ring = torch.empty(ring_objs * stride, dtype=torch.uint8, device=f"cuda:{dev}")
        if cfg.get("keystream"):
            # chunk index space continues across ranks: seed_base = first chunk of the rank
            for s0 in range(0, n_rank, ring_objs):
                k = min(ring_objs, n_rank - s0)
                launches.append(("keystream", k * stride, (lo + s0) * stride // (2 * MiB)))
                slot_obj = {t: (lo + s0 + t, size, t * stride) for t in range(k)}
        for s0 in ([] if cfg.get("keystream") else range(0, n_rank, ring_objs)):
            k = min(ring_objs, n_rank - s0)
            launches.append(("stream", size, stride, k, lo + s0))
            for s in range(k):
                slot_obj[s] = (lo + s0 + s, size, s * stride)
        step_bytes = n_rank * size
    else:
        sizes = ([cfg["uniform"]] * n_rank) if cfg.get("uniform") else log_uniform_sizes(lo + n_rank)[lo:]
        offs, cur, batch_start, batches = [], 0, 0, []
        for j, sz in enumerate(sizes):
            st = (sz + 4095) // 4096 * 4096
            if cur + st > ring_cap and cur > 0:
                batches.append((batch_start, j, offs))
                batch_start, cur, offs = j, 0, []
            offs.append(cur)
            cur += st
        batches.append((batch_start, len(sizes), offs))
        ring_bytes = max(sum((s + 4095) // 4096 * 4096 for s in sizes[b0:b1]) for b0, b1, _ in batches)
        ring = torch.empty(ring_bytes, dtype=torch.uint8, device=f"cuda:{dev}")
        for b0, b1, o in batches:
            arr = (ObjDesc * (b1 - b0))()
            for k in range(b1 - b0):
                j = lo + b0 + k
                arr[k] = ObjDesc(o[k], sizes[b0 + k], object_entropy(SEED_BASE, j), cfg["dedup"], fn, fd)
                slot_obj[o[k]] = (j, sizes[b0 + k], o[k])
            launches.append(("batch", arr, b1 - b0))
        step_bytes = sum(sizes)
    base_ptr = int(ring.data_ptr())
    # large uniform streams run through the tiled batch kernel unless --stream-tiles 0
    # (s3dg_set_stream_tiles; 8 MiB objects are 32 KiB-aligned to each other)
    tiled = (cfg["size"] is not None and not cfg.get("keystream") and args.stream_tiles != 0
             and all(L[0] == "stream" and L[3] * ((L[1] + 4095) // 4096) >= 16384 for L in launches))
    batch = cfg["size"] is None or tiled
    if cfg.get("keystream"):
        launch_shape = ("k_keystream<64,4>: 128 lanes x 2048 draws per 2 MiB chunk (jump-ahead), "
                        "64-draw LDS stage per lane, 512-B row pieces per store")
    else:
        waves = args.waves_per_block or (1 if batch else 2)
        launch_shape = (f"one {64 * waves}-thread workgroup per 4 KiB block, "
                        f"{ctx.query_occupancy(batch=batch)} resident per CU")

    def step(evs=None):
        for L in launches:
            if evs is not None:
                evs.append(torch.cuda.Event(enable_timing=True))
                evs[-1].record(stream)
            if L[0] == "keystream":
                call("s3dg_xoshiro_fill", ctx._h, base_ptr, L[1], 2 * MiB, L[2], sh)
            elif L[0] == "stream":
                _, size, stride, k, first = L
                call("s3dg_fill_controlled_stream", ctx._h, base_ptr, size, stride, k,
                     cfg["dedup"], fn, fd, SEED_BASE, first, sh)
            else:
                call("s3dg_fill_controlled_batch", ctx._h, base_ptr, L[1], L[2], sh)
            if evs is not None:
                evs.append(torch.cuda.Event(enable_timing=True))
                evs[-1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    cp.barrier()
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(evs)
    torch.cuda.synchronize()
    cp.barrier()
    t1 = time.perf_counter()
    elapsed = cp.max(t1 - t0)
    kern_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(0, len(evs), 2)]
    launch_bytes = [step_bytes / len(launches)] * len(kern_ms)   # uniform split (exact for one launch)
    if len(launches) > 1 and cfg["size"] is None:
        per = [sum(L[1][k].size for k in range(L[2])) for L in launches]
        launch_bytes = per * args.steps
    elif len(launches) > 1:
        per = [L[1] if L[0] == "keystream" else L[3] * L[1] for L in launches]
        launch_bytes = per * args.steps
    avg_ms = sum(kern_ms) / len(kern_ms)
    achieved_gbs = sum(launch_bytes) / (sum(kern_ms) * 1e-3) / 1e9

    total_bytes = cp.sum(step_bytes) * args.steps
    value = total_bytes / elapsed / GiB

    # ---- verification: sampled ring slots vs the C oracle -------------------------------
    verified = None
    if not args.no_verify:
        from oracle import oracle_c as OC
        import random
        base = OC.base_block(BASE_SEED)
        slots = sorted(slot_obj)
        rnd = random.Random(1234 + rank)
        pick = {slots[0], slots[-1]} | set(rnd.sample(slots, min(16, len(slots))))
        ok = True
        for s in sorted(pick):
            j, size, off = slot_obj[s]
            if cfg.get("keystream"):
                last = launches[-1]
                chunk0 = last[2] + s * 4           # 4 x 2 MiB chunks per 8 MiB slot
                got = ring[off:off + 2 * MiB].cpu().numpy()
                exp = OC.xoshiro_chunks(2 * MiB, 2 * MiB, chunk0)
                ok &= sha(got) == sha(exp)
                continue
            got = ring[off:off + size].cpu().numpy()
            exp = OC.fill_controlled(size, cfg["dedup"], fn, fd, object_entropy(SEED_BASE, j), base)
            ok &= sha(got) == sha(exp)
        verified = bool(cp.max(0.0 if ok else 1.0) == 0.0)
        if not verified:
            print("bench: VERIFICATION FAILED: sampled objects differ from the oracle", file=sys.stderr)

    # ---- write-only ceiling on the same buffer -----------------------------------------
    # a store-only kernel (one 4 KiB chunk per workgroup, 16-byte stores) in the
    # stream fill kernel's launch shape and in the shapes that measured fastest
    # for pure stores on MI355X (tools/batch_lab.py); the largest is the ceiling
    ceil_bytes = min(int(ring.numel()), 16 * GiB) // 4096 * 4096

    def ceiling_rate(fn=None):
        fn = fn or ctx.write_ceiling
        fn(ring, ceil_bytes, stream=stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(3):
            fn(ring, ceil_bytes, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        return 3 * ceil_bytes / (e0.elapsed_time(e1) * 1e-3) / 1e9
    ceil_shapes = {}
    names = {-1: "default", 0: "plain", 1: "nt", 2: "sc1", 3: "ntsc1"}
    for waves, occ, sp in [(args.waves_per_block or 2, -1 if args.occupancy is None else args.occupancy, store),
                           (4, 4, 2), (4, 3, 2), (2, 4, 2), (4, 0, 0), (4, 4, 0)]:
        ctx.set_waves_per_block(waves)
        ctx.set_occupancy(occ, occ)
        ctx.set_store_policy(sp, sp)
        ceil_shapes[f"{waves}w_{ctx.query_occupancy()}perCU_{names[sp]}"] = round(ceiling_rate(), 1)
    # the tiled fill's shape: batch knobs (1 wave, uncapped, sc1) + trailing record loads
    ctx.set_waves_per_block(args.waves_per_block or 0)
    ctx.set_occupancy(-1 if args.occupancy is None else args.occupancy, -1 if args.occupancy is None else args.occupancy)
    ctx.set_store_policy(store, store)
    ceil_shapes[f"tiled_1w_{ctx.query_occupancy(batch=True)}perCU_{names[store]}"] = round(
        ceiling_rate(ctx.write_ceiling_tiled), 1)
    # the runtime's own fill (SURVEY.md §8d names it as a ceiling option)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]

    def memset_d32(buf, nbytes, stream):
        sh = int(getattr(stream, "cuda_stream", stream or 0))
        assert hip.hipMemsetD32Async(buf.data_ptr(), 0x5A5A5A5A, nbytes // 4, sh) == 0
    ceil_shapes["hipMemsetD32Async"] = round(ceiling_rate(memset_d32), 1)
    ceiling_gbs = max(ceil_shapes.values())
    ctx.set_waves_per_block(args.waves_per_block or 0)
    occ = -1 if args.occupancy is None else args.occupancy
    ctx.set_occupancy(occ, occ)

    # ---- D2H-inclusive rate (bounded sample; never `value`) -------------------------------
    d2h = None
    if not args.no_d2h and cfg["size"] is not None:
        d2h = d2h_inclusive(torch, ctx, lib, call, dev, cfg, fn, fd, lo)
        # every rank measures at the same time: the aggregate is what the node moves
        d2h["aggregate_all_ranks"] = round(cp.sum(d2h["value"]), 2)

    # ---- CPU baseline (rank 0, N=1 only) ------------------------------------------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not cfg.get("keystream"):
        if cfg["size"] is not None:
            cpu = cpu_baseline(cfg, fn, fd, args.cpu_seconds)
        else:
            cpu = cpu_baseline_batch(cfg, fn, fd, args.cpu_seconds, sizes)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": cfg["scaling"],
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded: seed_base=0x5EED000000000001, base block seed 0xBA5EB10C00000000)",
            "config": {"workload": cfg["name"], "objects_per_rank": n_rank,
                       "bytes_per_step_all_ranks": int(total_bytes // args.steps),
                       "dedup": cfg["dedup"], "compress": list(cfg["compress"]) if isinstance(cfg["compress"], tuple) else cfg["compress"],
                       "launches_per_step": len(launches), "parallelism": f"object-stream x{world}",
                       "stores": (args.store if args.store != "default"
                                  else ("sc1" if batch else "nt sc1"))},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                         "traffic": traffic_from_profiles(args.config, int(sum(launch_bytes) / len(launch_bytes))),
                         "kernel": "k_keystream" if cfg.get("keystream") else (
                             "k_fill_batch" + (" (uniform tile records)" if tiled else "") if batch else "k_fill_stream"),
                         "launch_shape": launch_shape,
                         "avg_launch_ms": round(avg_ms, 3),
                         "algorithmic_bytes_per_launch": int(sum(launch_bytes) / len(launch_bytes)),
                         "write_ceiling_GBps": round(ceiling_gbs, 1),
                         "write_ceiling_shapes_GBps": ceil_shapes,
                         "frac_of_write_ceiling": round(achieved_gbs / ceiling_gbs, 4)},
            "cpu_baseline": cpu,
            "d2h_inclusive": d2h,
            "verified_vs_oracle": verified,
        }
        print(json.dumps(out), flush=True)
    cp.close()
    return 0


def traffic_from_profiles(config: int, launch_bytes: int):
    """HBM bytes per launch from the committed PMC pass (profiles/traffic.json),
    only when it was taken on this exact config and launch size."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(p) as f:
            t = json.load(f).get(str(config))
        if t and t.get("algorithmic_bytes_per_launch") == launch_bytes:
            return t.get("traffic_bytes_per_launch")
    except Exception:
        pass
    return None


def d2h_inclusive(torch, ctx, lib, call, dev, cfg, fn, fd, lo, n_objs=1024, per_chunk=32):
    """Generate n_objs objects through two device chunk buffers and copy each
    chunk to a pinned host ring on the GPU's NUMA node, on a second stream
    (the PUT path's input)."""
    import ctypes
    size = cfg["size"]
    cb = per_chunk * size
    gen = torch.cuda.Stream(device=dev)
    cpy = torch.cuda.Stream(device=dev)
    devbuf = [torch.empty(cb, dtype=torch.uint8, device=f"cuda:{dev}") for _ in range(2)]
    host = []
    for _ in range(2):
        p = ctypes.c_void_p()
        call("s3dg_host_alloc_pinned_local", dev, cb, ctypes.byref(p))
        host.append(p.value)
    node = ctypes.c_int(-1)
    call("s3dg_device_numa_node", dev, ctypes.byref(node))
    gen_done = [torch.cuda.Event() for _ in range(2)]
    cpy_done = [torch.cuda.Event() for _ in range(2)]

    def run(n):
        for k in range(n // per_chunk):
            s = k & 1
            gen.wait_event(cpy_done[s])
            call("s3dg_fill_controlled_stream", ctx._h, int(devbuf[s].data_ptr()), size, size,
                 per_chunk, cfg["dedup"], fn, fd, SEED_BASE, lo + k * per_chunk,
                 int(gen.cuda_stream))
            gen_done[s].record(gen)
            cpy.wait_event(gen_done[s])
            call("s3dg_d2h_async", ctx._h, host[s], int(devbuf[s].data_ptr()), cb, int(cpy.cuda_stream))
            cpy_done[s].record(cpy)
    try:
        for s in range(2):
            cpy_done[s].record(cpy)
        run(n_objs // 2)          # the first GiBs into fresh pinned pages copy slower
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(n_objs)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        torch.cuda.synchronize()
        for p in host:
            call("s3dg_host_free_pinned", p)
    return {"value": round(n_objs * size / dt / GiB, 2), "unit": "GiB/s",
            "sample": f"{n_objs} x {size // MiB} MiB objects, 2 x {per_chunk}-object device chunks, "
                      f"pinned host ring on NUMA node {node.value}, generate || D2H on two streams"}


def cpu_baseline_batch(cfg, fn, fd, seconds, sizes):
    """Mixed-size configs: the C restatement per object (s3dgo_fill_controlled),
    objects spread over a pool of host threads.  Each thread writes its objects
    one after another into its own 256 MiB host ring (wrapping), so the bytes
    stream to DRAM as the GPU's do to HBM instead of staying in the caches."""
    import ctypes
    import threading
    import numpy as np
    from oracle import oracle_c as OC
    threads = max(1, min(16, os.cpu_count() or 1))
    base = OC.base_block(BASE_SEED)
    L = OC.lib()
    ring = max(256 * MiB, max(sizes))
    lock = threading.Lock()
    state = {"next": 0, "bytes": 0, "objs": 0, "stop": False}
    start = threading.Event()

    def worker():
        buf = np.ones(ring, np.uint8)                     # faulted in before timing starts
        addr = buf.ctypes.data
        pp = base.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        done = nobj = pos = 0
        start.wait()
        while not state["stop"]:
            with lock:
                j = state["next"]
                state["next"] += 1
            sz = sizes[j % len(sizes)]
            if pos + sz > ring:
                pos = 0
            L.s3dgo_fill_controlled(ctypes.cast(addr + pos, ctypes.POINTER(ctypes.c_uint8)), sz, cfg["dedup"],
                                    fn, fd, object_entropy_py(SEED_BASE, j), pp)
            pos += (sz + 4095) // 4096 * 4096
            done += sz
            nobj += 1
        with lock:
            state["bytes"] += done
            state["objs"] += nobj
    ts = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ts:
        t.start()
    time.sleep(1.0)                                       # rings allocated and touched
    t0 = time.perf_counter()
    start.set()
    time.sleep(seconds)
    state["stop"] = True
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": round(state["bytes"] / dt / GiB, 2), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{state['objs']} objects of the config's sizes ({state['bytes'] / GiB:.0f} GiB) over "
                      f"{dt:.1f} s, one object per task on {threads} threads, each thread writing a "
                      f"{ring // MiB} MiB host ring; {model}"}


def object_entropy_py(seed_base: int, j: int) -> int:
    return (seed_base + (j << 32)) & (2**64 - 1)


def cpu_baseline(cfg, fn, fd, seconds):
    """The C restatement (oracle, kind='port') on this host's cores, like the
    reference's Rayon par_chunks_mut(4096) (src/data_gen.rs:198)."""
    import numpy as np
    from oracle import oracle_c as OC
    threads = max(1, min(16, os.cpu_count() or 1))
    size = cfg["size"]
    per = max(1, (1 * GiB) // size)            # 1 GiB host ring, reused
    buf = np.zeros(per * size, np.uint8)
    buf[:] = 1                                   # fault the pages in before timing
    base = OC.base_block(BASE_SEED)
    OC.fill_stream(size, per, cfg["dedup"], fn, fd, SEED_BASE, 0, base, threads=threads, out=buf)
    done, t0, k = 0, time.perf_counter(), 0
    while True:
        OC.fill_stream(size, per, cfg["dedup"], fn, fd, SEED_BASE, k * per, base,
                       threads=threads, out=buf)
        done += per
        k += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    t1s = time.perf_counter()
    OC.fill_stream(size, per, cfg["dedup"], fn, fd, SEED_BASE, 0, base, threads=1, out=buf)
    one = per * size / (time.perf_counter() - t1s) / GiB
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": round(done * size / dt / GiB, 2), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"{done} x {size // MiB} MiB objects ({done * size / GiB:.0f} GiB) over "
                      f"{dt:.1f} s into a reused 1 GiB host ring; {model}",
            "single_thread_GiBps": round(one, 2)}


if __name__ == "__main__":
    sys.exit(main())

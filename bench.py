#!/usr/bin/env python3
"""bench.py — device-resident synthetic-payload GiB/s (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C]

A "step" is one pass of the hot path over one batch: every object of the
configuration generated once into HBM by the gfx950 kernel (src/data_gen.rs
fill_controlled_data semantics, one payload per object).  Default workload =
BASELINE config 2: 10 000 x 8 MiB objects, dedup=1, compress=1 per GPU.
N>1: launched by torch.distributed.run, one rank per GPU; each rank owns its
own object-index range (weak scaling, no data-path collective; a gloo
control plane does the barrier and the max over ranks).

Configs 2-5 are BASELINE.json's; the others measure the surfaces around the
path: 6 the K2 keystream (npz.rs:376-383), 7 config 2 through
the batch API, 8/9 config 1's 64 KiB objects on the GPU (stream / batch API),
10 small ragged objects through the batch API, 11-13 one
s3dg_fill_controlled call on a single 1/4/16 MiB buffer (the reference's own
criterion shape, benches/performance_microbenchmarks.rs:43-64), 14/15 the
DG1 byte path behind generate_data / Generator (one launch per object), 16/17
the same objects through s3dg_dgen_fill_stream (one launch per step), 18-22
the host-buffer drop-ins (the reference's own API: s3dlio_fill_controlled_data
on 1/4/16 MiB and 1 GiB host buffers from a native loop, generate_into_buffer
from 8 threads; --host-mem pageable|pinned; roofline bound = PCIe), 23-28 the
reference's streaming callers (ObjectGen::fill_chunk at 64 KiB / 256 KiB /
32 MiB over 8 MiB and 1 GiB objects from 8 threads).
--d2h-full: the D2H-inclusive rate over the rank's whole object range (config 5
as BASELINE states it), not an 8 GiB sample.

Prints ONE JSON line on rank 0 (contract in the task statement), including
`roofline` (kernel-event timing vs the 8 TB/s HBM peak; the fill's store-only
reference shapes beside it, which the fill beats) and `cpu_baseline` (the C
port of the same generator on this host's cores — rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

KiB = 1 << 10
MiB = 1 << 20
GiB = 1 << 30
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
SEED_BASE = 0x5EED000000000001
BASE_SEED = 0xBA5EB10C00000000
METRIC = "device-resident synthetic-payload GiB/s, 8 MiB objects, 1/2/4/8 MI355X"

CONFIGS = {
    2: dict(name="cfg2: 10000 x 8 MiB, dedup=1 compress=1 (pure fill)", kind="stream", n=10000,
            size=8 * MiB, dedup=1, compress=1, scaling="weak"),
    3: dict(name="cfg3: 10000 x 8 MiB, dedup=4 compress=2", kind="stream", n=10000, size=8 * MiB,
            dedup=4, compress=2, scaling="weak"),
    4: dict(name="cfg4: 10000 x log-uniform 4 KiB..64 MiB, dedup=2 compress=1.5", kind="batch", n=10000,
            size=None, dedup=2, compress=(3, 2), scaling="weak"),
    5: dict(name="cfg5: 100000 x 8 MiB, dedup=2 compress=3 (total over all GPUs)", kind="stream", n=100000,
            size=8 * MiB, dedup=2, compress=3, scaling="strong"),
    # not BASELINE configs: the surfaces around the path (module docstring)
    6: dict(name="k2: keystream fill, 10000 x 8 MiB as 2 MiB Xoshiro256++ chunks", kind="keystream", n=10000,
            size=8 * MiB, dedup=1, compress=1, scaling="weak"),
    7: dict(name="diag: cfg2 objects (10000 x 8 MiB, d1 c1) through the batch API", kind="batch", n=10000,
            size=None, uniform=8 * MiB, dedup=1, compress=1, scaling="weak"),
    8: dict(name="cfg1-shape: 1000000 x 64 KiB, dedup=1 compress=1, stream API", kind="stream", n=1000000,
            size=64 * KiB, dedup=1, compress=1, scaling="weak"),
    9: dict(name="cfg1-shape: 1000000 x 64 KiB, dedup=1 compress=1, batch API", kind="batch", n=1000000,
            size=None, uniform=64 * KiB, dedup=1, compress=1, scaling="weak"),
    10: dict(name="small: 2000000 x (20 KiB + 5 B), dedup=1 compress=1, batch API", kind="batch", n=2000000,
             size=None, uniform=20 * KiB + 5, dedup=1, compress=1, scaling="weak"),
    11: dict(name="single buffer: 1000 x s3dg_fill_controlled on one 1 MiB buffer, d1 c1", kind="single",
             n=1000, size=1 * MiB, dedup=1, compress=1, scaling="weak"),
    12: dict(name="single buffer: 1000 x s3dg_fill_controlled on one 4 MiB buffer, d1 c1", kind="single",
             n=1000, size=4 * MiB, dedup=1, compress=1, scaling="weak"),
    13: dict(name="single buffer: 1000 x s3dg_fill_controlled on one 16 MiB buffer, d1 c1", kind="single",
             n=1000, size=16 * MiB, dedup=1, compress=1, scaling="weak"),
    14: dict(name="dg1: 10 x 8 GiB DG1 objects (generate_data byte path), dedup=1 compress=1", kind="dgen",
             n=10, size=8 * GiB, dedup=1, compress=1, scaling="weak"),
    15: dict(name="dg1: 10 x 8 GiB DG1 objects (generate_data byte path), dedup=2 compress=2", kind="dgen",
             n=10, size=8 * GiB, dedup=2, compress=2, scaling="weak"),
    16: dict(name="dg1 stream: 10 x 8 GiB DG1 objects in one s3dg_dgen_fill_stream launch, dedup=1 compress=1",
             kind="dgen_stream", n=10, size=8 * GiB, dedup=1, compress=1, scaling="weak"),
    17: dict(name="dg1 stream: 10 x 8 GiB DG1 objects in one s3dg_dgen_fill_stream launch, dedup=2 compress=2",
             kind="dgen_stream", n=10, size=8 * GiB, dedup=2, compress=2, scaling="weak"),
    # the host-buffer drop-ins (the reference's own API: host memory in, host memory out)
    18: dict(name="host: 1000 x s3dlio_fill_controlled_data on one 1 MiB host buffer, d1 c1 (criterion shape)",
             kind="host", n=1000, size=1 * MiB, dedup=1, compress=1, scaling="weak"),
    19: dict(name="host: 500 x s3dlio_fill_controlled_data on one 4 MiB host buffer, d1 c1 (criterion shape)",
             kind="host", n=500, size=4 * MiB, dedup=1, compress=1, scaling="weak"),
    20: dict(name="host: 200 x s3dlio_fill_controlled_data on one 16 MiB host buffer, d1 c1 (criterion shape)",
             kind="host", n=200, size=16 * MiB, dedup=1, compress=1, scaling="weak"),
    21: dict(name="host: 8 x s3dlio_fill_controlled_data on one 1 GiB host buffer, d1 c1 (split over host slots)",
             kind="host", n=8, size=1 * GiB, dedup=1, compress=1, scaling="weak"),
    22: dict(name="host: generate_into_buffer (s3dg_generate_data) from 8 threads, 8 MiB each, 100 calls per thread",
             kind="host", n=100, size=8 * MiB, threads=8, dedup=1, compress=1, scaling="weak"),
    # the reference's streaming callers: ObjectGen::fill_chunk loops from 8 threads, one generator per object
    23: dict(name="chunks: ObjectGen::fill_chunk(64 KiB) over 8 MiB objects, 8 threads x 100 objects "
                  "(StreamingDataWriter::generate_remaining)", kind="host", n=100, size=8 * MiB, chunk=64 * KiB,
             threads=8, dedup=1, compress=1, scaling="weak"),
    24: dict(name="chunks: ObjectGen::fill_chunk(256 KiB) over 8 MiB objects, 8 threads x 100 objects "
                  "(Config::chunk_size)", kind="host", n=100, size=8 * MiB, chunk=256 * KiB, threads=8, dedup=1,
             compress=1, scaling="weak"),
    25: dict(name="chunks: ObjectGen::fill_chunk(32 MiB) over 8 MiB objects, 8 threads x 100 objects "
                  "(fill_remaining)", kind="host", n=100, size=8 * MiB, chunk=32 * MiB, threads=8, dedup=1,
             compress=1, scaling="weak"),
    26: dict(name="chunks: ObjectGen::fill_chunk(64 KiB) over 1 GiB objects, 8 threads x 1 object", kind="host",
             n=1, size=1 * GiB, chunk=64 * KiB, threads=8, dedup=1, compress=1, scaling="weak"),
    27: dict(name="chunks: ObjectGen::fill_chunk(256 KiB) over 1 GiB objects, 8 threads x 1 object", kind="host",
             n=1, size=1 * GiB, chunk=256 * KiB, threads=8, dedup=1, compress=1, scaling="weak"),
    28: dict(name="chunks: ObjectGen::fill_chunk(32 MiB) over 1 GiB objects, 8 threads x 1 object", kind="host",
             n=1, size=1 * GiB, chunk=32 * MiB, threads=8, dedup=1, compress=1, scaling="weak"),
}
PCIE_PEAK_GBS = 63.0    # PCIe Gen5 x16, one direction, before protocol overhead


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
    p.add_argument("--batch-tile", type=int, default=None, help="batch tile blocks (1 = dense; default: per launch)")
    p.add_argument("--pace", type=int, default=None,
                   help="batch kernel wall-clock store floor in 10-ns ticks (0 = off; default: per launch)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-no-pin", action="store_true",
                   help="leave the CPU baseline's threads to the scheduler (default: bound to the cgroup's share of "
                        "CPUs, GPU-local and idlest first)")
    p.add_argument("--legacy-stream", action="store_true",
                   help="launch on torch's default (legacy null) stream, as rounds 1-5 did")
    p.add_argument("--no-d2h", action="store_true")
    p.add_argument("--d2h-reps", type=int, default=1, help="D2H-inclusive samples (diagnosis of run-to-run spread)")
    p.add_argument("--d2h-full", action="store_true",
                   help="D2H-inclusive rate over the rank's WHOLE object range (SURVEY 8d: first launch to last "
                        "D2H completion), instead of an 8 GiB sample; reported beside the device-resident value")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--no-ceiling", action="store_true")
    p.add_argument("--host-mem", choices=["pageable", "pinned", "registered"], default="pageable",
                   help="host configs (18-22): the caller's buffer is pageable (a reused Vec / bytearray), pinned "
                        "by the library, or pageable and page-locked by s3dg_host_register")
    p.add_argument("--device-override", type=int, default=None,
                   help="rehearsal only: put every rank on this device (e.g. 8 ranks on a 1-GPU box)")
    return p.parse_args()


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def source_digest() -> str:
    """Digest of the library sources in this tree (s3dlio_amd/build.py's
    source_digest, loaded by path so the package is not imported): the
    library compiles the same digest in (s3dg_build_digest), and a traffic
    record (profiles/traffic.json) counts only for the same digest."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_s3dg_build", os.path.join(ROOT, "s3dlio_amd", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.source_digest()


def cpu_share() -> dict:
    """CPUs this process may use: scheduler affinity and the cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except Exception:
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except Exception:
            pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return {"threads": threads, "affinity_cpus": aff, "cgroup_quota_cpus": quota}


def cpu_model() -> str:
    try:
        return [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        return "unknown"


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
    from s3dlio_amd._lib import ObjDesc, call, lib
    from s3dlio_amd.shard import ControlPlane, object_range

    # the timed binary must be the one these sources build
    lib_digest = (lib.s3dg_build_digest() or b"").decode()
    src_digest = source_digest()
    if lib_digest != src_digest:
        print(f"bench: the loaded library ({lib._name}) was built from sources {lib_digest}, this tree is "
              f"{src_digest}: rebuild (python s3dlio_amd/build.py) before measuring", file=sys.stderr)
        return 3
    cp = ControlPlane()
    rank, world = cp.rank, cp.world
    dev = cp.local_rank if args.device_override is None else args.device_override
    torch.cuda.set_device(dev)
    cfg = CONFIGS[args.config]
    kind = cfg["kind"]
    ctx = Context(dev, base_seed=BASE_SEED, waves_per_block=args.waves_per_block)
    store = {"default": -1, "plain": 0, "nt": 1, "sc1": 2, "ntsc1": 3}[args.store]
    ctx.set_store_policy(store, store)
    ctx.set_stream_tiles(args.stream_tiles)
    if args.occupancy is not None:
        ctx.set_occupancy(args.occupancy, args.occupancy)
    if args.prefetch is not None:
        ctx.set_batch_prefetch(args.prefetch)
    if args.batch_tile is not None:
        ctx.set_batch_tile(args.batch_tile)
    if args.pace is not None:
        ctx.set_batch_pace(args.pace)
    # every launch on a (non-blocking) stream of torch's pool, not the legacy
    # default stream, whose launches HIP orders against every blocking stream
    # (the single-call configs 11-13 paid ~0.8 us per call for it)
    if not args.legacy_stream:
        torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    stream = torch.cuda.current_stream()
    sh = int(stream.cuda_stream)
    fn, fd = compress_ratio(cfg["compress"])
    d = cfg["dedup"]

    # ---- this rank's objects -------------------------------------------------------
    if cfg["scaling"] == "strong":
        lo, hi = object_range(args.objects or cfg["n"], rank, world)
    else:
        n_rank = args.objects or cfg["n"]
        lo, hi = rank * n_rank, (rank + 1) * n_rank
    n_rank = hi - lo
    ring_cap = int(args.ring_gib * GiB)

    launches = []      # (callable, algorithmic bytes) per launch, all on `sh`
    samples = []       # (ring offset, check) of the step's last writes, for verification
    sizes = None
    if kind in ("stream", "keystream"):
        size = cfg["size"]
        stride = (size + 4095) // 4096 * 4096
        ring_objs = even_ring(n_rank, ring_cap // stride)
        ring = torch.empty(ring_objs * stride, dtype=torch.uint8, device=f"cuda:{dev}")
        base_ptr = int(ring.data_ptr())
        for s0 in range(0, n_rank, ring_objs):
            k = min(ring_objs, n_rank - s0)
            if kind == "keystream":
                # chunk index space continues across ranks: seed_base = first chunk of the rank
                c0 = (lo + s0) * stride // (2 * MiB)
                launches.append((lambda k=k, c0=c0: call("s3dg_xoshiro_fill", ctx._h, base_ptr, k * stride,
                                                         2 * MiB, c0, sh), k * size))
                samples = [(t * stride, ("chunk", c0 + t * stride // (2 * MiB))) for t in range(k)]
            else:
                launches.append((lambda k=k, first=lo + s0: call(
                    "s3dg_fill_controlled_stream", ctx._h, base_ptr, size, stride, k, d, fn, fd, SEED_BASE,
                    first, sh), k * size))
                samples = [(t * stride, ("obj", lo + s0 + t, size)) for t in range(k)]
        step_bytes = n_rank * size
    elif kind == "batch":
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
        base_ptr = int(ring.data_ptr())
        for b0, b1, o in batches:
            arr = (ObjDesc * (b1 - b0))()
            for k in range(b1 - b0):
                arr[k] = ObjDesc(o[k], sizes[b0 + k], object_entropy(SEED_BASE, lo + b0 + k), d, fn, fd)
            launches.append((lambda arr=arr, m=b1 - b0: call("s3dg_fill_controlled_batch", ctx._h, base_ptr, arr, m,
                                                             sh), sum(sizes[b0:b1])))
            # the last batch overwrites the ring: only its objects are checkable
            samples = [(o[k], ("obj", lo + b0 + k, sizes[b0 + k])) for k in range(b1 - b0)]
        step_bytes = sum(sizes)
    elif kind == "single":
        size = cfg["size"]
        ring = torch.empty(size, dtype=torch.uint8, device=f"cuda:{dev}")
        base_ptr = int(ring.data_ptr())
        calls = args.objects or cfg["n"]
        # the calls come from a native loop (tools/native_loop.c), as the
        # reference's criterion loop calls from Rust; the Python-loop rate is
        # reported beside it (single_call)
        nl = ctypes.CDLL(os.path.join(ROOT, "tools", "_native", "libnative_loop.so"))
        u64, u32, vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p
        nl.nl_fill_loop.restype = ctypes.c_int
        nl.nl_fill_loop.argtypes = [vp, vp, vp, u64, u64, u64, u32, u32, u64, vp]
        fill_ptr = ctypes.cast(lib.s3dg_fill_controlled, vp)

        def single_step(size=size, calls=calls):
            r = nl.nl_fill_loop(fill_ptr, ctx._h, base_ptr, size, calls, d, fn, fd, 7, sh)
            if r:
                raise RuntimeError(f"s3dg_fill_controlled failed in the native loop ({r})")

        def single_step_py(size=size, calls=calls):
            for _ in range(calls):
                call("s3dg_fill_controlled", ctx._h, base_ptr, size, d, fn, fd, 7, sh)
        launches.append((single_step, calls * size))
        samples = [(0, ("single", size))]
        step_bytes = calls * size
    elif kind == "host":
        # synchronous host-buffer calls from a native loop; the work runs on
        # the library's host slots (S3DLIO_GPU_DEVICE(S)), timed by wall clock
        size, calls, nthr = cfg["size"], args.objects or cfg["n"], cfg.get("threads", 1)
        nl = ctypes.CDLL(os.path.join(ROOT, "tools", "_native", "libnative_loop.so"))
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        nl.nl_host_fill_loop.argtypes = [vp, vp, u64, u64, u64, u64]
        nl.nl_threads_gen_loop.argtypes = [vp, ctypes.POINTER(vp), u64, ctypes.c_int, u64, u64, u64]
        chunk = cfg.get("chunk")
        hbufs = [host_buffer(chunk or size, args.host_mem, call) for _ in range(nthr)]
        ring = None
        if chunk:
            nl.nl_threads_chunk_loop.argtypes = [vp, vp, vp, ctypes.POINTER(vp), ctypes.c_int, u64, u64, u64, u64,
                                                 u64, u64, ctypes.POINTER(u64)]
            fns = [ctypes.cast(getattr(lib, f), vp) for f in ("s3dg_gen_create", "s3dg_gen_fill_chunk",
                                                               "s3dg_gen_destroy")]
            arr = (vp * nthr)(*[b for b, _ in hbufs])
            made = ctypes.c_uint64()

            def host_step():
                r = nl.nl_threads_chunk_loop(*fns, arr, nthr, size, chunk, calls, d, cfg["compress"], SEED_BASE,
                                             ctypes.byref(made))
                if r or made.value != nthr * calls * size:
                    raise RuntimeError(f"fill_chunk loop failed ({r}, {made.value} bytes): "
                                       f"{lib.s3dg_last_error().decode()}")
        elif nthr == 1:
            fptr = ctypes.cast(lib.s3dlio_fill_controlled_data, vp)

            def host_step(b=hbufs[0][0]):
                r = nl.nl_host_fill_loop(fptr, b, size, calls, d, cfg["compress"])
                if r:
                    raise RuntimeError(f"s3dlio_fill_controlled_data failed ({r}): {lib.s3dg_last_error().decode()}")
        else:
            gptr = ctypes.cast(lib.s3dg_generate_data, vp)
            arr = (vp * nthr)(*[b for b, _ in hbufs])

            def host_step():
                r = nl.nl_threads_gen_loop(gptr, arr, size, nthr, calls, d, cfg["compress"])
                if r:
                    raise RuntimeError(f"s3dg_generate_data failed ({r}): {lib.s3dg_last_error().decode()}")
        launches.append((host_step, calls * nthr * size))
        samples = [(0, ("host", size, nthr))]
        step_bytes = calls * nthr * size
    elif kind == "dgen_stream":   # DG1 objects, one launch per ring pass
        size = cfg["size"]
        ring_objs = even_ring(n_rank, ring_cap // size)
        ring = torch.empty(ring_objs * size, dtype=torch.uint8, device=f"cuda:{dev}")
        base_ptr = int(ring.data_ptr())
        for s0 in range(0, n_rank, ring_objs):
            k = min(ring_objs, n_rank - s0)
            launches.append((lambda k=k, first=lo + s0: call("s3dg_dgen_fill_stream", ctx._h, base_ptr, size, size,
                                                             k, d, fn, fd, SEED_BASE, first, sh), k * size))
            samples = [(t * size, ("dgen", lo + s0 + t)) for t in range(k)]
        step_bytes = n_rank * size
    else:   # dgen
        size = cfg["size"]
        ring_objs = max(1, min(n_rank, ring_cap // size))
        ring = torch.empty(ring_objs * size, dtype=torch.uint8, device=f"cuda:{dev}")
        base_ptr = int(ring.data_ptr())
        for j in range(n_rank):
            t = j % ring_objs
            launches.append((lambda t=t, j=lo + j: call("s3dg_dgen_fill", ctx._h, base_ptr + t * size, size, 0,
                                                        1 << 40, d, fn, fd, object_entropy(SEED_BASE, j), sh),
                             size))
        samples = [((j % ring_objs) * size, ("dgen", lo + j)) for j in range(max(0, n_rank - ring_objs), n_rank)]
        step_bytes = n_rank * size

    # kernel and launch shape of the dominant launch
    tiled = (kind == "stream" and args.stream_tiles != 0
             and all(b // cfg["size"] * ((cfg["size"] + 4095) // 4096) >= 16384 for _, b in launches)
             and cfg["size"] % (32 * KiB) == 0)
    if kind == "host" and cfg.get("chunk"):
        kernel, launch_shape = (
            "k_keystream (DG1) into the generators' pinned read-ahead rings (chunks below a ring half) or "
            "+ hipMemcpyAsync D2H on the host slots' staging streams (larger chunks)"), (
            f"{cfg['threads']} caller threads, one generator per {cfg['size'] // MiB} MiB object, "
            f"fill_chunk({cfg['chunk'] // KiB} KiB) into a reused {args.host_mem} buffer per thread, slots "
            f"{os.environ.get('S3DLIO_GPU_DEVICES') or os.environ.get('S3DLIO_GPU_DEVICE') or 'every visible GPU'}, "
            f"ring half {os.environ.get('S3DLIO_GEN_RING_HALF_MIB', '4')} MiB")
    elif kind == "host":
        kernel, launch_shape = ("k_fill_stream + hipMemcpyAsync D2H on the host slots' staging streams"
                                if cfg.get("threads", 1) == 1 else
                                "k_keystream (DG1) + hipMemcpyAsync D2H on the host slots' staging streams"), (
            f"{cfg.get('threads', 1)} caller thread(s), {args.host_mem} host buffer, slots "
            f"{os.environ.get('S3DLIO_GPU_DEVICES') or os.environ.get('S3DLIO_GPU_DEVICE') or 'every visible GPU'}, "
            f"D2H mode {os.environ.get('S3DLIO_HOST_D2H', 'direct')}")
    elif kind == "keystream":
        kernel, launch_shape = "k_keystream", ("k_keystream<64,1>: 64 lanes x 4096 draws per 2 MiB chunk "
                                               "(jump-ahead, state sequence on the scalar unit), 64-draw LDS stage "
                                               "per lane, 512-B row pieces per store, 1-wave workgroups in XCD "
                                               "groups of 16; a persistent grid over per-XCD unit queues from 6 "
                                               "rounds of resident waves up")
    elif kind in ("dgen", "dgen_stream"):
        kernel, launch_shape = ("k_zero_prefix + k_keystream (DG1 tails)" if fn else "k_keystream (DG1 mode)"), (
            ("k_zero_prefix: each 1 MiB DG1 block's whole 4 KiB granules of zeros in the fill's store shape "
             "(prefixes on a 64-B line: 4-wave workgroups, 5 per CU, nt sc1, before the tails; mid-line: 1-wave, "
             "14 per CU, on a side stream beside them), then k_keystream<64,1> over the blocks' tails (64 lanes "
             "per tail, jump state sequence on the scalar unit, the rest of the prefix zeroed in the lane rows)"
             if fn else
             "k_keystream<64,1>: 2048 draws per lane, 64 lanes per 1 MiB DG1 block, jump state sequence on the "
             "scalar unit, XCD groups of 16 waves, a persistent grid over per-XCD unit queues from 6 rounds of "
             "resident waves up")
            + ("; all objects of the step in one launch" if kind == "dgen_stream" else "; one launch per object"))
    else:
        batch = kind == "batch" or tiled
        kernel = ("k_fill_batch" + (" (uniform tile records)" if tiled else "")) if batch else "k_fill_stream"
        waves = args.waves_per_block or (1 if batch else 2)
        launch_shape = (f"one {64 * waves}-thread workgroup per 4 KiB block, "
                        f"{ctx.query_occupancy(batch=batch)} resident per CU")

    # first touch of the output ring before the warm-up steps (untimed setup):
    # a process's first fill of freshly allocated HBM ran 13.7 ms against
    # 11.1 (profiles/r05/kernel_stats_cfg2.csv), which only the rocprof
    # averages (they include the warm-up launches) ever saw
    if ring is not None:
        ring.zero_()
        torch.cuda.synchronize()

    # per-launch HIP events on the launch stream (the single-buffer step is one group)
    def step(evs=None):
        for f, _ in launches:
            if evs is not None:
                evs.append(torch.cuda.Event(enable_timing=True))
                evs[-1].record(stream)
            f()
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
    if kind == "host":     # synchronous calls on the library's own streams: wall clock
        kern_ms = [(t1 - t0) * 1e3 / args.steps] * args.steps
    launch_bytes = [b for _, b in launches] * args.steps
    avg_ms = sum(kern_ms) / len(kern_ms)
    achieved_gbs = sum(launch_bytes) / (sum(kern_ms) * 1e-3) / 1e9
    if kind in ("single", "host"):             # one "launch" = one call
        avg_ms /= launches[0][1] // cfg["size"]
    algo_per_launch = int(sum(launch_bytes) / len(launch_bytes))
    if kind in ("single", "host"):
        algo_per_launch = cfg["size"]
    if kind == "host" and cfg.get("chunk"):   # one "call" = one fill_chunk
        avg_ms = avg_ms * min(cfg["chunk"], cfg["size"]) / cfg["size"]
        algo_per_launch = min(cfg["chunk"], cfg["size"])

    total_bytes = cp.sum(step_bytes) * args.steps
    value = total_bytes / elapsed / GiB

    single_call = None
    if kind == "single":   # the same calls from a Python loop (ctypes), once, for comparison
        single_step_py()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream); single_step_py(); e1.record(stream); torch.cuda.synchronize()
        py_s = e0.elapsed_time(e1) * 1e-3
        single_call = {"caller": "native loop (tools/native_loop.c) over the C ABI",
                       "us_per_call": round(avg_ms * 1e3, 3),
                       "python_loop_us_per_call": round(py_s / calls * 1e6, 3),
                       "python_loop_GBps": round(calls * cfg["size"] / py_s / 1e9, 1)}

    # ---- verification: sampled objects of the last writes vs the C oracle ---------------
    verified = None
    if not args.no_verify:
        verified = (verify_host(hbufs, cfg, fn, fd, call, cp) if kind == "host"
                    else verify(torch, ring, samples, cfg, fn, fd, rank, cp))

    # ---- write ceilings on the same buffer ----------------------------------------------
    ceil = None
    if not args.no_ceiling and kind in ("stream", "batch", "keystream"):
        ceil = ceilings(torch, ctx, ring, stream, args, store)
        ctx.set_waves_per_block(args.waves_per_block or 0)
        occ = -1 if args.occupancy is None else args.occupancy
        ctx.set_occupancy(occ, occ)
        ctx.set_store_policy(store, store)

    # ---- D2H-inclusive rate (bounded sample; never `value`) -------------------------------
    d2h = None
    if not args.no_d2h and kind in ("stream", "keystream", "dgen", "dgen_stream"):
        cp.barrier()
        reps = [d2h_inclusive(torch, ctx, call, dev, cfg, fn, fd, lo, n_objs=n_rank if args.d2h_full else None)
                for _ in range(max(1, args.d2h_reps))]
        d2h = reps[-1]
        if len(reps) > 1:
            d2h["all_samples_GiBps"] = [r["value"] for r in reps]
        # every rank measures at the same time: the aggregate is what the node moves
        d2h["aggregate_all_ranks"] = round(cp.sum(d2h["value"]), 2)
        if args.d2h_full:
            # whole job: every rank's bytes over the slowest rank's first-launch-to-last-copy time
            d2h["whole_job_GiBps"] = round(cp.sum(d2h["bytes"]) / cp.max(d2h["seconds"]) / GiB, 2)
            d2h["verified_vs_oracle"] = bool(cp.max(0.0 if d2h["verified_vs_oracle"] else 1.0) == 0.0)

    # every rank's object range and device (disjoint ranges: no object written twice)
    rank_map = cp.gather({"rank": rank, "device": dev, "object_range": [lo, hi]})

    # ---- CPU baseline (rank 0, N=1 only) ------------------------------------------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, fn, fd, args.cpu_seconds, sizes, dev=dev, pin=not args.cpu_no_pin)

    if rank == 0:
        if kind == "host":
            # the host-buffer path is bound by the PCIe link, not HBM
            roof = {"bound": "pcie", "achieved": round(achieved_gbs, 1), "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved_gbs / PCIE_PEAK_GBS, 4), "traffic": None, "kernel": kernel,
                    "launch_shape": launch_shape, "avg_call_ms": round(avg_ms, 4),
                    "algorithmic_bytes_per_call": algo_per_launch, "host_mem": args.host_mem,
                    "source_digest": src_digest, "library_digest": lib_digest}
        else:
            roof = {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                    "traffic": traffic_from_profiles(args.config, algo_per_launch),
                    "kernel": kernel, "launch_shape": launch_shape,
                    "avg_launch_ms": round(avg_ms, 4),
                    "algorithmic_bytes_per_launch": algo_per_launch,
                    "launch_ms_distribution": launch_distribution(kern_ms, launch_bytes, len(launches)),
                    "source_digest": src_digest, "library_digest": lib_digest}
        if kind in ("stream", "batch"):
            # the zero-class setting the context measured and chose (s3dg_query_zero_tune)
            zc = lib.s3dg_zero_class(fn, fd)
            if zc:
                best, rg, pg, nt = ctypes.c_int(), ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
                call("s3dg_query_zero_tune", ctx._h, zc, ctypes.byref(best), ctypes.byref(rg), ctypes.byref(pg),
                     ctypes.byref(nt))
                roof["zero_tune"] = {"zero_class": zc, "setting": {1: "occupancy cap 29", 2: "store floor 100"}[zc],
                                     "chosen": "class setting" if best.value == 0 else "plain",
                                     "class_setting_GBps": round(rg.value, 1), "plain_GBps": round(pg.value, 1),
                                     "timed_launches": nt.value}
        if ceil:
            roof.update(ceil)
            roof["frac_of_store_only_best"] = round(achieved_gbs / ceil["store_only_best_GBps"], 4)
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
                       "dedup": d, "compress": list(cfg["compress"]) if isinstance(cfg["compress"], tuple)
                       else cfg["compress"],
                       "launches_per_step": len(launches), "parallelism": f"object-stream x{world}",
                       "stores": (args.store if args.store != "default"
                                  else {"keystream": "sc1", "dgen": "sc1", "dgen_stream": "sc1",
                                        "batch": "sc1 (tiled layouts), nt sc1 (dense layout)"}.get(
                                      kind, "sc1" if tiled else "nt sc1"))},
            "roofline": roof,
            "cpu_baseline": cpu,
            "d2h_inclusive": d2h,
            "verified_vs_oracle": verified,
            "ranks": rank_map,
        }
        if single_call:
            out["single_call"] = single_call
        print(json.dumps(out), flush=True)
    cp.close()
    return 0


def even_ring(n: int, cap_objs: int) -> int:
    """Objects per ring pass: the fewest passes the ring capacity allows, with
    the objects spread evenly over them, so every launch of a step writes the
    same bytes (100 000 objects as 10 x 10 000, not
    9 x 10 240 + 7 840)."""
    cap_objs = max(1, min(n, cap_objs))
    passes = -(-n // cap_objs)
    return -(-n // passes)


def launch_distribution(ms: list, nbytes: list, per_step: int = 1) -> dict:
    """Per-launch HIP-event times of the timed steps (the mean is
    what the line scores, and a bimodal run shows here): mean, p10/p50/p90,
    max, and per-launch rates (per byte, so launches of
    different sizes are not mixed) with the share of launches slower than the
    fast mode, i.e. a rate below p90(rate) / 1.06."""
    v = sorted(ms)
    if not v:
        return {}

    def pct(a, q):
        return round(a[min(len(a) - 1, int(q * len(a)))], 4)
    rates = sorted(b / (m * 1e6) for m, b in zip(ms, nbytes) if m > 0)
    fast = rates[min(len(rates) - 1, int(0.9 * len(rates)))] if rates else 0.0
    out = {"n": len(v), "launch_bytes": sorted(set(int(b) for b in nbytes)), "mean": round(sum(v) / len(v), 4),
           "p10": pct(v, 0.1), "p50": pct(v, 0.5), "p90": pct(v, 0.9), "max": round(v[-1], 4)}
    if rates:
        out.update({"GBps_min": round(rates[0], 1), "GBps_p10": round(pct(rates, 0.1), 1),
                    "GBps_p50": round(pct(rates, 0.5), 1), "GBps_p90": round(fast, 1),
                    "slow_share_rate_below_p90_over_1.06": round(sum(r < fast / 1.06 for r in rates) / len(rates), 4)})
        # where the slow launches sit: their indices in the timed sequence
        # (launch k is step k // per_step, position k % per_step)
        slow = [k for k, (m, b) in enumerate(zip(ms, nbytes)) if m > 0 and b / (m * 1e6) < fast / 1.06]
        out["slow_launch_indices"] = slow[:64]
        if per_step > 1:
            out["slow_by_position_in_step"] = [sum(1 for k in slow if k % per_step == q) for q in range(per_step)]
    return out


def host_buffer(n: int, kind: str, call):
    """(address, keepalive) of an n-byte host buffer, touched once (a reused
    Vec / bytearray: pageable; or pinned by the library)."""
    import numpy as np
    if kind == "pinned":
        p = ctypes.c_void_p()
        call("s3dg_host_alloc_pinned", n, ctypes.byref(p))
        ctypes.memset(p.value, 1, n)
        return p.value, p
    a = np.ones(n, np.uint8)
    if kind == "registered":   # a reused pageable buffer the caller page-locks (s3dg_host_register)
        call("s3dg_host_register", int(a.ctypes.data), n)
    return int(a.ctypes.data), a


def verify_host(hbufs, cfg, fn, fd, call, cp) -> bool:
    """The host path's seeded forms into the same buffer, byte for byte against
    the C oracle: fill_controlled_data_seeded (entropy 7, the slot context's
    default base block) or generate_data (DG1, seed 7)."""
    import numpy as np
    from oracle import oracle_c as OC
    size = cfg["size"]
    b = hbufs[0][0]
    if cfg.get("chunk"):
        # thread 0's last fill_chunk holds the tail of its last object (seed SEED_BASE + calls - 1); and one
        # whole object re-made through the same chunk size, both vs the DG1 oracle
        chunk, calls = cfg["chunk"], cfg["n"]
        tail = size % chunk or min(chunk, size)
        got = np.ctypeslib.as_array((ctypes.c_uint8 * tail).from_address(b))
        exp = OC.dgen_fill(size, cfg["dedup"], fn, fd, SEED_BASE + calls - 1)
        ok = sha(got) == sha(exp[size - tail:])
        n1 = min(size, 64 * MiB)
        g = ctypes.c_void_p()
        call("s3dg_gen_create", n1, cfg["dedup"], cfg["compress"], 1, 7, ctypes.byref(g))
        out = np.empty(n1, np.uint8)
        w, pos = ctypes.c_uint64(), 0
        while pos < n1:
            call("s3dg_gen_fill_chunk", g, out.ctypes.data + pos, min(chunk, n1 - pos), ctypes.byref(w))
            pos += w.value
        call("s3dg_gen_destroy", g)
        ok &= sha(out) == sha(OC.dgen_fill(n1, cfg["dedup"], fn, fd, 7))
        verified = bool(cp.max(0.0 if ok else 1.0) == 0.0)
        if not verified:
            print("bench: VERIFICATION FAILED: fill_chunk output differs from the oracle", file=sys.stderr)
        return verified
    got = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(b))
    if cfg.get("threads", 1) == 1:
        call("s3dlio_fill_controlled_data_seeded", b, size, cfg["dedup"], cfg["compress"], 7, None)
        exp = OC.fill_controlled(size, cfg["dedup"], fn, fd, 7, OC.base_block(BASE_SEED))
    else:
        call("s3dg_generate_data", b, size, cfg["dedup"], cfg["compress"], 1, 7)
        exp = OC.dgen_fill(size, cfg["dedup"], fn, fd, 7)
    ok = sha(got) == sha(exp)
    verified = bool(cp.max(0.0 if ok else 1.0) == 0.0)
    if not verified:
        print("bench: VERIFICATION FAILED: host-buffer output differs from the oracle", file=sys.stderr)
    return verified


def verify(torch, ring, samples, cfg, fn, fd, rank, cp) -> bool:
    """The first, the last and 16 random samples of the step's last writes,
    byte for byte against the C oracle."""
    import random
    from oracle import oracle_c as OC
    base = OC.base_block(BASE_SEED)
    rnd = random.Random(1234 + rank)
    idx = sorted({0, len(samples) - 1} | set(rnd.sample(range(len(samples)), min(16, len(samples)))))
    ok = True
    for i in idx:
        off, what = samples[i]
        if what[0] == "chunk":                  # 2 MiB keystream chunk
            got = ring[off:off + 2 * MiB].cpu().numpy()
            ok &= sha(got) == sha(OC.xoshiro_chunks(2 * MiB, 2 * MiB, what[1]))
        elif what[0] == "obj":
            _, j, size = what
            got = ring[off:off + size].cpu().numpy()
            exp = OC.fill_controlled(size, cfg["dedup"], fn, fd, object_entropy_py(SEED_BASE, j), base)
            ok &= sha(got) == sha(exp)
        elif what[0] == "single":
            got = ring[:what[1]].cpu().numpy()
            ok &= sha(got) == sha(OC.fill_controlled(what[1], cfg["dedup"], fn, fd, 7, base))
        else:                                   # DG1: block 0 of the object (1 MiB)
            got = ring[off:off + MiB].cpu().numpy()
            exp = OC.dgen_fill(MiB, cfg["dedup"], fn, fd, object_entropy_py(SEED_BASE, what[1]))
            ok &= sha(got) == sha(exp)
    verified = bool(cp.max(0.0 if ok else 1.0) == 0.0)
    if not verified:
        print("bench: VERIFICATION FAILED: sampled objects differ from the oracle", file=sys.stderr)
    return verified


def ceilings(torch, ctx, ring, stream, args, store) -> dict:
    """Store-only references on the same buffer (<= 16 GiB).  The ceiling the
    fill is judged against is its own launch with the PRNG chain and the
    window patches compiled out (s3dg_write_ceiling_fill: same records, grid,
    LDS image, barrier, stores and trailing loads); the other shapes are kept
    for comparison (pure store kernels overdrive the L2's
    write path and run slower than the fill)."""
    ceil_bytes = min(int(ring.numel()), 16 * GiB) // (8 * MiB) * (8 * MiB)
    if ceil_bytes == 0:
        return {}

    def rate(fn):
        fn(ring, ceil_bytes, stream=stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(3):
            fn(ring, ceil_bytes, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        return 3 * ceil_bytes / (e0.elapsed_time(e1) * 1e-3) / 1e9
    ctx.set_waves_per_block(args.waves_per_block or 0)
    occ = -1 if args.occupancy is None else args.occupancy
    ctx.set_occupancy(occ, occ)
    ctx.set_store_policy(store, store)
    # the ablated fill at several store pacings (wave-0 delay where the fill
    # plans); the best is the ceiling
    paced = {pace: round(rate(lambda b, n, stream, pace=pace: ctx.write_ceiling_fill(b, n, pace=pace, stream=stream)), 1)
             for pace in (0, 2, 4, 8, 16)}
    best_pace = max(paced, key=paced.get)
    fill_ceiling = paced[best_pace]
    shapes = {f"ablated_fill_pace{p_}": v for p_, v in paced.items()}
    names = {-1: "default", 0: "plain", 1: "nt", 2: "sc1", 3: "ntsc1"}
    shapes[f"tiled_1w_{ctx.query_occupancy(batch=True)}perCU_{names[store]}"] = round(
        rate(ctx.write_ceiling_tiled), 1)
    for waves, occ_, sp in [(4, 4, 2), (2, 4, 2), (4, 0, 0)]:
        ctx.set_waves_per_block(waves)
        ctx.set_occupancy(occ_, occ_)
        ctx.set_store_policy(sp, sp)
        shapes[f"{waves}w_{ctx.query_occupancy()}perCU_{names[sp]}"] = round(rate(ctx.write_ceiling), 1)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]

    def memset_d32(buf, nbytes, stream):
        assert hip.hipMemsetD32Async(buf.data_ptr(), 0x5A5A5A5A, nbytes // 4, int(stream.cuda_stream)) == 0
    shapes["hipMemsetD32Async"] = round(rate(memset_d32), 1)
    # not a ceiling: the fill runs above every store-only shape
    return {"store_only_best_GBps": fill_ceiling,
            "store_only_best_kind": f"k_fill_batch with the PRNG chain and window patches compiled out "
                                    f"(s3dg_write_ceiling_fill), 8 MiB objects, best pacing {best_pace}; "
                                    f"a reference shape, not a bound: the fill writes faster (DESIGN.md §5.1.1)",
            "store_only_shapes_GBps": shapes}


def traffic_from_profiles(config: int, launch_bytes: int):
    """HBM bytes per launch from the committed PMC passes (profiles/traffic.json),
    only when they were taken on this config, this launch size and this
    library source (source_digest)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(p) as f:
            t = json.load(f).get(str(config))
        if (t and t.get("algorithmic_bytes_per_launch") == launch_bytes
                and t.get("source_digest") == source_digest()):
            return t.get("traffic_bytes_per_launch")
    except Exception:
        pass
    return None


def pcie_link(torch, dev: int):
    """The GPU function's PCIe link and its upstream port's, as sysfs reports
    them ("32.0 GT/s PCIe x16"), or None where unreadable."""
    try:
        pr = torch.cuda.get_device_properties(dev)
        bdf = "%04x:%02x:%02x.0" % (getattr(pr, "pci_domain_id", 0), pr.pci_bus_id, pr.pci_device_id)
        p = os.path.realpath(f"/sys/bus/pci/devices/{bdf}")
        out = []
        for d in (p, os.path.dirname(p)):
            with open(d + "/current_link_speed") as f, open(d + "/current_link_width") as g:
                out.append(f"{f.read().strip()} x{g.read().strip()}")
        return out
    except Exception:
        return None


def numa_of(ptr: int) -> dict:
    """NUMA placement of the mapping holding `ptr` (/proc/self/numa_maps:
    pages per node of the mapping that starts at or below ptr)."""
    best, line = -1, ""
    try:
        for l in open("/proc/self/numa_maps"):
            a = int(l.split()[0], 16)
            if best < a <= ptr:
                best, line = a, l
    except Exception:
        return {}
    return {k: int(v) for k, v in (f.split("=") for f in line.split() if f[:1] == "N" and "=" in f)}


def d2h_inclusive(torch, ctx, call, dev, cfg, fn, fd, lo, total=8 * GiB, chunk=256 * MiB, n_objs=None):
    """Generate the config's objects through two device chunk buffers and
    copy each chunk to a pinned host ring on the GPU's NUMA node, on a second
    stream (the PUT path's input).  Default: an 8 GiB sample.  n_objs (the
    --d2h-full mode): all of the rank's objects [lo, lo + n_objs),
    timed from the first launch to the last D2H completion, the last host
    chunk checked against the oracle.  Logs where the ring's pages are, the
    CPUs the process runs on and the per-copy rates (HIP events on the copy
    stream), so run-to-run spread can be attributed."""
    kind = cfg["kind"]
    size = cfg["size"]
    dg = kind in ("dgen", "dgen_stream")
    per_chunk = max(1, chunk // size) if not dg else 1
    cb = per_chunk * size if not dg else chunk
    if n_objs is None:
        nchunks = total // cb
        chunk_objs = [per_chunk] * nchunks
    elif dg:             # DG1: the objects' 1 MiB blocks, chunk by chunk
        tot = n_objs * size
        nchunks = (tot + cb - 1) // cb
        chunk_objs = [1] * nchunks
    else:
        nchunks = (n_objs + per_chunk - 1) // per_chunk
        chunk_objs = [min(per_chunk, n_objs - k * per_chunk) for k in range(nchunks)]
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
    cev = []
    blocks_per_obj = (size + MiB - 1) // MiB if dg else 0

    def chunk_bytes(k):
        if dg:
            if n_objs is None:
                return cb
            return min(cb, n_objs * size - k * cb)
        return chunk_objs[k] * size

    def run(n, timed):
        for k in range(n):
            s = k & 1
            nb = chunk_bytes(k)
            gen.wait_event(cpy_done[s])
            if kind == "keystream":
                call("s3dg_xoshiro_fill", ctx._h, int(devbuf[s].data_ptr()), nb, 2 * MiB,
                     (lo * size + k * cb) // (2 * MiB), int(gen.cuda_stream))
            elif dg:
                # chunk k = MiB blocks [k*cb, k*cb + nb) of the objects laid end to end
                b0 = k * (cb >> 20)
                j, blk = divmod(b0, blocks_per_obj)
                call("s3dg_dgen_fill", ctx._h, int(devbuf[s].data_ptr()), size, blk, blk + (nb >> 20),
                     cfg["dedup"], fn, fd, object_entropy_py(SEED_BASE, lo + j) if n_objs is not None else SEED_BASE,
                     int(gen.cuda_stream))
            else:
                call("s3dg_fill_controlled_stream", ctx._h, int(devbuf[s].data_ptr()), size, size,
                     chunk_objs[k], cfg["dedup"], fn, fd, SEED_BASE, lo + k * per_chunk, int(gen.cuda_stream))
            gen_done[s].record(gen)
            cpy.wait_event(gen_done[s])
            if timed:
                cev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                cev[-1][0].record(cpy)
            call("s3dg_d2h_async", ctx._h, host[s], int(devbuf[s].data_ptr()), nb, int(cpy.cuda_stream))
            if timed:
                cev[-1][1].record(cpy)
            cpy_done[s].record(cpy)
    verified = None
    try:
        for s in range(2):
            cpy_done[s].record(cpy)
        # the first GiBs into fresh pinned pages copy slower
        run(max(2, nchunks // 4) if n_objs is None else min(4, nchunks), False)
        torch.cuda.synchronize()
        link_before = pcie_link(torch, dev)
        t0 = time.perf_counter()
        run(nchunks, True)
        link_during = pcie_link(torch, dev)   # read while the last copies run
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        pages = [numa_of(p) for p in host]
        if n_objs is not None and kind == "stream":
            # the last chunk's first object, from pinned host memory, vs the oracle
            import numpy as np
            from oracle import oracle_c as OC
            k = nchunks - 1
            got = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(host[k & 1]))
            exp = OC.fill_controlled(size, cfg["dedup"], fn, fd, object_entropy_py(SEED_BASE, lo + k * per_chunk),
                                     OC.base_block(BASE_SEED))
            verified = bool(np.array_equal(got, exp))
    finally:
        torch.cuda.synchronize()
        for p in host:
            call("s3dg_host_free_pinned", p)
    done_bytes = sum(chunk_bytes(k) for k in range(nchunks))
    seq = [chunk_bytes(k) / (a.elapsed_time(b) * 1e-3) / GiB for k, (a, b) in enumerate(cev)]
    rates = sorted(seq)
    cpus = sorted(os.sched_getaffinity(0))
    cpu_nodes = set()
    for nd in os.listdir("/sys/devices/system/node") if os.path.isdir("/sys/devices/system/node") else []:
        if nd.startswith("node"):
            try:
                from_list = open(f"/sys/devices/system/node/{nd}/cpulist").read().strip()
                ids = set()
                for part in from_list.split(","):
                    a, _, b = part.partition("-")
                    ids.update(range(int(a), int(b or a) + 1))
                if ids & set(cpus):
                    cpu_nodes.add(int(nd[4:]))
            except Exception:
                pass
    what = (f"the rank's whole object range ({n_objs} objects, {done_bytes / 1e9:.1f} GB), first launch to last "
            f"D2H completion" if n_objs is not None else f"{nchunks} x {cb // MiB} MiB device chunks "
            f"({done_bytes // GiB} GiB) of the config's objects")
    out = {"value": round(done_bytes / dt / GiB, 2), "unit": "GiB/s",
           "mode": "full" if n_objs is not None else "sample",
           "bytes": done_bytes, "seconds": round(dt, 4),
           "sample": f"{what}, 2 device chunks of {cb // MiB} MiB, pinned host ring (hipHostMalloc default flags, "
                     f"allocated from a thread bound to the GPU's local CPUs), generate || D2H on two streams",
           "gpu_numa_node": node.value, "ring_pages_per_node": pages,
           "pcie_link_gpu_upstream": {"before": link_before, "end": link_during},
           "process_cpu_nodes": sorted(cpu_nodes),
           "copy_GiBps_min_med_max": [round(rates[0], 1), round(rates[len(rates) // 2], 1), round(rates[-1], 1)],
           # per host slot (copy k lands in slot k % 2), and the timed copies
           # below 3/4 of the best slot's median, by position (0 = first timed copy)
           "copy_GiBps_med_by_slot": [round(statistics.median(seq[s::2]), 1) for s in range(2) if seq[s::2]],
           "slow_copies": [[k, round(r, 1)] for k, r in enumerate(seq)
                           if r < 0.75 * max(statistics.median(seq[s::2]) for s in range(2) if seq[s::2])][:16]}
    if n_objs is not None:
        out["verified_vs_oracle"] = verified
    return out


def object_entropy_py(seed_base: int, j: int) -> int:
    return (seed_base + (j << 32)) & (2**64 - 1)


def cpu_idle_fractions(window: float = 0.25) -> dict:
    """Per-CPU idle share over `window` seconds (/proc/stat idle + iowait)."""
    def snap():
        out = {}
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3].isdigit():
                f = line.split()
                v = [int(x) for x in f[1:]]
                out[int(f[0][3:])] = (v[3] + v[4], sum(v))
        return out
    try:
        a = snap()
        time.sleep(window)
        b = snap()
    except Exception:
        return {}
    return {c: (b[c][0] - a[c][0]) / max(1, b[c][1] - a[c][1]) for c in a if c in b}


def pin_cpus(dev: int, n: int, policy: str = "local") -> list[int]:
    """n CPUs of this process's affinity: those on the GPU's NUMA node first,
    one per physical core, up to S3DG_CPU_PER_CCD (4) from each L3 domain
    (CCD), the idlest CCDs and cores first (/proc/stat over 0.25 s, a core as
    idle as its busiest hardware thread), so a baseline pinned on a shared
    host neither lands on cores other jobs are busy on nor packs its threads
    onto one or two CCDs' memory links."""
    aff = sorted(os.sched_getaffinity(0))
    local = []
    try:
        if policy != "local":
            raise LookupError("no node preference")
        from s3dlio_amd._lib import lib
        node = ctypes.c_int(-1)
        lib.s3dg_device_numa_node(dev, ctypes.byref(node))
        if node.value >= 0:
            ids = set()
            for part in open(f"/sys/devices/system/node/node{node.value}/cpulist").read().strip().split(","):
                a, _, b = part.partition("-")
                ids.update(range(int(a), int(b or a) + 1))
            local = [c for c in aff if c in ids]
    except Exception:
        local = []
    idle = cpu_idle_fractions()

    def siblings(c):
        try:
            out = set()
            for part in open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip().split(","):
                a, _, b = part.partition("-")
                out.update(range(int(a), int(b or a) + 1))
            return out
        except Exception:
            return {c}
    # one logical CPU per physical core, the cores whose every hardware thread
    # is idle first: an "idle" CPU whose SMT sibling runs another job's thread
    # gives a baseline thread half a core (round 6's first pinned lines ran
    # 30-50 % below the unpinned samples beside them)
    def core_score(c):
        return min(idle.get(x, 0.0) for x in siblings(c))
    # ... by L3 domain (CCD): a CCD's link to memory carries ~60 GB/s, so 16
    # threads packed on two CCDs wrote 85 GiB/s where the same count spread by
    # the scheduler wrote 150 (round 6, profiles/r06/cpu/)
    def l3(c):
        try:
            return open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list").read().strip()
        except Exception:
            return "?"
    # whole CCDs when they are idle: the idlest L3 domains first, up to
    # per_dom cores from each (one CCD link ~60 GB/s: four CCDs carry the
    # port's ~150 GiB/s, and a CCD no other job runs on keeps the samples
    # tight; spreading one core over every CCD shared each with other jobs)
    per_dom = int(os.environ.get("S3DG_CPU_PER_CCD", "4"))
    picked, used = [], set()
    for group in (local, [c for c in aff if c not in local]):
        doms = {}
        for c in sorted(group, key=lambda c: (-core_score(c), c)):
            doms.setdefault(l3(c), []).append(c)
        order = sorted(doms.values(), key=lambda q: -sum(core_score(c) for c in q) / max(1, len(q)))
        for q in order:
            took = 0
            for c in q:
                if took >= per_dom or len(picked) >= n:
                    break
                if c in used:
                    continue
                picked.append(c)
                used |= siblings(c)
                took += 1
    if len(picked) < n:   # fewer cores than threads: add second hardware threads
        picked += [c for c in sorted(aff, key=lambda c: -idle.get(c, 0.0)) if c not in picked]
    return picked[:n]


def cpu_baseline(cfg, fn, fd, seconds, sizes, dev=0, reps=7, pin=True):
    """The C restatement of the same generator (oracle, kind 'port') on this
    host's cores, parallel like the reference's Rayon loops: a warm-up sample,
    then `reps` samples of seconds/reps each, the median reported with min and
    max.  pin (default since round 6, VERDICT r05 next
    #6): threads bound to the cgroup's share of CPUs, those on the GPU's NUMA
    node first and the idlest ones at the time (threads inherit the calling
    thread's affinity; the sample's buffers are first touched by the pinned
    thread, so they sit on that node).  Round 4 pinned to the first CPUs of
    the affinity list and its samples spread 10-400 % on the shared 256-CPU
    host (profiles/r04/bench/d_*), where others' jobs ran on them."""
    share = cpu_share()
    cpus = pin_cpus(dev, share["threads"], os.environ.get("S3DG_CPU_PIN_POLICY", "local")) if pin else None
    saved = os.sched_getaffinity(0)
    runs = []
    try:
        if cpus:
            os.sched_setaffinity(0, cpus)
        _cpu_sample(cfg, fn, fd, min(1.0, seconds / reps), sizes, share)   # warm-up: pools, rings, pages
        for _ in range(reps):
            runs.append(_cpu_sample(cfg, fn, fd, seconds / reps, sizes, share))
    finally:
        if cpus:
            os.sched_setaffinity(0, saved)
    vals = sorted(r["value"] for r in runs)
    med = vals[len(vals) // 2]
    q1, q3 = vals[len(vals) // 4], vals[(3 * len(vals)) // 4]
    out = dict(next(r for r in runs if r["value"] == med))
    # spread: (max - min) / median; iqr_spread: (q3 - q1) / median, which a
    # single sample disturbed by another job on the shared host does not move
    out.update(value=med, samples_GiBps=[r["value"] for r in runs],
               min_med_max_GiBps=[vals[0], med, vals[-1]], q1_q3_GiBps=[q1, q3],
               spread=round((vals[-1] - vals[0]) / med, 4) if med else None,
               iqr_spread=round((q3 - q1) / med, 4) if med else None,
               pinned_cpus=(f"{len(cpus)} CPUs: " + ",".join(str(c) for c in sorted(cpus))) if cpus
               else "no (scheduler's choice)",
               sample=f"median of {reps} samples; one sample: " + out["sample"])
    if cpus:
        # beside it, five samples left to the scheduler (the reference's Rayon
        # pool is not pinned): the pinned median is the reported value (tight,
        # VERDICT r05 next #6), this shows what pinning costs on the shared
        # host (up to 30 % in round 6's lines)
        _cpu_sample(cfg, fn, fd, min(1.0, seconds / reps), sizes, share)
        un = sorted(_cpu_sample(cfg, fn, fd, seconds / reps, sizes, share)["value"] for _ in range(5))
        out["unpinned_min_med_max_GiBps"] = [un[0], un[2], un[-1]]
    return out


def _cpu_sample(cfg, fn, fd, seconds, sizes, share):
    """One bounded sample (~`seconds`) of the port into reused host memory."""
    import threading
    import numpy as np
    from oracle import oracle_c as OC
    threads = share["threads"]
    base = OC.base_block(BASE_SEED)
    kind = cfg["kind"]
    meta = {"cores": threads, "kind": "port", "affinity_cpus": share["affinity_cpus"],
            "cgroup_quota_cpus": share["cgroup_quota_cpus"]}
    if kind == "host" and cfg.get("threads", 1) == 1:
        # the criterion loop: one reused buffer, one call at a time, over a
        # persistent pool (Rayon's global pool) of the host's share of CPUs
        size = cfg["size"]
        buf = np.ones(size, np.uint8)
        OC.pool_fill_controlled(buf, cfg["dedup"], fn, fd, 0, base, threads)
        done, t0 = 0, time.perf_counter()
        while True:
            used = OC.pool_fill_controlled(buf, cfg["dedup"], fn, fd, done + 1, base, threads)
            done += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                break
        meta["cores"] = used
        return dict(meta, value=round(done * size / dt / GiB, 2), unit="GiB/s",
                    sample=f"{done} fill_controlled_data calls on one reused {size // MiB} MiB host buffer over "
                           f"{dt:.1f} s, persistent pool of {used} threads over 4 KiB blocks; {cpu_model()}")
    if kind in ("stream", "single") or (kind == "batch" and cfg.get("uniform")):
        # fill_controlled_data's par_chunks_mut(4096) over a reused 1 GiB ring
        # (uniform batches: the same objects, laid out back to back)
        size = cfg["size"] or cfg["uniform"]
        per = max(1, GiB // size)
        buf = np.ones(per * size, np.uint8)                        # fault the pages in before timing
        OC.fill_stream(size, per, cfg["dedup"], fn, fd, SEED_BASE, 0, base, threads=threads, out=buf)
        done, t0, k = 0, time.perf_counter(), 0
        while True:
            OC.fill_stream(size, per, cfg["dedup"], fn, fd, SEED_BASE, k * per, base, threads=threads, out=buf)
            done += per
            k += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                break
        t1s = time.perf_counter()
        OC.fill_stream(size, per, cfg["dedup"], fn, fd, SEED_BASE, 0, base, threads=1, out=buf)
        one = per * size / (time.perf_counter() - t1s) / GiB
        return dict(meta, value=round(done * size / dt / GiB, 2), unit="GiB/s", single_thread_GiBps=round(one, 2),
                    sample=f"{done} x {size / KiB:g} KiB objects ({done * size / GiB:.0f} GiB) over {dt:.1f} s into "
                           f"a reused 1 GiB host ring, {threads} threads over 4 KiB blocks; {cpu_model()}")
    # per-object (or per-chunk) tasks from a pool of host threads, each thread
    # writing its own reused host ring
    L = OC.lib()
    if kind == "batch":
        ring = max(256 * MiB, max(sizes))
        items = sizes

        def work(buf, pos, j):
            sz = items[j % len(items)]
            if pos + sz > ring:
                pos = 0
            L.s3dgo_fill_controlled(ctypes.cast(buf.ctypes.data + pos, ctypes.POINTER(ctypes.c_uint8)), sz,
                                    cfg["dedup"], fn, fd, object_entropy_py(SEED_BASE, j),
                                    base.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
            return pos + (sz + 4095) // 4096 * 4096, sz
        what = "objects of the config's sizes, one object per task"
    elif kind == "host" and cfg.get("chunk"):
        # the same loop on the CPU: 8 threads streaming DG1 objects chunk by chunk (PRNG state carried across
        # chunks, s3dgo_dgen_stream_fill) into a reused chunk buffer each
        nthr = cfg["threads"]
        chunk = min(cfg["chunk"], cfg["size"])
        b, dt = OC.dgen_chunk_bench(nthr, cfg["size"], chunk, cfg["dedup"], fn, fd, SEED_BASE, seconds)
        meta["cores"] = nthr
        return dict(meta, value=round(b / dt / GiB, 2), unit="GiB/s",
                    sample=f"{b / GiB:.1f} GiB of {cfg['size'] // MiB} MiB DG1 objects as {chunk // KiB} KiB "
                           f"fill_chunk calls over {dt:.1f} s on {nthr} threads (streaming port, one object "
                           f"at a time per thread); {cpu_model()}")
    elif kind == "host":     # generate_into_buffer from several threads: DG1 objects, one per call
        ring, nthr = cfg["size"], cfg["threads"]
        threads = nthr
        meta["cores"] = nthr

        def work(buf, pos, j):
            OC.dgen_fill(ring, cfg["dedup"], fn, fd, object_entropy_py(SEED_BASE, j), out=buf)
            return 0, ring
        what = f"{ring // MiB} MiB DG1 objects, one generate_into_buffer-shaped call per task"
    elif kind == "keystream":
        ring = 256 * MiB

        def work(buf, pos, j):
            if pos + 2 * MiB > ring:
                pos = 0
            OC.xoshiro_chunks(2 * MiB, 2 * MiB, j, out=buf[pos:pos + 2 * MiB])
            return pos + 2 * MiB, 2 * MiB
        what = "2 MiB keystream chunks (npz.rs:376-383), one chunk per task"
    else:   # dgen: 8 MiB pieces of DG1 objects
        ring = 256 * MiB

        def work(buf, pos, j):
            if pos + 8 * MiB > ring:
                pos = 0
            OC.dgen_fill(8 * MiB, cfg["dedup"], fn, fd, object_entropy_py(SEED_BASE, j), out=buf[pos:pos + 8 * MiB])
            return pos + 8 * MiB, 8 * MiB
        what = "8 MiB DG1 objects, one object per task"
    lock = threading.Lock()
    state = {"next": 0, "bytes": 0, "tasks": 0, "stop": False}
    start = threading.Event()

    def worker():
        buf = np.ones(ring, np.uint8)
        done = ntask = pos = 0
        start.wait()
        while not state["stop"]:
            with lock:
                j = state["next"]
                state["next"] += 1
            pos, b = work(buf, pos, j)
            done += b
            ntask += 1
        with lock:
            state["bytes"] += done
            state["tasks"] += ntask
    ts = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ts:
        t.start()
    time.sleep(0.3)                                       # rings allocated and touched
    t0 = time.perf_counter()
    start.set()
    time.sleep(seconds)
    state["stop"] = True
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    return dict(meta, value=round(state["bytes"] / dt / GiB, 2), unit="GiB/s",
                sample=f"{state['tasks']} {what} ({state['bytes'] / GiB:.0f} GiB) over {dt:.1f} s on {threads} "
                       f"threads, each writing a {ring // MiB} MiB host ring; {cpu_model()}")


if __name__ == "__main__":
    sys.exit(main())

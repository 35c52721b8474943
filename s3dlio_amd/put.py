"""PUT of synthetic objects to file:// targets, one payload per object.

Mirrors the reference's put surface:
    put(prefix, num, template=None, max_in_flight=64, size=None, ...)
                                    src/python_api/python_core_api.rs:777-818
    build_uri_list(prefix, template, num)          python_core_api.rs:657-691
    put_objects_with_random_data_and_type(uris, size, max_in_flight, config)
                                    src/s3_utils.rs:1717-1750
The work runs in the native pipeline s3dg_put_objects (s3dg_put.cpp): GPU
generation + GPU CRC-32 -> pinned host ring -> writer threads.

Deliberate differences from the reference:
  * object j gets its own payload (entropy object_entropy(seed_base, j));
    the reference PUTs one generated buffer to every URI (s3_utils.rs:1741);
  * only file:// targets: the S3 / Azure / GCS back ends are out of scope;
  * the call returns per-object CRC-32s (crc32fast of each file's bytes, the
    StreamingDataWriter checksum, src/streaming_writer.rs:183-186) and stats.
Payload kinds follow generate_object's dispatch (data_gen.rs:29-94):
use_controlled (dedup != 1 or compress != 1) -> the DG1 stream, otherwise the
generate_random_data layout; payload="controlled" selects the
fill_controlled_data layout instead (the benchmark kernel).
"""
from __future__ import annotations

import ctypes
import threading
import os
import time
from dataclasses import dataclass, field

from ._lib import PutStats, call
from .device import compress_ratio
from .objects import Config, DataGenMode, ObjectType

DEFAULT_OBJECT_SIZE = 20 * 1024 * 1024          # src/s3_utils.rs:217
_PAYLOADS = {"controlled": 0, "random": 1, "dgen": 2}


def build_uri_list(prefix: str, template: str, num: int) -> tuple[str, list[str]]:
    """python_core_api.rs:657-691: scheme://bucket/key_prefix/ + template with
    the first "{}" -> index and the second "{}" -> num."""
    k = prefix.find("://")
    if k < 0:
        raise ValueError("URI must contain scheme (e.g., s3://, az://, file://)")
    scheme, rest = prefix[:k + 3], prefix[k + 3:]
    bucket, _, key_prefix = rest.partition("/")
    if key_prefix and not key_prefix.endswith("/"):
        key_prefix += "/"
    uris = []
    for i in range(num):
        name = template.replace("{}", str(i), 1).replace("{}", str(num), 1)
        uris.append(f"{scheme}{bucket}/{key_prefix}{name}")
    return bucket, uris


def _uri_to_path(uri: str) -> str:
    """FileSystemObjectStore::uri_to_path (src/file_store.rs:287-295)."""
    if not uri.startswith("file://"):
        raise ValueError(f"only file:// targets are built in this drop-in (got {uri!r}); "
                         "object-store back ends are out of scope")
    return uri[7:]


@dataclass
class PutResult:
    checksums: list[int] = field(default_factory=list)   # CRC-32 of each file as written
    objects: int = 0
    bytes: int = 0
    seconds: float = 0.0
    gpu_seconds: float = 0.0
    seed_base: int = 0

    def checksum_str(self, j: int) -> str:
        """StreamingDataWriter::checksum format (streaming_writer.rs:183-186)."""
        return f"crc32c:{self.checksums[j]:08x}"


def _contexts(devices):
    """Contexts for `devices`: None / "all" = every visible GPU, else a list of
    device indices (repeats give several lanes on one GPU)."""
    from .device import Context
    if devices is None or devices == "all":
        n = ctypes.c_int()
        call("s3dg_device_count", ctypes.byref(n))
        devices = list(range(max(1, n.value)))
    ctxs = []
    for d in devices:
        key = (int(d), sum(1 for c in ctxs if c.device == int(d)))
        with _LANE_LOCK:
            if key not in _LANE_CTX:
                _LANE_CTX[key] = Context(int(d))
            ctxs.append(_LANE_CTX[key])
    return ctxs


_LANE_CTX: dict = {}      # (device, lane) -> Context, kept for the process
_LANE_LOCK = threading.Lock()


def put_objects(uris, size: int, max_in_flight: int = 64, config: Config | None = None,
                seed: int | None = None, payload: str | None = None, context=None,
                devices=None) -> PutResult:
    """Generate one payload per URI on the GPU(s) and write the files.
    `context` pins the call to one GPU; otherwise `devices` (default: every
    visible GPU) each take a contiguous range of the objects.  Output files
    and checksums do not depend on the GPU count."""
    import numpy as np
    cfg = config or Config.new_with_defaults(ObjectType.RAW, 1, size, 1, 1)
    if cfg.object_type == ObjectType.HDF5:
        raise ValueError("HDF5 format is not available in this build")
    paths = [_uri_to_path(u) for u in uris]
    if payload is None:
        payload = "dgen" if cfg.use_controlled else "random"
    kind = _PAYLOADS[payload]
    dedup = max(1, int(cfg.dedup_factor))
    fn, fd = compress_ratio(max(1, int(cfg.compress_factor)))
    if seed is None:   # the reference's time entropy
        seed = (time.time_ns() ^ (os.getpid() << 32)) & (2**64 - 1)
    n = len(paths)
    arr = (ctypes.c_char_p * max(1, n))(*[p.encode() for p in paths])
    crcs = np.zeros(max(1, n), np.uint32)
    st = PutStats()
    ctxs = [context] if context is not None else _contexts(devices)
    harr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    call("s3dg_put_objects_multi", harr, len(ctxs), arr, n, int(size), int(cfg.object_type), kind, dedup,
         fn, fd, int(seed) & (2**64 - 1), int(max_in_flight), int(crcs.ctypes.data), ctypes.byref(st))
    return PutResult([int(c) for c in crcs[:n]], st.objects, st.bytes, st.seconds, st.gpu_seconds,
                     int(seed) & (2**64 - 1))


def put_objects_with_random_data_and_type(uris, size: int, max_in_flight: int, config: Config,
                                          seed: int | None = None) -> PutResult:
    """src/s3_utils.rs:1717-1724 (per-object payloads; see module docstring)."""
    return put_objects(uris, size, max_in_flight, config, seed)


def put(prefix: str, num: int, template: str | None = None, max_in_flight: int = 64,
        size: int | None = None, should_create_bucket: bool = False, object_type: str = "zeros",
        dedup_factor: int = 1, compress_factor: int = 1, data_gen_algorithm: str = "random",
        data_gen_mode: str = "streaming", chunk_size: int = 262144, seed: int | None = None,
        devices=None) -> None:
    """python_core_api.rs:777-818.  should_create_bucket: parents are always
    created for file:// (file_store.rs:562-564); data_gen_algorithm: only
    "random" exists (prand deprecated, :696-701)."""
    sz = DEFAULT_OBJECT_SIZE if size is None else int(size)
    _, uris = build_uri_list(prefix, template or "object-{}", num)
    jobs = min(max_in_flight, num)
    mode = DataGenMode.SINGLE_PASS if data_gen_mode.lower() in (
        "single-pass", "single_pass", "singlepass") else DataGenMode.STREAMING
    cfg = (Config.new_with_defaults(ObjectType.from_str(object_type), 1, sz, dedup_factor,
                                    compress_factor)
           .with_data_gen_mode(mode).with_chunk_size(chunk_size))
    put_objects(uris, sz, jobs, cfg, seed, devices=devices)

"""Device-resident generation API over the C ABI (one Context per GPU).

This is the MI355X-native core the drop-in surfaces sit on:

    ctx = Context(device=0)                       # s3dg_ctx_create
    out = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    ctx.fill_stream(out, obj_size=size, n_objs=n, dedup=1, compress=1, seed_base=S)

Semantics per object are src/data_gen.rs:151-224 (fill_controlled_data) with
the entropy and base block made explicit.
"""
from __future__ import annotations

import ctypes
from fractions import Fraction

import numpy as np

from . import _lib
from ._lib import ObjDesc, c_u32, c_vp, call, lib

BLOCK_SIZE = 4096
DEFAULT_BASE_SEED = 0xBA5EB10C00000000


def compress_ratio(compress) -> tuple[int, int]:
    """(f_num, f_den) of the zero prefix per 4 KiB block.

    Integer c maps to (c-1, c) and c <= 1 to (0, 1), exactly as
    src/data_gen.rs:169-173.  A rational p/q (Fraction, (p, q) tuple or a
    float such as 1.5) maps to (p-q, p): the build-defined generalisation
    needed by BASELINE config 4 (compress=1.5 -> (1, 3)); no reference API
    accepts it, so parity is defined for integer c only.
    """
    if isinstance(compress, (int, np.integer)) and not isinstance(compress, bool):
        fn, fd = c_u32(), c_u32()
        call("s3dg_compress_ratio", int(compress), ctypes.byref(fn), ctypes.byref(fd))
        return fn.value, fd.value
    if isinstance(compress, tuple):
        fr = Fraction(int(compress[0]), int(compress[1]))
    else:
        fr = Fraction(compress).limit_denominator(1 << 16)
    if fr <= 1:
        return 0, 1
    p, q = fr.numerator, fr.denominator
    return p - q, p


def unique_blocks(nblocks: int, dedup: int) -> int:
    return int(lib.s3dg_unique_blocks(nblocks, dedup))


def object_entropy(seed_base: int, j: int) -> int:
    return int(lib.s3dg_object_entropy(seed_base & (2**64 - 1), j))


def _ptr(x) -> int:
    """Device pointer of a torch CUDA tensor (contiguous) or a raw int."""
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        if not x.is_cuda:
            raise ValueError("device generation needs a GPU tensor (tensor.is_cuda)")
        if not x.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return int(x.data_ptr())
    raise TypeError(f"expected a torch CUDA tensor or an int device pointer, got {type(x)}")


def _nbytes(x) -> int | None:
    if hasattr(x, "numel") and hasattr(x, "element_size"):
        return int(x.numel() * x.element_size())
    return None


def _stream(stream, device: int | None = None) -> int:
    """hipStream_t handle: an int, a torch stream, or None = torch's current
    stream on `device` (the current device when None), so torch events time
    our launches."""
    if stream is None:
        t = _lib.torch
        if t is not None and t.cuda.is_available():
            cs = t.cuda.current_stream() if device is None else t.cuda.current_stream(device)
            return int(cs.cuda_stream)
        return 0
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


class Context:
    """One GPU's generator context (s3dg_ctx)."""

    @classmethod
    def _borrow(cls, handle: int, device: int) -> "Context":
        """A context owned elsewhere (the host slot pool): never destroyed here."""
        self = cls.__new__(cls)
        self._h = c_vp(handle)
        self.device = int(device)
        self._borrowed = True
        return self

    def __init__(self, device: int = 0, base_block=None, base_seed: int | None = None,
                 waves_per_block: int | None = None, nontemporal: bool = False):
        h = c_vp()
        call("s3dg_ctx_create", int(device), ctypes.byref(h))
        self._h = h
        self.device = int(device)
        if base_block is not None:
            self.set_base_block(base_block)
        elif base_seed is not None:
            call("s3dg_set_base_block_seed", self._h, int(base_seed))
        if waves_per_block is not None:
            call("s3dg_set_waves_per_block", self._h, int(waves_per_block))
        if nontemporal:
            call("s3dg_set_nontemporal", self._h, 1)

    # -- lifecycle -------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_borrowed", False):
            return
        if getattr(self, "_h", None):
            call("s3dg_ctx_destroy", self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- configuration -----------------------------------------------------------
    def set_base_block(self, base) -> None:
        b = np.ascontiguousarray(np.frombuffer(bytes(base), np.uint8))
        if b.size != BLOCK_SIZE:
            raise ValueError("base block must be exactly 4096 bytes")
        call("s3dg_set_base_block", self._h, b.ctypes.data_as(_lib.c_u8p))

    @property
    def base_block(self) -> bytes:
        out = np.empty(BLOCK_SIZE, np.uint8)
        call("s3dg_get_base_block", self._h, out.ctypes.data_as(_lib.c_u8p))
        return out.tobytes()

    def set_waves_per_block(self, waves: int) -> None:
        call("s3dg_set_waves_per_block", self._h, int(waves))

    def set_nontemporal(self, on: bool) -> None:
        call("s3dg_set_nontemporal", self._h, 1 if on else 0)

    def set_store_policy(self, stream_policy: int = -1, batch_policy: int = -1) -> None:
        """Fill-kernel store cache policy: 0 plain, 1 nt, 2 sc1, 3 nt sc1, -1 default;
        results are identical."""
        call("s3dg_set_store_policy", self._h, int(stream_policy), int(batch_policy))

    def set_occupancy(self, stream_wgs_per_cu: int = -1, batch_wgs_per_cu: int = -1) -> None:
        """Cap resident fill workgroups per CU (0 = hardware max, negative = library
        default); results are identical."""
        call("s3dg_set_occupancy", self._h, int(stream_wgs_per_cu), int(batch_wgs_per_cu))

    def set_batch_pace(self, ticks: int = -1) -> None:
        """Batch kernel: hold each block's stores until `ticks` wall-clock ticks
        (10 ns) after its workgroup started (0 = off, negative = per launch);
        results are identical."""
        call("s3dg_set_batch_pace", self._h, int(ticks))

    def set_batch_prefetch(self, tiles: int = -1) -> None:
        """Tile-record prefetch distance of batch launches in units of 64 blocks
        (0 = off, negative = library default); results are identical."""
        call("s3dg_set_batch_prefetch", self._h, 0xFFFFFFFF if int(tiles) < 0 else int(tiles))

    def set_stream_tiles(self, on: int = -1) -> None:
        """1: large uniform streams run through the tiled batch kernel; 0: the 2D
        stream kernel; negative: library default.  Results are identical."""
        call("s3dg_set_stream_tiles", self._h, int(on))

    def set_batch_tile(self, blocks: int = 0) -> None:
        """Blocks per batch tile record: 8, 16, 32, 64, or 0 = chosen per launch;
        results are identical."""
        call("s3dg_set_batch_tile", self._h, int(blocks))

    def set_batch_split(self, blocks: int = -1) -> None:
        """Objects of fewer than `blocks` blocks get a batch launch of their own
        (0 = one launch, negative = default); results are identical."""
        call("s3dg_set_batch_split", self._h, int(blocks))

    def set_keystream_shape(self, mode: int, draws: int = 0, waves: int = 0, wgs_per_cu: int = 0,
                            min_lane_draws: int = 0, store_policy: int = -1) -> None:
        """k_keystream launch shape for mode 0 (npz keystream) or 1 (DG1);
        0 (store: -1) = default for each; results are identical."""
        call("s3dg_set_keystream_shape", self._h, int(mode), int(draws), int(waves), int(wgs_per_cu),
             int(min_lane_draws), int(store_policy))

    def set_keystream_xcd_group(self, mode: int, waves: int = 0) -> None:
        """Keystream launches: each XCD writes runs of `waves` adjacent waves'
        lane regions (power of two; 0 = default 16); results are identical."""
        call("s3dg_set_keystream_xcd_group", self._h, int(mode), int(waves))

    def set_keystream_persist(self, rounds: int = -1) -> None:
        """Keystream launches of >= `rounds` rounds of resident waves run a
        persistent grid over per-XCD work queues (0 = never, negative = default:
        1-wave workgroups from 6 rounds).  Results are identical."""
        call("s3dg_set_keystream_persist", self._h, int(rounds))

    def set_keystream_tail(self, chunks: int = -1) -> None:
        """One-object DG1 launches on a persistent grid: the last `chunks`
        blocks in half-length lanes, handed out last (0 = off, negative =
        default).  Results are identical."""
        call("s3dg_set_keystream_tail", self._h, int(chunks))

    def set_dgen_zero_split(self, chunks: int = -1, waves: int = -1, occupancy: int = -1, store: int = -1,
                            overlap: int = -1) -> None:
        """DG1 launches with a zero prefix over >= `chunks` full 1 MiB blocks run
        as a zero-prefix launch in the fill's store shape plus a keystream
        launch over the tails (0 = never, negative = default 64); `waves`,
        `occupancy`, `store` and `overlap` (side stream) tune the zero launch.
        Results are identical."""
        call("s3dg_set_dgen_zero_split", self._h, int(chunks), int(waves), int(occupancy), int(store), int(overlap))

    def query_keystream_occupancy(self, mode: int = 0) -> int:
        out = ctypes.c_int()
        call("s3dg_query_keystream_occupancy", self._h, int(mode), ctypes.byref(out))
        return out.value

    def query_occupancy(self, batch: bool = False, zero_lines: bool = False) -> int:
        """Resident fill workgroups per CU under the current settings (batch
        launches: `zero_lines` = zero prefixes ending on a 64-B line)."""
        out = ctypes.c_int()
        call("s3dg_query_occupancy", self._h, (2 if zero_lines else 1) if batch else 0, ctypes.byref(out))
        return out.value

    # -- generation (asynchronous on `stream`) ----------------------------------
    # A torch tensor destination must live on this context's device and hold
    # every byte the call writes (ValueError otherwise: the C ABI only sees a
    # pointer and would write past the allocation).  A raw int pointer is the
    # caller's responsibility.
    def _dst(self, x, need: int) -> int:
        p = _ptr(x)
        if not isinstance(x, int):
            idx = x.device.index if x.device.index is not None else 0
            if idx != self.device:
                raise ValueError(f"tensor is on cuda:{idx}, this context is on cuda:{self.device}")
            have = _nbytes(x)
            if need > have:
                raise ValueError(f"the call writes {need} bytes, the tensor holds {have}")
        return p

    def _s(self, stream) -> int:
        return _stream(stream, self.device)

    def fill_controlled(self, dst, nbytes: int | None = None, dedup: int = 1, compress=1,
                        entropy: int = 0, stream=None) -> None:
        """One object (src/data_gen.rs:151) of `nbytes` at dst."""
        n = _nbytes(dst) if nbytes is None else int(nbytes)
        fn, fd = compress_ratio(compress)
        call("s3dg_fill_controlled", self._h, self._dst(dst, n), n, int(dedup), fn, fd,
             int(entropy) & (2**64 - 1), self._s(stream))

    def random_data(self, dst, nbytes: int | None = None, entropy: int = 0, stream=None) -> None:
        """generate_random_data's layout (src/data_gen.rs:102-132): no zero
        prefix, one window at 0 and one at L-32 (L > 2048), seeded by `entropy`."""
        n = _nbytes(dst) if nbytes is None else int(nbytes)
        call("s3dg_random_data", self._h, self._dst(dst, n), n, int(entropy) & (2**64 - 1),
             self._s(stream))

    def fill_range(self, dst, length: int, blk_lo: int, blk_hi: int, dedup: int = 1,
                   compress=1, entropy: int = 0, stream=None) -> None:
        """Blocks [blk_lo, blk_hi) of a `length`-byte object, block blk_lo at dst."""
        fn, fd = compress_ratio(compress)
        hi = min(int(blk_hi) * BLOCK_SIZE, int(length))
        need = max(0, hi - int(blk_lo) * BLOCK_SIZE)
        call("s3dg_fill_controlled_range", self._h, self._dst(dst, need), int(length), int(blk_lo),
             int(blk_hi), int(dedup), fn, fd, int(entropy) & (2**64 - 1), self._s(stream))

    def fill_stream(self, dst, obj_size: int, n_objs: int, stride: int | None = None,
                    dedup: int = 1, compress=1, seed_base: int = 0, first_obj: int = 0,
                    stream=None) -> None:
        """n_objs equal objects, object j at dst + j*stride with entropy
        object_entropy(seed_base, first_obj + j)."""
        stride = obj_size if stride is None else stride
        need = (int(n_objs) - 1) * int(stride) + int(obj_size) if n_objs > 0 and obj_size > 0 else 0
        fn, fd = compress_ratio(compress)
        call("s3dg_fill_controlled_stream", self._h, self._dst(dst, need), int(obj_size), int(stride),
             int(n_objs), int(dedup), fn, fd, int(seed_base) & (2**64 - 1), int(first_obj),
             self._s(stream))

    def fill_batch(self, dst, objects, stream=None) -> None:
        """objects: iterable of (dst_off, size, entropy, dedup, compress).

        The descriptors are checked here first (bounds against `dst`), and the
        library validates them again sub-batch by sub-batch (16 Ki objects,
        doubling) while earlier sub-batches are already enqueued: a call that
        raises on an invalid descriptor past the first sub-batch may have
        written the objects before it (include/s3dlio_gpu.h)."""
        objs = list(objects)
        arr = (ObjDesc * max(1, len(objs)))()
        need = 0
        for k, (off, size, ent, dd, comp) in enumerate(objs):
            fn, fd = compress_ratio(comp)
            arr[k] = ObjDesc(int(off), int(size), int(ent) & (2**64 - 1), int(dd), fn, fd)
            if size:
                need = max(need, int(off) + int(size))
        call("s3dg_fill_controlled_batch", self._h, self._dst(dst, need), arr, len(objs), self._s(stream))

    def xoshiro_fill(self, dst, nbytes: int | None = None, chunk_bytes: int = 2 << 20,
                     seed_base: int = 0, stream=None) -> None:
        """Keystream fill, chunk k = Xoshiro256PlusPlus::seed_from_u64(seed_base + k)
        .fill_bytes(chunk) (src/data_formats/npz.rs:376-383)."""
        n = _nbytes(dst) if nbytes is None else int(nbytes)
        call("s3dg_xoshiro_fill", self._h, self._dst(dst, n), n, int(chunk_bytes),
             int(seed_base) & (2**64 - 1), self._s(stream))

    def dgen_fill(self, dst, obj_size: int, blk_lo: int = 0, blk_hi: int | None = None,
                  dedup: int = 1, compress=1, seed: int = 0, stream=None) -> None:
        """DG1 blocks [blk_lo, blk_hi) of an obj_size-byte object (1 MiB blocks)."""
        fn, fd = compress_ratio(compress)
        hi = (obj_size + (1 << 20) - 1) >> 20 if blk_hi is None else blk_hi
        need = max(0, min(int(hi) << 20, int(obj_size)) - (int(blk_lo) << 20))
        call("s3dg_dgen_fill", self._h, self._dst(dst, need), int(obj_size), int(blk_lo), int(hi),
             int(dedup), fn, fd, int(seed) & (2**64 - 1), self._s(stream))

    def dgen_fill_stream(self, dst, obj_size: int, n_objs: int, stride: int | None = None,
                         dedup: int = 1, compress=1, seed_base: int = 0, first_obj: int = 0,
                         stream=None) -> None:
        """n_objs DG1 objects in one launch, object j at dst + j*stride seeded
        object_entropy(seed_base, first_obj + j): the bytes of n_objs dgen_fill calls."""
        stride = obj_size if stride is None else stride
        need = (int(n_objs) - 1) * int(stride) + int(obj_size) if n_objs > 0 and obj_size > 0 else 0
        fn, fd = compress_ratio(compress)
        call("s3dg_dgen_fill_stream", self._h, self._dst(dst, need), int(obj_size), int(stride), int(n_objs),
             int(dedup), fn, fd, int(seed_base) & (2**64 - 1), int(first_obj), self._s(stream))

    def write_ceiling(self, dst, nbytes: int | None = None, pattern: int = 0xA5A5A5A5,
                      stream=None) -> None:
        n = _nbytes(dst) if nbytes is None else int(nbytes)
        call("s3dg_write_ceiling", self._h, self._dst(dst, n), n, int(pattern), self._s(stream))

    def write_ceiling_tiled(self, dst, nbytes: int | None = None, pattern: int = 0xA5A5A5A5,
                            stream=None) -> None:
        """Store-only kernel in the tiled fill shape (batch knobs + trailing record loads)."""
        n = _nbytes(dst) if nbytes is None else int(nbytes)
        call("s3dg_write_ceiling_tiled", self._h, self._dst(dst, n), n, int(pattern), self._s(stream))

    def write_ceiling_fill(self, dst, nbytes: int | None = None, pace: int = 0, stream=None) -> None:
        """The tiled fill itself with the PRNG chain and window patches compiled
        out (s3dg_write_ceiling_fill): the fill's own store-only bound; `pace`
        delays wave 0 by pace x 128 cycles where the fill plans its block."""
        n = _nbytes(dst) if nbytes is None else int(nbytes)
        call("s3dg_write_ceiling_fill", self._h, self._dst(dst, n), n, int(pace), self._s(stream))

    def sync(self, stream=None) -> None:
        call("s3dg_sync", self._h, 0 if stream is None else _stream(stream))

    def release_stream(self, stream) -> None:
        """Drain `stream` and free this context's launch state for it (tile
        maps, batch staging; s3dg_stream_release).  Call before a stream the
        context launched on goes away."""
        call("s3dg_stream_release", self._h, _stream(stream))

    def stream_state_count(self) -> int:
        n = ctypes.c_uint64()
        call("s3dg_stream_state_count", self._h, ctypes.byref(n))
        return n.value


def xoshiro_jump(state, n: int) -> list[int]:
    """Host jump-ahead of a Xoshiro256 state by n steps (the kernels' method)."""
    s = (ctypes.c_uint64 * 4)(*[int(v) & (2**64 - 1) for v in state])
    call("s3dg_xoshiro_jump", s, int(n))
    return list(s)


def device_count() -> int:
    n = ctypes.c_int()
    call("s3dg_device_count", ctypes.byref(n))
    return n.value


def host_slots() -> list[int]:
    """Devices of the host-buffer drop-ins' slots (include/s3dlio_gpu.h): one
    per visible GPU unless S3DLIO_GPU_DEVICE / S3DLIO_GPU_DEVICES say otherwise."""
    n = ctypes.c_int()
    call("s3dg_host_slot_count", ctypes.byref(n))
    out = []
    for k in range(n.value):
        d = ctypes.c_int()
        call("s3dg_host_slot_device", k, ctypes.byref(d))
        out.append(d.value)
    return out


def host_context(slot: int = -1) -> Context:
    """A host slot's context (borrowed: owned by the pool); slot < 0 takes the
    next slot round-robin."""
    h = c_vp()
    call("s3dg_host_slot_context", int(slot), ctypes.byref(h))
    d = ctypes.c_int()
    call("s3dg_ctx_device", h, ctypes.byref(d))
    return Context._borrow(h.value, d.value)


def parse_devices(pin: str | None, lst: str | None, ndev: int, local_rank: str | None = None,
                  world_size: str | None = None) -> list[int]:
    """The slot device list for given env values (pure; s3dg_host_parse_devices_env):
    S3DLIO_GPU_DEVICE, S3DLIO_GPU_DEVICES, LOCAL_RANK, WORLD_SIZE."""
    out = (ctypes.c_int * 64)()
    n = ctypes.c_int()
    enc = lambda v: v.encode() if v is not None else None  # noqa: E731
    call("s3dg_host_parse_devices_env", enc(pin), enc(lst), enc(local_rank), enc(world_size), int(ndev), out, 64,
         ctypes.byref(n))
    return list(out[:n.value])

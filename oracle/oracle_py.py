"""Independent pure-Python restatement of s3dlio's payload generator.

TEST INFRASTRUCTURE ONLY: used by tests/ and tests/golden/make_golden.py to
cross-check the C oracle (oracle/s3dg_oracle.c).  Written separately from the
C file (closed-form zero-prefix lengths instead of the Bresenham loop, bytes
assembled with Python ints) so that the two restatements only agree if both
follow the reference:

  * fill_controlled_data   /root/reference/src/data_gen.rs:151-224
  * const_lens (closed form of the accumulator)  src/data_gen.rs:174-190
  * unique_blocks          src/data_gen.rs:162-167
  * rand 0.9.2 SmallRng = Xoshiro256++ seeded by SplitMix64; rand_core 0.9
    fill_bytes_via_next
  * npz x-fill             src/data_formats/npz.rs:376-383

Pure-Python loops: only for small cases (a few hundred KiB at most).
"""
from __future__ import annotations

import math

M64 = (1 << 64) - 1
BLK = 4096
HALF = 2048
MOD = 32


def _rotl(x: int, k: int) -> int:
    return ((x << k) | (x >> (64 - k))) & M64


def splitmix64_stream(state: int, n: int) -> list[int]:
    out = []
    for _ in range(n):
        state = (state + 0x9E3779B97F4A7C15) & M64
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        out.append(z ^ (z >> 31))
    return out


class Xoshiro256pp:
    def __init__(self, state):
        self.s = [int(v) & M64 for v in state]

    @classmethod
    def seed_from_u64(cls, seed: int) -> "Xoshiro256pp":
        return cls(splitmix64_stream(seed & M64, 4))

    def next_u64(self) -> int:
        s0, s1, s2, s3 = self.s
        r = (_rotl((s0 + s3) & M64, 23) + s0) & M64
        t = (s1 << 17) & M64
        s2 ^= s0
        s3 ^= s1
        s1 ^= s2
        s0 ^= s3
        s2 ^= t
        s3 = _rotl(s3, 45)
        self.s = [s0, s1, s2, s3]
        return r

    def next_u32(self) -> int:
        return self.next_u64() >> 32

    def fill_bytes(self, n: int) -> bytes:
        out = bytearray()
        while n - len(out) >= 8:
            out += self.next_u64().to_bytes(8, "little")
        tail = n - len(out)
        if tail > 4:
            out += self.next_u64().to_bytes(8, "little")[:tail]
        elif tail > 0:
            out += self.next_u32().to_bytes(4, "little")[:tail]
        return bytes(out)


def base_block(seed: int) -> bytes:
    return Xoshiro256pp.seed_from_u64(seed).fill_bytes(BLK)


def unique_blocks(nblocks: int, dedup: int) -> int:
    d = 1 if dedup == 0 else dedup
    if d <= 1:
        return nblocks
    q = nblocks / d                      # f64 division, as `as f64 / as f64`
    r = math.floor(q)                    # f64::round: half away from zero
    if q - r >= 0.5:
        r += 1
    return max(1, int(r))


def compress_ratio(compress) -> tuple[int, int]:
    """Integer c -> (c-1, c) as src/data_gen.rs:169-173; rational p/q given
    as a (p, q) tuple -> (p-q, p) (build-defined generalisation)."""
    if isinstance(compress, tuple):
        p, q = compress
        if p <= q:
            return 0, 1
        return p - q, p
    return (compress - 1, compress) if compress > 1 else (0, 1)


def const_len(k: int, f_num: int, f_den: int) -> int:
    total = f_num * BLK
    floor_len, rem = divmod(total, f_den)
    return floor_len + ((k + 1) * rem) // f_den - (k * rem) // f_den


def object_entropy(seed_base: int, j: int) -> int:
    return (seed_base + (j << 32)) & M64


def fill_controlled(length: int, dedup: int, f_num: int, f_den: int,
                    entropy: int, base: bytes) -> bytes:
    if length == 0:
        return b""
    nb = -(-length // BLK)
    U = unique_blocks(nb, dedup)
    out = bytearray()
    for i in range(nb):
        L = min(BLK, length - i * BLK)
        u = i % U
        rng = Xoshiro256pp.seed_from_u64((u + entropy) & M64)
        blk = bytearray(base[:L])
        c = min(const_len(u, f_num, f_den), L)
        blk[:c] = bytes(c)
        m = min(L - c, MOD)
        if m > 0:
            blk[c:c + m] = rng.fill_bytes(m)
            so = max(HALF, c)
            if so + m <= L:
                blk[so:so + m] = rng.fill_bytes(m)
        out += blk
    return bytes(out)


def xoshiro_chunks(length: int, chunk: int, seed_base: int) -> bytes:
    out = bytearray()
    k = 0
    while len(out) < length:
        n = min(chunk, length - len(out))
        out += Xoshiro256pp.seed_from_u64((seed_base + k) & M64).fill_bytes(n)
        k += 1
    return bytes(out)


def dgen_fill(size: int, dedup: int, f_num: int, f_den: int, seed: int) -> bytes:
    """DG1 (build-defined dgen-contract layout): independent restatement."""
    B = 1 << 20
    nb = -(-size // B)
    U = unique_blocks(nb, 1 if dedup == 0 else dedup)
    out = bytearray()
    for i in range(nb):
        L = min(B, size - i * B)
        blk = bytearray(Xoshiro256pp.seed_from_u64(seed ^ (((i % U) * 0x9E3779B97F4A7C15) & M64)).fill_bytes(L))
        z = (L * f_num) // f_den
        blk[:z] = bytes(z)
        out += blk
    return bytes(out)


def random_data(size: int, entropy: int, base: bytes) -> bytes:
    """Seeded analogue of generate_random_data (src/data_gen.rs:102-132), per-block seeds."""
    out = bytearray()
    i = 0
    while len(out) < size:
        bs = min(BLK, size - len(out))
        blk = bytearray(base[:bs])
        rng = Xoshiro256pp.seed_from_u64((entropy + i) & M64)
        m = min(bs, MOD)
        blk[:m] = rng.fill_bytes(m)
        if bs > HALF:
            blk[bs - MOD:] = rng.fill_bytes(MOD)
        out += blk
        i += 1
    return bytes(out)

"""CPU: pin the oracle against the PRNG known-answer vectors and the golden
fixtures, and cross-check the C and Python restatements."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle_py as P

MiB = 1 << 20


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def test_kat_splitmix64(oracle):
    kat = load("kat.json")
    assert [f"0x{v:016x}" for v in oracle.splitmix64(0, 4)] == kat["splitmix64_state0"]
    assert [f"0x{v:016x}" for v in P.splitmix64_stream(0, 4)] == kat["splitmix64_state0"]


def test_kat_xoshiro256pp(oracle):
    kat = load("kat.json")
    assert oracle.xoshiro_stream([1, 2, 3, 4], 4) == kat["xoshiro256pp_state_1234"]
    r = P.Xoshiro256pp([1, 2, 3, 4])
    assert [r.next_u64() for _ in range(4)] == kat["xoshiro256pp_state_1234"]
    assert [f"0x{v:016x}" for v in oracle.xoshiro_seeded_stream(0, 2)] == \
        kat["xoshiro256pp_seed_from_u64_0"]


def test_kat_rand_crate_vectors(oracle):
    """Ten-value known answers from the rand crates' own tests (rand_xoshiro
    0.7 / rand 0.9 Xoshiro256PlusPlus `reference` and rand 0.9
    `stable_seed_from_u64`; the crates are not in the checkout, the values
    are restated in tests/golden/make_golden.py).  The second pins the
    seed_from_u64 (SplitMix64) + next_u64 path every block seed of
    src/data_gen.rs:203 takes, in both oracles and the library's host jump."""
    kat = load("kat.json")
    assert oracle.xoshiro_stream([1, 2, 3, 4], 10) == kat["xoshiro256pp_state_1234_x10"]
    assert oracle.xoshiro_seeded_stream(0, 10) == kat["rand_seed_from_u64_0_x10"]
    r = P.Xoshiro256pp.seed_from_u64(0)
    assert [r.next_u64() for _ in range(10)] == kat["rand_seed_from_u64_0_x10"]


def test_fill_bytes_tail_rule():
    """1..4-byte tails take next_u32 = high half of next_u64 (rand_core 0.9)."""
    kat = load("kat.json")
    r = P.Xoshiro256pp.seed_from_u64(42)
    w0, w1 = r.next_u64(), r.next_u64()
    assert bytes.fromhex(kat["fill_bytes_seed42_len12"]) == \
        w0.to_bytes(8, "little") + (w1 >> 32).to_bytes(4, "little")
    assert bytes.fromhex(kat["fill_bytes_seed42_len13"]) == \
        w0.to_bytes(8, "little") + w1.to_bytes(8, "little")[:5]


def test_base_block_fixture(oracle, golden_base):
    assert bytes(oracle.base_block(0xBA5EB10C00000000)) == golden_base
    assert P.base_block(0xBA5EB10C00000000) == golden_base


def test_edge_fixtures(oracle, golden_base):
    base = np.frombuffer(golden_base, np.uint8)
    for c in load("edge_cases.json")["cases"]:
        got = oracle.fill_controlled(c["len"], c["dedup"], c["f_num"], c["f_den"],
                                     int(c["entropy"]), base)
        assert sha(got) == c["sha256"], c


def test_blob_fixtures(oracle, golden_base):
    base = np.frombuffer(golden_base, np.uint8)
    for name, (L, d, comp, e) in {"blob_4097_d1_c3": (4097, 1, 3, 11),
                                  "blob_12288_d2_c2": (12288, 2, 2, 12),
                                  "blob_8192_d1_c1": (8192, 1, 1, 13)}.items():
        with open(os.path.join(GOLDEN, name + ".bin"), "rb") as f:
            exp = f.read()
        fn, fd = P.compress_ratio(comp)
        assert bytes(oracle.fill_controlled(L, d, fn, fd, e, base)) == exp
        assert P.fill_controlled(L, d, fn, fd, e, golden_base) == exp


def test_cfg1_digests(oracle, golden_base):
    g = load("cfg1_1000x64KiB.json")
    base = np.frombuffer(golden_base, np.uint8)
    out = oracle.fill_stream(g["size"], g["objects"], 1, 0, 1, int(g["seed_base"], 16), 0, base,
                             threads=4)
    size = g["size"]
    digests = [sha(out[j * size:(j + 1) * size]) for j in range(g["objects"])]
    assert digests == g["sha256"]
    assert sha("".join(digests).encode()) == g["sha256_of_digests"]


def test_xoshiro_chunk_fixtures(oracle):
    for c in load("xoshiro_chunks.json"):
        assert sha(oracle.xoshiro_chunks(c["len"], c["chunk"], c["seed_base"])) == c["sha256"]


@pytest.mark.parametrize("nb,d", [(2048, 4), (2048, 3), (5, 2), (3, 2), (1, 2), (7, 100),
                                  (2049, 2), (10, 4), (6, 4), (2, 4)])
def test_unique_blocks_rounding(oracle, nb, d):
    """round-half-away-from-zero of nb/d, min 1 (src/data_gen.rs:162-167)."""
    exp = max(1, int(np.floor(nb / d + 0.5)))
    assert oracle.unique_blocks(nb, d) == exp == P.unique_blocks(nb, d)


def test_const_len_closed_form_matches_accumulator():
    """The kernels' closed form equals the reference's Bresenham loop."""
    for (fn, fd) in [(1, 2), (2, 3), (4, 5), (1, 3), (126, 127), (4999, 5000), (2, 5)]:
        total = fn * 4096
        floor_len, rem = divmod(total, fd)
        acc, seq = 0, []
        for _ in range(3000):
            acc += rem
            if acc >= fd:
                acc -= fd
                seq.append(floor_len + 1)
            else:
                seq.append(floor_len)
        assert [P.const_len(k, fn, fd) for k in range(3000)] == seq


def test_mt_equals_single_thread(oracle, golden_base):
    base = np.frombuffer(golden_base, np.uint8)
    a = oracle.fill_stream(4096 * 33 + 5, 7, 3, 2, 3, 99, 5, base, stride=4096 * 34, threads=1)
    b = oracle.fill_stream(4096 * 33 + 5, 7, 3, 2, 3, 99, 5, base, stride=4096 * 34, threads=6)
    assert np.array_equal(a, b)


def test_zero_fraction_and_dedup_structure(oracle, golden_base):
    """Structural contract on the in-tree algorithm:
    zero fraction ~ (c-1)/c, unique 4 KiB blocks ~ nblocks/dedup."""
    base = np.frombuffer(golden_base, np.uint8)
    n = 8 * 2**20
    x = oracle.fill_controlled(n, 4, 1, 2, 5, base)
    blocks = x.reshape(-1, 4096)
    assert len({b.tobytes() for b in blocks}) == 512
    zero_frac = float((blocks[:, :2048] == 0).mean())
    assert zero_frac == 1.0
    y = oracle.fill_controlled(n, 1, 2, 3, 5, base)
    zf = float((y == 0).mean())
    assert abs(zf - 2 / 3) < 0.01


@pytest.mark.parametrize("size,chunk", [(1, 1), (13, 5), (4100, 3), (MiB + 9, 777), (3 * MiB + 5, 65536),
                                        (2 * MiB + 4, 1 << 20), (5 * MiB + 1, 777777)])
@pytest.mark.parametrize("d,fn,fd", [(1, 0, 1), (2, 1, 2), (3, 2, 3)])
def test_dgen_stream_port_equals_dgen_fill(oracle, size, chunk, d, fn, fd):
    """The CPU streaming port behind bench.py's fill_chunk baselines writes
    the DG1 bytes whatever the chunk size."""
    assert bytes(oracle.dgen_stream(size, d, fn, fd, 77 + size, chunk)) == bytes(oracle.dgen_fill(size, d, fn, fd,
                                                                                                77 + size))

"""Generate the committed golden fixtures under tests/golden/.

    python tests/golden/make_golden.py

Provenance: the reference (Rust, needs cargo + the
external rand/dgen crates) cannot be built or imported in this image and
holds no byte-level vectors for this path.  The fixtures are therefore the
output of the C restatement (oracle/s3dg_oracle.c), accepted only where the
independent Python restatement (oracle/oracle_py.py) produces the same bytes,
and anchored by the published PRNG known-answer vectors in kat.json.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle_c as C  # noqa: E402
from oracle import oracle_py as P  # noqa: E402

BASE_SEED = 0xBA5EB10C00000000
SEED_BASE = 0x5EED000000000001

# Published known answers:
#  * SplitMix64 from state 0 (Vigna's splitmix64.c reference output)
#  * Xoshiro256++ from state [1,2,3,4] (xoshiro256plusplus.c reference output,
#    also the rand_xoshiro test vector)
KAT = {
    "splitmix64_state0": ["0xe220a8397b1dcdaf", "0x6e789e6aa1b965f4",
                          "0x06c45d188009454f", "0xf88bb8a8724c81ec"],
    "xoshiro256pp_state_1234": [41943041, 58720359, 3588806011781223, 3591011842654386],
    # the ten values of the `reference` test of rand_xoshiro 0.7's (and rand
    # 0.9's) Xoshiro256PlusPlus (from_seed of the little-endian words 1,2,3,4;
    # values produced by the xoshiro256plusplus.c reference implementation)
    "xoshiro256pp_state_1234_x10": [41943041, 58720359, 3588806011781223, 3591011842654386,
                                    9228616714210784205, 9973669472204895162, 14011001112246962877,
                                    12406186145184390807, 15849039046786891736, 10450023813501588000],
    # rand 0.9's `stable_seed_from_u64` test: Xoshiro256PlusPlus::seed_from_u64(0)
    # (the SmallRng seeding path of src/data_gen.rs:203), ten next_u64 outputs
    "rand_seed_from_u64_0_x10": [5987356902031041503, 7051070477665621255, 6633766593972829180,
                                 211316841551650330, 9136120204379184874, 379361710973160858,
                                 15813423377499357806, 15596884590815070553, 5439680534584881407,
                                 1369371744833522710],
}

# (length, dedup, compress, entropy) — compress is an int or a (p, q) ratio
EDGE_CASES = []
for L in [1, 4, 5, 7, 8, 9, 31, 32, 33, 63, 100, 2047, 2048, 2049, 2080, 2081, 4064,
          4065, 4095, 4096, 4097, 6144, 8191, 8192, 12288 + 2730, 65536, 65536 + 17]:
    for d in [0, 1, 2, 3]:
        for c in [0, 1, 2, 3, 5]:
            EDGE_CASES.append((L, d, c, 0x0123456789ABCDEF))
for c in [127, 128, 129, 130, 200, 1000, 4096, 5000, (3, 2), (5, 3), (7, 4)]:
    for L in [4096, 4096 * 5 + 123]:
        EDGE_CASES.append((L, 1, c, 7))
for d in [4, 7, 16, 100, 1000, 5000]:
    EDGE_CASES.append((40960 + 1, d, 2, 99999))
EDGE_CASES.append((65536, 1, 1, 2**64 - 3))          # entropy wrap-around in u + E
EDGE_CASES.append((65536, 2, 3, 2**64 - 1))


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def ratio(c):
    return P.compress_ratio(c)


def main() -> None:
    C.build()
    # --- KATs -----------------------------------------------------------------
    got_sm = [f"0x{v:016x}" for v in C.splitmix64(0, 4)]
    assert got_sm == KAT["splitmix64_state0"], got_sm
    got_x = C.xoshiro_stream([1, 2, 3, 4], 4)
    assert got_x == KAT["xoshiro256pp_state_1234"], got_x
    seeded0 = C.xoshiro_seeded_stream(0, 2)
    _r = P.Xoshiro256pp.seed_from_u64(0)
    assert seeded0 == [_r.next_u64(), _r.next_u64()], seeded0
    kat = dict(KAT)
    kat["xoshiro256pp_seed_from_u64_0"] = [f"0x{v:016x}" for v in seeded0]
    # fill_bytes tail rule: 1..4-byte tails come from next_u32 = next_u64 >> 32
    kat["fill_bytes_seed42_len13"] = P.Xoshiro256pp.seed_from_u64(42).fill_bytes(13).hex()
    kat["fill_bytes_seed42_len12"] = P.Xoshiro256pp.seed_from_u64(42).fill_bytes(12).hex()
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)

    base = C.base_block(BASE_SEED)
    assert bytes(base) == P.base_block(BASE_SEED)
    with open(os.path.join(HERE, "base_block_ba5eb10c.bin"), "wb") as f:
        f.write(bytes(base))

    # --- edge sweep ---------------------------------------------------------------
    edges = []
    for (L, d, c, e) in EDGE_CASES:
        fn, fd = ratio(c)
        a = C.fill_controlled(L, d, fn, fd, e, base)
        b = P.fill_controlled(L, d, fn, fd, e, bytes(base))
        assert bytes(a) == b, (L, d, c, e)
        edges.append({"len": L, "dedup": d, "compress": list(c) if isinstance(c, tuple) else c,
                      "f_num": fn, "f_den": fd, "entropy": str(e), "sha256": sha(a)})
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump({"base_seed": hex(BASE_SEED), "cases": edges}, f, indent=0)

    # a few raw blobs (inputs are the parameters; expected output is the file)
    for name, (L, d, c, e) in {"blob_4097_d1_c3": (4097, 1, 3, 11),
                               "blob_12288_d2_c2": (12288, 2, 2, 12),
                               "blob_8192_d1_c1": (8192, 1, 1, 13)}.items():
        fn, fd = ratio(c)
        a = C.fill_controlled(L, d, fn, fd, e, base)
        with open(os.path.join(HERE, name + ".bin"), "wb") as f:
            f.write(bytes(a))

    # --- BASELINE config 1: 1000 x 64 KiB, d=1 c=1 -----------------------------------
    n, size = 1000, 65536
    out = C.fill_stream(size, n, 1, 0, 1, SEED_BASE, 0, base)
    digests = []
    for j in range(n):
        obj = out[j * size:(j + 1) * size]
        ent = P.object_entropy(SEED_BASE, j)
        assert bytes(obj) == P.fill_controlled(size, 1, 0, 1, ent, bytes(base)), j
        digests.append(sha(obj))
    cfg1 = {"objects": n, "size": size, "dedup": 1, "compress": 1,
            "seed_base": hex(SEED_BASE), "base_seed": hex(BASE_SEED),
            "entropy_rule": "seed_base + j * 2**32",
            "sha256": digests,
            "sha256_of_digests": sha("".join(digests).encode())}
    with open(os.path.join(HERE, "cfg1_1000x64KiB.json"), "w") as f:
        json.dump(cfg1, f, indent=0)

    # --- npz x-fill (src/data_formats/npz.rs:376-383) ------------------------------
    xs = []
    for (L, chunk, sb) in [(5 * 2**20 + 13, 2 * 2**20, 0), (100000, 4096, 0), (4096 * 3 + 7, 4096, 5)]:
        a = C.xoshiro_chunks(L, chunk, sb)
        if L <= 200000:
            assert bytes(a) == P.xoshiro_chunks(L, chunk, sb)
        else:
            assert bytes(a[:chunk]) == P.xoshiro_chunks(chunk, chunk, sb)
        xs.append({"len": L, "chunk": chunk, "seed_base": sb, "sha256": sha(a)})
    with open(os.path.join(HERE, "xoshiro_chunks.json"), "w") as f:
        json.dump(xs, f, indent=1)
    print("golden fixtures written")


if __name__ == "__main__":
    main()

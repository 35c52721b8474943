"""Object assembly: generate_object (src/data_gen.rs:29-94) and the format
builders (src/data_formats/{raw,tfrecord,npz}.rs).

CPU tests: the C-ABI framing vs oracle/format_oracle.py, which is itself pinned
by the reference's fixtures (tests/object_format_tests.rs:19-125).  GPU tests:
payload bytes vs the C oracle (random-data layout / DG1) + framing.
"""
import io
import struct
import zipfile
import zlib

import numpy as np
import pytest

from oracle import format_oracle as F


@pytest.fixture(scope="module")
def S():
    import s3dlio_amd
    return s3dlio_amd


# ---- reference known-answer cases (tests/object_format_tests.rs) ---------------------

def test_oracle_raw_roundtrip():                                     # :19-24
    d = bytes([0, 1, 2, 3, 4, 5, 255])
    assert F.build_raw(d) == d


def test_oracle_npz_roundtrip_and_content():                          # :27-58
    data = b"\x42" * 5
    z = zipfile.ZipFile(io.BytesIO(F.build_npz(5, data)))
    assert z.testzip() is None and z.namelist() == ["data.npy"]
    c = z.read("data.npy")
    assert c.startswith(b"\x93NUMPY")
    hl = struct.unpack_from("<H", c, 8)[0]
    assert c[10 + hl:] == data
    assert (10 + hl) % 16 == 0


def test_oracle_tfrecord_index_and_stream_consistency():              # :86-125
    records, rs = 3, 4
    data = bytes(i % 256 for i in range(records * rs))
    tf, idx = F.build_tfrecord_with_index(records, rs, data)
    assert len(idx) == records * 16
    off0, len0 = struct.unpack_from("<QQ", idx, 0)
    assert off0 == 0 and len0 == 8 + 4 + rs + 4
    assert len(tf) == sum(struct.unpack_from("<Q", idx, 16 * i + 8)[0] for i in range(records))


def test_oracle_tfrecord_masked_crc_definition():
    # TensorFlow's masked CRC32C convention applied to crc32fast (tfrecord.rs:10-12)
    assert F.masked_crc(0) == 0xA282EAD8
    assert F.masked_crc(0xFFFFFFFF) == (0xFFFFFFFF + 0xA282EAD8) & 0xFFFFFFFF


# ---- C ABI builders vs the oracle (host code; no GPU) ----------------------------

def test_capi_raw(S):
    d = bytes([0, 1, 2, 3, 4, 5, 255])
    assert S.build_raw(d) == d


@pytest.mark.parametrize("records,rs", [(0, 4), (1, 0), (3, 4), (7, 1000), (2, 65537)])
def test_capi_tfrecord_matches_oracle(S, records, rs):
    rng = np.random.default_rng(records * 7 + rs)
    data = rng.integers(0, 256, records * rs, dtype=np.uint8).tobytes()
    assert S.build_tfrecord_with_index(records, rs, data) == F.build_tfrecord_with_index(records, rs, data)
    assert S.build_tfrecord(records, rs, data) == F.build_tfrecord(records, rs, data)


def test_capi_tfrecord_rejects_short_data(S):
    with pytest.raises(ValueError):
        S.build_tfrecord(3, 4, b"\x00" * 11)


@pytest.mark.parametrize("elements", [0, 1, 5, 99, 100, 4096, 123457])
def test_capi_npz_matches_oracle_and_numpy(S, elements):
    data = np.random.default_rng(elements).integers(0, 256, elements, dtype=np.uint8).tobytes()
    b = S.build_npz(elements, 1, data)
    assert b == F.build_npz(elements, data)
    a = np.load(io.BytesIO(b))["data"]
    assert a.dtype == np.uint8 and a.shape == (elements,) and a.tobytes() == data


@pytest.mark.parametrize("t,elements,es,expect", [
    ("RAW", 10, 3, 30), ("TFRECORD", 10, 3, 190), ("NPZ", 5, 1, len(F.build_npz(5, b"\0" * 5))),
    ("zeros", 4, 4, 16)])
def test_object_size(S, t, elements, es, expect):
    assert S.object_size(S.ObjectType.from_str(t), elements, es) == expect


def test_object_type_from_str(S):
    # s3_utils.rs:362-371: case-insensitive, unknown -> Raw
    assert S.ObjectType.from_str("npz") == S.ObjectType.NPZ
    assert S.ObjectType.from_str("TfRecord") == S.ObjectType.TFRECORD
    assert S.ObjectType.from_str("hdf5") == S.ObjectType.HDF5
    assert S.ObjectType.from_str("anything") == S.ObjectType.RAW


def test_config_defaults(S):
    # config.rs:115-133
    c = S.Config.new_with_defaults("NPZ", 10, 4, 1, 1)
    assert not c.use_controlled and c.chunk_size == 256 * 1024
    assert c.data_gen_mode == S.DataGenMode.STREAMING
    assert S.Config.new_with_defaults(S.ObjectType.RAW, 1, 1, 2, 1).use_controlled
    assert S.Config.new_with_defaults(S.ObjectType.RAW, 1, 1, 1, 3).use_controlled


def test_hdf5_unavailable(S):
    # generate_object without the hdf5 feature fails (data_gen.rs:75-87)
    with pytest.raises(ValueError, match="HDF5"):
        S.generate_object(S.Config.new_with_defaults("HDF5", 4, 4, 1, 1), seed=1)


# ---- GPU: payload + framing -------------------------------------------------------

def _payload(oracle, golden_base, cfg, seed):
    total = cfg.elements * cfg.element_size
    if not cfg.use_controlled:
        return oracle.random_data(total, seed, np.frombuffer(golden_base, np.uint8)).tobytes()
    from s3dlio_amd import compress_ratio
    fn, fd = compress_ratio(max(1, cfg.compress_factor))
    return oracle.dgen_fill(total, max(1, cfg.dedup_factor), fn, fd, seed).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("t", ["RAW", "TFRECORD", "NPZ"])
@pytest.mark.parametrize("elements,es,dedup,comp", [
    (1, 1, 1, 1), (1, 5000, 1, 1), (3, 4096, 1, 1), (257, 4099, 1, 1),
    (64, 65536, 2, 3), (5, 3 * 2**20 + 17, 4, 2), (1, 9 * 2**20 + 1, 1, 5)])
def test_gpu_generate_object_vs_oracle(S, oracle, golden_base, gpu_ctx, t, elements, es, dedup, comp):
    cfg = S.Config.new_with_defaults(t, elements, es, dedup, comp)
    seed = elements * 1000003 + es
    got = bytes(S.generate_object(cfg, seed=seed))
    pay = _payload(oracle, golden_base, cfg, seed)
    if t == "RAW":
        exp = F.build_raw(pay)
    elif t == "TFRECORD":
        exp = F.build_tfrecord(elements, es, pay)
    else:
        exp = F.build_npz(elements, pay)
    assert len(got) == S.object_size(cfg.object_type, elements, es)
    assert got == exp


@pytest.mark.gpu
def test_gpu_generate_object_modes_agree(S, gpu_ctx):
    cfg = S.Config.new_with_defaults("RAW", 4, 300000, 2, 2)
    a = bytes(S.generate_object(cfg, seed=9))
    b = bytes(S.generate_object(cfg.with_data_gen_mode(S.DataGenMode.SINGLE_PASS), seed=9))
    assert a == b


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 31, 32, 33, 2048, 2049, 4096, 4097, 1 << 20, 5 * 2**20 + 3])
def test_gpu_random_data_vs_oracle(S, oracle, golden_base, gpu_ctx, n):
    """generate_random_data's layout (data_gen.rs:102-132), seeded: Context.random_data."""
    import torch
    buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    buf.fill_(0xAB)
    gpu_ctx.random_data(buf, n, entropy=n * 3 + 1)
    gpu_ctx.sync()
    h = buf.cpu().numpy()
    assert h[:n].tobytes() == oracle.random_data(n, n * 3 + 1, np.frombuffer(golden_base, np.uint8)).tobytes()
    assert (h[n:] == 0xAB).all()


@pytest.mark.gpu
def test_gpu_generate_random_data_unseeded(S, gpu_ctx):
    """Unseeded: time entropy + per-process random base block; sizes exact,
    successive calls differ.  Like the reference (data_gen.rs:102-132), every
    block is the same base block outside its two 32-B windows, so the output
    is highly compressible -- that is the reference's behaviour."""
    n = 3 * 2**20 + 5
    a, b = S.generate_random_data(n), S.generate_random_data(n)
    assert len(a) == len(b) == n and a != b
    blocks = np.frombuffer(a[:n - n % 4096], np.uint8).reshape(-1, 4096)
    assert (blocks[:, 32:4064] == blocks[0, 32:4064]).all()
    assert len({bytes(r[:32]) for r in blocks}) == len(blocks)
    assert len({bytes(r[-32:]) for r in blocks}) == len(blocks)
    assert len(zlib.compress(a, 1)) < 0.1 * n
    assert S.generate_random_data(0) == b""

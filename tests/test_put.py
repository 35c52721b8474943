"""PUT pipeline: per-object payloads -> file:// objects.

Reference: put (src/python_api/python_core_api.rs:777-818), build_uri_list
(:657-691), put_objects_with_random_data_and_type (src/s3_utils.rs:1717-1750),
FileSystemObjectStore::put (src/file_store.rs:550-569).  Parity anchor (SURVEY
§8f): sizes / counts and a file:// round trip; here every file is also compared
byte for byte with the oracle's payload + oracle framing, and the returned
CRC-32 with zlib's.
"""
import os
import zlib

import numpy as np
import pytest

from oracle import format_oracle as F

MiB = 1 << 20


@pytest.fixture(scope="module")
def S():
    import s3dlio_amd
    return s3dlio_amd


# ---- CPU: host logic ---------------------------------------------------------------

def test_build_uri_list(S):
    b, u = S.build_uri_list("s3://bkt/pre", "object-{}", 3)
    assert b == "bkt" and u == ["s3://bkt/pre/object-0", "s3://bkt/pre/object-1", "s3://bkt/pre/object-2"]
    b, u = S.build_uri_list("file:///tmp/a/b/", "f-{}-of-{}.npz", 2)
    assert b == "" and u == ["file:///tmp/a/b/f-0-of-2.npz", "file:///tmp/a/b/f-1-of-2.npz"]
    b, u = S.build_uri_list("az://cont", "x{}", 1)
    assert b == "cont" and u == ["az://cont/x0"]
    with pytest.raises(ValueError, match="scheme"):
        S.build_uri_list("no-scheme/path", "o{}", 1)


def test_put_rejects_non_file_targets(S):
    with pytest.raises(ValueError, match="file://"):
        S.put_objects(["s3://bkt/o"], 10)


def test_put_rejects_hdf5(S):
    cfg = S.Config.new_with_defaults("HDF5", 1, 10, 1, 1)
    with pytest.raises(ValueError, match="HDF5"):
        S.put_objects(["file:///tmp/never"], 10, config=cfg)


# ---- GPU: round trips --------------------------------------------------------------

def _expect(oracle, golden_base, kind, size, d, c, seed, j):
    from s3dlio_amd import compress_ratio
    fn, fd = compress_ratio(max(1, c))
    e = oracle.object_entropy(seed, j)
    base = np.frombuffer(golden_base, np.uint8)
    if kind == "controlled":
        return oracle.fill_controlled(size, max(1, d), fn, fd, e, base).tobytes()
    if kind == "random":
        return oracle.random_data(size, e, base).tobytes()
    return oracle.dgen_fill(size, max(1, d), fn, fd, e).tobytes()


def _frame(t, size, payload):
    if t == "TFRECORD":
        return F.build_tfrecord(1, size, payload)
    if t == "NPZ":
        return F.build_npz(1, payload)
    return payload


def _dump_failure(oracle, kind, t, size, d, c, seed, j, got, pay, bad):
    """Diagnostics for a payload mismatch (written under gpurun_out/ when present)."""
    import json
    from s3dlio_amd import compress_ratio
    info = {"case": [kind, t, size, d, c, seed, j], "ndiff": int(bad.size), "first": bad[:8].tolist()}
    off = len(got) - size - (4 if t == "TFRECORD" else 0) - (76 if t == "NPZ" else 0)
    off = {"RAW": 0, "TFRECORD": 12}.get(t, off)
    gp = np.frombuffer(got[off:off + size], np.uint8)
    info["payload_equal"] = gp.tobytes() == pay
    fn, fd = compress_ratio(max(1, c))
    hits = []
    if kind == "dgen":
        for dj in range(-3, 4):
            e2 = oracle.object_entropy(seed, j + dj) if j + dj >= 0 else None
            if e2 is not None and oracle.dgen_fill(size, max(1, d), fn, fd, e2).tobytes() == gp.tobytes():
                hits.append(f"dgen seed of object {j + dj}")
        xs = oracle.xoshiro_chunks(size, 1 << 20, oracle.object_entropy(seed, j)).tobytes()
        if xs == gp.tobytes():
            hits.append("seed_mode 0")
    info["matches"] = hits
    info["got_zero_frac"] = float((gp == 0).mean())
    blk = 1 << 20
    nb = (size + blk - 1) // blk
    per_block = []
    for b in range(nb):
        a, z = b * blk, min(size, (b + 1) * blk)
        per_block.append(int(np.count_nonzero(gp[a:z] != np.frombuffer(pay[a:z], np.uint8))))
    info["diff_per_MiB_block"] = per_block[:64]
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/put_fail_{kind}_{t}_{j}.json", "w") as f:
        json.dump(info, f)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,t,n,size,d,c", [
    ("controlled", "RAW", 70, 3 * MiB + 5, 2, 3),     # one 256 MiB chunk of packed objects, ragged size
    # 7 chunks of 64 packed objects: the 4-slot pinned ring wraps (chunk index >= kHostSlots)
    ("controlled", "RAW", 400, 4 * MiB, 1, 2),
    ("dgen", "RAW", 1, 1300 * MiB + 3, 2, 2),         # one object in 6 slot-sized pieces (ring wraps)
    ("random", "TFRECORD", 300, 5000, 1, 1),
    ("dgen", "NPZ", 5, 2 * MiB + 17, 2, 2),
    ("controlled", "RAW", 1, 600 * MiB + 123, 1, 1),  # split into 3 slot-sized pieces
    ("dgen", "TFRECORD", 1, 300 * MiB + 7, 1, 4),     # split, DG1 pieces on 1 MiB blocks
    ("random", "RAW", 3, 4096, 1, 1),
    ("controlled", "NPZ", 4, 1, 1, 1),
])
def test_gpu_put_round_trip(S, oracle, golden_base, gpu_ctx, tmp_path, kind, t, n, size, d, c):
    uris = [f"file://{tmp_path}/sub/dir/obj-{j}" for j in range(n)]
    cfg = S.Config.new_with_defaults(t, 1, size, d, c)
    seed = 0x1234 + n
    r = S.put_objects(uris, size, 16, cfg, seed=seed, payload=kind, context=gpu_ctx)
    framed = S.object_size(cfg.object_type, 1, size)
    assert r.objects == n and r.bytes == n * framed
    for j in range(n):
        got = open(f"{tmp_path}/sub/dir/obj-{j}", "rb").read()
        assert len(got) == framed
        pay = _expect(oracle, golden_base, kind, size, d, c, seed, j)
        exp = _frame(t, size, pay)
        if got != exp:
            g, e = np.frombuffer(got, np.uint8), np.frombuffer(exp, np.uint8)
            bad = np.nonzero(g != e)[0]
            _dump_failure(oracle, kind, t, size, d, c, seed, j, got, pay, bad)
            raise AssertionError(f"object {j}: {bad.size} bytes differ, first at {bad[:4].tolist()}; "
                                 f"file crc {zlib.crc32(got):08x} returned {r.checksums[j]:08x} "
                                 f"payload crc expected {zlib.crc32(pay):08x}")
        assert r.checksums[j] == zlib.crc32(got)
    assert r.checksum_str(0).startswith("crc32c:")


@pytest.mark.gpu
def test_gpu_put_zero_size_and_thread_counts(S, gpu_ctx, tmp_path):
    r = S.put_objects([f"file://{tmp_path}/z{j}" for j in range(3)], 0,
                      config=S.Config.new_with_defaults("TFRECORD", 1, 0, 1, 1), seed=1, context=gpu_ctx)
    assert r.objects == 3 and all(os.path.getsize(f"{tmp_path}/z{j}") == 16 for j in range(3))
    # the writer count changes nothing in the bytes
    a = S.put_objects([f"file://{tmp_path}/a{j}" for j in range(40)], 70000, 1, seed=5,
                      payload="controlled", context=gpu_ctx)
    b = S.put_objects([f"file://{tmp_path}/b{j}" for j in range(40)], 70000, 64, seed=5,
                      payload="controlled", context=gpu_ctx)
    assert a.checksums == b.checksums
    assert len(set(a.checksums)) == 40       # one payload per object, not one buffer for all


@pytest.mark.gpu
def test_gpu_put_surface(S, gpu_ctx, tmp_path):
    """python_core_api.rs:777-818 defaults: template object-{}, parents created."""
    S.put(f"file://{tmp_path}/bucket/prefix", 12, size=3 * MiB, dedup_factor=4,
          compress_factor=2, max_in_flight=8, seed=7)
    files = sorted(os.listdir(f"{tmp_path}/bucket/prefix"))
    assert files == sorted(f"object-{i}" for i in range(12))
    for f in files:
        b = open(f"{tmp_path}/bucket/prefix/{f}", "rb").read()
        assert len(b) == 3 * MiB
        z = np.frombuffer(b, np.uint8)
        # DG1 with c=2: the first half of each 1 MiB block is zero
        assert not z[:MiB // 2].any() and z[MiB // 2:MiB].any()
    S.put(f"file://{tmp_path}/t", 2, template="f-{}-of-{}", size=100, object_type="npz", seed=1)
    assert sorted(os.listdir(f"{tmp_path}/t")) == ["f-0-of-2", "f-1-of-2"]


@pytest.mark.gpu
def test_gpu_put_io_error_is_loud(S, gpu_ctx, tmp_path):
    blocker = tmp_path / "file"
    blocker.write_bytes(b"x")
    with pytest.raises(OSError):
        S.put_objects([f"file://{blocker}/under-a-file"], 4096, seed=1, context=gpu_ctx)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,t,n,size,d,c", [
    ("controlled", "RAW", 70, 3 * MiB + 5, 2, 3),
    ("dgen", "TFRECORD", 9, 2 * MiB + 17, 2, 2),
    ("controlled", "NPZ", 3, 300 * MiB + 9, 1, 3),        # split objects on every lane
])
def test_gpu_put_lanes_give_identical_files(S, oracle, golden_base, gpu_ctx, tmp_path, kind, t, n, size, d, c):
    """s3dg_put_objects_multi: 1, 2 and 3 lanes (contexts) on this GPU write
    the same files and return the same checksums (object j's bytes depend
    only on (seed, j)); spot-check against the oracle."""
    cfg = S.Config.new_with_defaults(t, 1, size, d, c)
    res = {}
    for lanes in (1, 2, 3):
        out = tmp_path / f"l{lanes}"
        uris = [f"file://{out}/o-{j}" for j in range(n)]
        r = S.put_objects(uris, size, 16, cfg, seed=77, payload=kind, devices=[0] * lanes)
        assert r.objects == n
        res[lanes] = (r.checksums, [zlib.crc32(open(f"{out}/o-{j}", "rb").read()) for j in range(n)])
        assert res[lanes][0] == res[lanes][1]
    assert res[1] == res[2] == res[3]
    j = n - 1
    got = open(f"{tmp_path}/l3/o-{j}", "rb").read()
    assert got == _frame(t, size, _expect(oracle, golden_base, kind, size, d, c, 77, j))


@pytest.mark.gpu
def test_gpu_put_lane_error_is_loud(S, gpu_ctx, tmp_path):
    blocker = tmp_path / "file"
    blocker.write_bytes(b"x")
    uris = [f"file://{tmp_path}/ok-{j}" for j in range(5)] + [f"file://{blocker}/bad"]
    with pytest.raises(OSError):
        S.put_objects(uris, 8192, seed=1, devices=[0, 0])


@pytest.mark.gpu
def test_numa_local_pinned_alloc_roundtrip():
    """s3dg_host_alloc_pinned_local: pinned memory on the GPU's NUMA node,
    usable as a D2H target."""
    import ctypes
    import numpy as np
    import torch
    import s3dlio_amd as S
    from s3dlio_amd._lib import call
    node = ctypes.c_int(-2)
    call("s3dg_device_numa_node", 0, ctypes.byref(node))
    assert node.value >= -1
    ctx = S.Context(0)
    n = 8 << 20
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.fill_controlled(dev, n, dedup=1, compress=1, entropy=3)
    p = ctypes.c_void_p()
    call("s3dg_host_alloc_pinned_local", 0, n, ctypes.byref(p))
    try:
        call("s3dg_d2h_async", ctx._h, p.value, dev.data_ptr(), n, 0)
        call("s3dg_sync", ctx._h, 0)
        host = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p.value))
        assert np.array_equal(host, dev.cpu().numpy())
    finally:
        call("s3dg_host_free_pinned", p.value)
        ctx.close()

"""NPZ builder (generate_npz_bytes_raw, src/data_formats/npz.rs:322-434) and CRC-32."""
import io
import os
import zipfile
import zlib

import numpy as np
import pytest

from oracle import npz_oracle as N

SHAPES = [([7], "<f4", 1), ([64, 33, 3], "<f4", 5), ([1000, 1000], "<i8", 0),
          ([3, 5, 7, 11], "|u1", 100), ([0], "<f4", 1), ([], "<f4", 1), ([257], "<f2", 3)]


@pytest.mark.parametrize("shape,dtype,ns", SHAPES)
def test_oracle_archive_is_valid_npz(shape, dtype, ns):
    """The restated framing is a valid ZIP (stored CRCs verified by zipfile)
    that numpy.load reads back with the right shapes."""
    b = N.generate_npz_bytes_raw(shape, dtype, ns)
    assert zipfile.ZipFile(io.BytesIO(b)).testzip() is None
    if dtype in ("<f4", "<i8", "|u1"):
        z = np.load(io.BytesIO(b))
        assert z["x"].shape == tuple(shape) and z["y"].shape == (ns,) and not z["y"].any()


@pytest.mark.parametrize("shape,dtype,ns", SHAPES)
def test_npz_size_matches_oracle(shape, dtype, ns):
    import s3dlio_amd as S
    assert S.npz_size(shape, dtype, ns) == len(N.generate_npz_bytes_raw(shape, dtype, ns))


def test_host_crc_helpers():
    import s3dlio_amd as S
    for n in (0, 1, 5, 4096, 100001):
        b = os.urandom(n)
        assert S.lib.s3dg_crc32_host(0, b, n) == zlib.crc32(b)
    a, b = os.urandom(12345), os.urandom(54321)
    assert S.crc32_combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(a + b)
    assert S.crc32_combine(zlib.crc32(a), 0, 0) == zlib.crc32(a)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,dtype,ns", SHAPES + [([6053, 6053, 1], "<f4", 1)])
def test_gpu_npz_byte_identical(shape, dtype, ns):
    """unet3d-style 140 MiB archive included (python_datagen_api.rs:389)."""
    import s3dlio_amd as S
    got = S.generate_npz_bytes(shape, dtype, ns)
    assert memoryview(got).readonly and isinstance(got, S.BytesView)
    assert bytes(got) == N.generate_npz_bytes_raw(shape, dtype, ns)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 16383, 16384, 16385, 128 * 1024 * 8, 5 * 2**20 + 3,
                               300 * 2**20 + 77])
def test_gpu_crc32_vs_zlib(gpu_ctx, n):
    import torch
    import s3dlio_amd as S
    g = torch.Generator().manual_seed(n)
    host = torch.randint(0, 256, (max(n, 1),), dtype=torch.uint8, generator=g)[:n]
    dev = host.cuda() if n else torch.empty(16, dtype=torch.uint8, device="cuda")
    assert S.crc32_device(gpu_ctx, dev, n) == zlib.crc32(host.numpy().tobytes())


@pytest.mark.gpu
def test_gpu_crc32_large_single_segment(gpu_ctx):
    """> 1 GiB in one segment: the plan widens regions past 256 KiB (at most
    4096 regions) and both CRC kernels agree with zlib."""
    import subprocess
    import sys
    import torch
    import s3dlio_amd as S
    n = 1536 * 2**20 + 5
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu_ctx.xoshiro_fill(dev, n, 2 << 20, seed_base=3)
    torch.cuda.synchronize()
    host = dev.cpu().numpy()
    exp = zlib.crc32(memoryview(host))
    assert S.crc32_device(gpu_ctx, dev, n) == exp
    del dev, host
    # the round-2 kernel (S3DG_CRC_KERNEL=1, read once per process) in a child
    code = ("import sys, zlib, torch; sys.path.insert(0, sys.argv[1]); import s3dlio_amd as S; "
            "c = S.Context(0); n = 1536 * 2**20 + 5; d = torch.empty(n, dtype=torch.uint8, device='cuda'); "
            "c.xoshiro_fill(d, n, 2 << 20, seed_base=3); torch.cuda.synchronize(); "
            f"assert S.crc32_device(c, d, n) == {exp}; print('ok')")
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code, root], env=dict(os.environ, S3DG_CRC_KERNEL="1"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]

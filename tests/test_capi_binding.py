"""The C ABI exactly as the reference-side Rust binding calls it
(integration/rust/src/gpu_data_gen.rs): tests/capi/
binding_abi.c has one block per reference function, with seeded layouts
compared byte for byte against the C oracle linked into the same program.
CPU: the program compiles and links against the library and the oracle.
GPU: it runs and every check passes; its NPZ archive equals the restated
generate_npz_bytes_raw (oracle/npz_oracle.py)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "capi", "binding_abi.c")


def build(tmp_path):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not available")
    from s3dlio_amd._lib import LIB_PATH
    from oracle import oracle_c
    olib = oracle_c.build()
    exe = tmp_path / "binding_abi"
    libdir, odir = os.path.dirname(LIB_PATH), os.path.dirname(olib)
    subprocess.check_call([gcc, "-std=c99", "-O1", "-Wall", "-Wextra", "-Werror", "-I",
                           os.path.join(ROOT, "include"), SRC, "-L", libdir, "-ls3dlio_amd",
                           odir + "/libs3dg_oracle.so", f"-Wl,-rpath,{libdir}", f"-Wl,-rpath,{odir}",
                           "-o", str(exe)])
    return exe


def test_binding_program_builds(tmp_path):
    assert build(tmp_path).exists()


@pytest.mark.gpu
def test_binding_program_runs(tmp_path):
    exe = build(tmp_path)
    out = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and "ALL PASS" in out.stdout, out.stdout[-3000:] + out.stderr[-3000:]
    assert out.stdout.count("PASS ") >= 60
    from oracle import npz_oracle
    got = (tmp_path / "npz_300x211x1_f4_2.npz").read_bytes()
    assert got == npz_oracle.generate_npz_bytes_raw([300, 211, 1], "<f4", 2)

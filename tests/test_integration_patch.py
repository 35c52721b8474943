"""CPU: static checks of the reference-side patches (integration/rust/), which
cannot be compiled here (no cargo / rustc / pyo3 in the image).

* every `extern "C"` function the Rust patch declares exists in
  include/s3dlio_gpu.h with the same parameter count, and is exported by the
  built library;
* the PyO3 patch keeps the reference's Python surface: names, signatures and
  defaults, the ValueError strings and the registration list of
  src/python_api/python_datagen_api.rs (restated below from that file, lines
  cited; the reference itself is not read at test time);
* the Rust patch provides the dgen-data items src/data_gen_alt.rs:14-16
  re-exports, with the GeneratorConfig fields of python_datagen_api.rs:59-68.
"""
import os
import re

import pytest

from conftest import ROOT

RS = os.path.join(ROOT, "integration", "rust", "src", "gpu_data_gen.rs")
PYO3 = os.path.join(ROOT, "integration", "rust", "src", "python_api", "python_datagen_api_gpu.rs")
HDR = os.path.join(ROOT, "include", "s3dlio_gpu.h")

# src/python_api/python_datagen_api.rs (reference): pyo3 signature strings
REF_SIGNATURES = {
    "generate_data": "(size, dedup=1, compress=1)",                                      # :50
    "generate_data_with_threads": "(size, dedup=1, compress=1, threads=None)",           # :96
    "generate_into_buffer": "(buffer, dedup=1, compress=1, threads=None)",               # :151
    "generate_npz_bytes": '(shape, dtype="<f4", num_samples=1)',                         # :396
    "new": "(size, dedup=1, compress=1, threads=None, chunk_size=None, seed=None)",     # :288 Generator
}
REF_REGISTERED = ["generate_data", "generate_data_with_threads", "generate_into_buffer", "generate_npz_bytes",
                  "py_default_data_gen_threads", "py_total_cpus"]                     # :425-432
REF_ERRORS = ["Buffer must be writable",                                                # :165, :334
              "Buffer must be C-contiguous for zero-copy operation",                   # :171
              "Buffer must be C-contiguous"]                                           # :340
REF_CONFIG_FIELDS = ["size", "dedup_factor", "compress_factor", "numa_mode", "max_threads", "numa_node",
                     "block_size", "seed"]                                              # :59-68
DGEN_ITEMS = ["generate_data", "generate_data_simple", "DataBuffer", "DataGenerator", "GeneratorConfig",
              "NumaMode"]                                                               # data_gen_alt.rs:14-16


def read(p):
    with open(p) as f:
        return f.read()


def header_params():
    """name -> parameter count of every function include/s3dlio_gpu.h declares."""
    text = re.sub(r"/\*.*?\*/", "", read(HDR), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(s3dg\w+|s3dlio\w+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def rust_externs():
    text = read(RS)
    block = re.search(r'extern "C" \{(.*?)\n\}', text, flags=re.S).group(1)
    out = {}
    for m in re.finditer(r"fn (\w+)\((.*?)\)", block, flags=re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if not args else args.count(",") + 1
    return out


def test_rust_externs_exist_in_header_with_same_arity():
    hdr = header_params()
    ext = rust_externs()
    assert len(ext) >= 15
    for name, n in ext.items():
        assert name in hdr, f"{name} is not declared in include/s3dlio_gpu.h"
        assert hdr[name] == n, f"{name}: {n} parameters in the Rust patch, {hdr[name]} in the header"


def test_rust_externs_are_exported():
    from s3dlio_amd._lib import lib
    for name in rust_externs():
        assert hasattr(lib, name), name


def test_pyo3_signatures_defaults_and_errors():
    text = read(PYO3)
    sigs = dict(re.findall(r"#\[pyo3\(signature = (\(.*?\))\)\]\s*(?:fn|\n\s*fn)\s+(\w+)", text, flags=re.S))
    found = {v: k for k, v in sigs.items()}
    for fn, sig in REF_SIGNATURES.items():
        assert found.get(fn) == sig, (fn, found.get(fn))
    for msg in REF_ERRORS:
        assert f'"{msg}"' in text, msg
    assert '#[pyclass(name = "Generator")]' in text
    for m in ("fn chunk_size(&self)", "fn fill_chunk(&mut self", "fn is_complete(&self)", "fn reset(&mut self)"):
        assert m in text, m
    assert text.count(".detach(") >= 4                           # every generation without the GIL


def test_pyo3_registration_list():
    text = read(PYO3)
    body = text[text.index("pub fn register_datagen_functions"):]
    assert "m.add_class::<PyGenerator>()" in body
    assert re.findall(r"wrap_pyfunction!\((\w+), m\)", body) == REF_REGISTERED


def test_rust_patch_has_dgen_surface():
    text = read(RS)
    for item in DGEN_ITEMS:
        assert re.search(rf"pub (fn|struct|enum) {item}\b", text), item
    cfg = re.search(r"pub struct GeneratorConfig \{(.*?)\}", text, flags=re.S).group(1)
    assert re.findall(r"pub (\w+):", cfg) == REF_CONFIG_FIELDS
    for m in ("pub fn into_bytes(self) -> bytes::Bytes", "pub fn as_slice(&self) -> &[u8]",
              "pub fn recommended_chunk_size() -> usize", "pub fn generate_data_with_config(config: GeneratorConfig)",
              "pub fn fill_controlled_data(buf: &mut [u8], dedup: usize, compress: usize)",
              "pub fn generate_random_data(size: usize) -> Vec<u8>",
              "pub fn generate_object(cfg: &Config) -> anyhow::Result<bytes::Bytes>"):
        assert m in text, m
    # the reference's own DataGenerator / ObjectGen / ObjectGenAlt stay in the reference
    for gone in ("pub struct ObjectGen ", "pub struct ObjectGenAlt", "fn begin_object",
                 "pub fn generate_controlled_data_streaming"):
        assert gone not in text, gone


def test_pyclass_fields_are_send_and_sync():
    """pyo3 >= 0.23 rejects a #[pyclass] that is not Sync (assert_pyclass_sync)
    unless it is marked `unsendable`; the reference pins pyo3 ^0.27
    (Cargo.toml:99).  A struct of the patch that holds a raw pointer is
    neither Send nor Sync by itself, so each one a pyclass holds needs both
    `unsafe impl`s."""
    rs, py = read(RS), read(PYO3)
    raw = {m.group(1) for m in re.finditer(r"pub struct (\w+) \{([^}]*)\}", rs, flags=re.S)
           if re.search(r"\*(mut|const) ", m.group(2))}
    assert "DataGenerator" in raw
    checked = 0
    for m in re.finditer(r"#\[pyclass\(([^)]*)\)\]\s*(?:pub )?struct (\w+) \{([^}]*)\}", py, flags=re.S):
        if "unsendable" in m.group(1):
            continue
        for ty in re.findall(r"\w+:\s*([A-Za-z_]\w*)", m.group(3)):
            if ty in raw:
                checked += 1
                for tr in ("Send", "Sync"):
                    assert re.search(rf"unsafe impl {tr} for {ty} \{{\}}", rs), \
                        f"#[pyclass] {m.group(2)} holds {ty}, which is not {tr}"
    assert checked >= 1

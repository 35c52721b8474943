// integration/rust/src/gpu_data_gen.rs — the reference-side binding a
// s3dlio maintainer adds as `src/gpu_data_gen.rs` (behind a `gpu` cargo
// feature) to put the MI355X generator (libs3dlio_amd.so, include/s3dlio_gpu.h)
// behind s3dlio's own data-generation API.
//
// A REFERENCE PATCH: cargo/rustc are not in this build's image, so this file is
// not compiled here.  Every extern "C" call below is made, with the same
// arguments, by tests/capi/binding_abi.c (built and run by
// tests/test_capi_binding.py), which is the tested form of this binding.
//
// What it replaces (paths relative to the s3dlio checkout):
//   * the in-tree generators of src/data_gen.rs, same signatures:
//       fill_controlled_data (:151), generate_random_data (:102),
//       generate_object (:29); plus the seeded sibling SURVEY §8b asks for;
//   * the dgen-data 0.2.4 items src/data_gen_alt.rs:14-16 re-exports:
//       generate_data, generate_data_simple, DataBuffer, DataGenerator,
//       GeneratorConfig, NumaMode (the `dgen` section below);
//   * generate_npz_bytes_raw (src/data_formats/npz.rs:322).
// What it leaves alone: data_gen.rs's DataGenerator / ObjectGen /
// generate_controlled_data_streaming (:232-371) and data_gen_alt.rs's
// ObjectGenAlt / generate_controlled_data_alt / generate_data_with_config
// (:56-149).  They only call the re-exported dgen items, so re-pointing the
// re-export moves them onto the GPU unchanged.
//
// Errors: the reference's infallible functions panic with the library's
// message (a GPU or HIP failure is a configuration error the CPU code cannot
// have); generate_object and generate_npz_bytes_raw return anyhow errors as the
// reference does; the try_* forms return them for the PyO3 layer
// (python_api/python_datagen_api_gpu.rs), which raises RuntimeError.

use std::ffi::{c_char, c_int, CStr, CString};

use crate::config::{Config, DataGenMode, ObjectType};

#[repr(C)]
struct S3dgCtx {
    _p: [u8; 0],
}
#[repr(C)]
struct S3dgGen {
    _p: [u8; 0],
}

// include/s3dlio_gpu.h constants
const S3DG_OBJ_NPZ: c_int = 0;
const S3DG_OBJ_TFRECORD: c_int = 1;
const S3DG_OBJ_HDF5: c_int = 2;
const S3DG_OBJ_RAW: c_int = 3;
const S3DG_MODE_STREAMING: c_int = 0;
const S3DG_MODE_SINGLE_PASS: c_int = 1;

#[link(name = "s3dlio_amd")]
extern "C" {
    fn s3dlio_fill_controlled_data(buf: *mut u8, len: usize, dedup: usize, compress: usize) -> c_int;
    fn s3dlio_fill_controlled_data_seeded(buf: *mut u8, len: usize, dedup: usize, compress: usize,
                                          entropy: u64, base4096: *const u8) -> c_int;
    fn s3dlio_generate_random_data(buf: *mut u8, size: usize) -> c_int;
    fn s3dg_object_size(object_type: c_int, elements: u64, element_size: u64, out: *mut u64) -> c_int;
    fn s3dg_generate_object(object_type: c_int, elements: u64, element_size: u64, use_controlled: c_int,
                            dedup: u64, compress: u64, mode: c_int, has_seed: c_int, seed: u64,
                            out: *mut u8, out_len: u64, written: *mut u64) -> c_int;
    fn s3dg_gen_create(size: u64, dedup: u64, compress: u64, has_seed: c_int, seed: u64,
                       out: *mut *mut S3dgGen) -> c_int;
    fn s3dg_gen_destroy(gen: *mut S3dgGen) -> c_int;
    fn s3dg_gen_fill_chunk(gen: *mut S3dgGen, buf: *mut u8, cap: u64, written: *mut u64) -> c_int;
    fn s3dg_gen_is_complete(gen: *mut S3dgGen) -> c_int;
    fn s3dg_gen_position(gen: *mut S3dgGen) -> u64;
    fn s3dg_gen_total_size(gen: *mut S3dgGen) -> u64;
    fn s3dg_gen_reset(gen: *mut S3dgGen) -> c_int;
    fn s3dg_generate_data(buf: *mut u8, size: u64, dedup: u64, compress: u64, has_seed: c_int,
                          seed: u64) -> c_int;
    fn s3dg_host_slot_context(slot: c_int, out: *mut *mut S3dgCtx) -> c_int;
    fn s3dg_npz_size(shape: *const u64, ndim: c_int, dtype: *const c_char, num_samples: u64,
                     total: *mut u64) -> c_int;
    fn s3dg_npz_build(ctx: *mut S3dgCtx, shape: *const u64, ndim: c_int, dtype: *const c_char,
                      num_samples: u64, out: *mut u8, out_len: u64) -> c_int;
    fn s3dg_host_register(buf: *mut u8, len: u64) -> c_int;
    fn s3dg_host_unregister(buf: *mut u8) -> c_int;
    fn s3dg_last_error() -> *const c_char;
}

fn last_error() -> String {
    unsafe { CStr::from_ptr(s3dg_last_error()).to_string_lossy().into_owned() }
}

fn check(rc: c_int) -> anyhow::Result<()> {
    if rc == 0 { Ok(()) } else { anyhow::bail!("s3dlio_amd: {}", last_error()) }
}

fn ok_or_panic(rc: c_int) {
    if let Err(e) = check(rc) {
        panic!("{e}");
    }
}

// ---- src/data_gen.rs (in-tree generators) ---------------------------------------

/// `fill_controlled_data` (src/data_gen.rs:151): same signature and byte
/// layout for a given entropy and base block; time entropy and a per-process
/// random A_BASE_BLOCK as the reference.  Generated on the GPUs (host slots)
/// and copied into `buf`; the Rayon `install()` context has no meaning here.
pub fn fill_controlled_data(buf: &mut [u8], dedup: usize, compress: usize) {
    if buf.is_empty() {
        return; // src/data_gen.rs:154-156
    }
    ok_or_panic(unsafe { s3dlio_fill_controlled_data(buf.as_mut_ptr(), buf.len(), dedup, compress) });
}

/// Seeded sibling: `entropy` replaces call_entropy, `base`
/// replaces A_BASE_BLOCK (None = the library's seeded default block).
pub fn fill_controlled_data_seeded(buf: &mut [u8], dedup: usize, compress: usize, entropy: u64,
                                   base: Option<&[u8; 4096]>) -> anyhow::Result<()> {
    if buf.is_empty() {
        return Ok(());
    }
    let p = base.map_or(std::ptr::null(), |b| b.as_ptr());
    check(unsafe { s3dlio_fill_controlled_data_seeded(buf.as_mut_ptr(), buf.len(), dedup, compress, entropy, p) })
}

/// A reused caller buffer page-locked for direct kernel stores
/// (`s3dg_host_register`; the criterion loop of
/// benches/performance_microbenchmarks.rs:43-64 reuses one buffer): ~33 us
/// per 1 MiB `fill_controlled_data` call against ~57 us through the bounce
/// path.  The guard mutably borrows the slice for as long as the pages are
/// registered, so safe Rust cannot free, move or shrink the buffer while the
/// GPU mapping exists (unmapped while registered, the next call into it would
/// be a GPU memory fault); dropping the guard unregisters it.  Fill through
/// `as_mut_slice()`.
pub struct HostRegistration<'a> {
    buf: &'a mut [u8],
}

impl<'a> HostRegistration<'a> {
    pub fn new(buf: &'a mut [u8]) -> anyhow::Result<Self> {
        if !buf.is_empty() {
            check(unsafe { s3dg_host_register(buf.as_mut_ptr(), buf.len() as u64) })?;
        }
        Ok(HostRegistration { buf })
    }

    pub fn as_mut_slice(&mut self) -> &mut [u8] {
        self.buf
    }
}

impl Drop for HostRegistration<'_> {
    fn drop(&mut self) {
        if !self.buf.is_empty() {
            unsafe { s3dg_host_unregister(self.buf.as_mut_ptr()) };
        }
    }
}

/// `generate_random_data` (src/data_gen.rs:102): BASE_BLOCK tiled, the first
/// min(32, L) and (L > 2048) last 32 bytes of every block random.  ThreadRng
/// cannot be reproduced; the GPU uses time entropy (seeded analogue layout).
pub fn generate_random_data(size: usize) -> Vec<u8> {
    let mut v = vec![0u8; size];
    if size > 0 {
        ok_or_panic(unsafe { s3dlio_generate_random_data(v.as_mut_ptr(), size) });
    }
    v
}

fn object_type_code(t: &ObjectType) -> c_int {
    match t {
        ObjectType::Npz => S3DG_OBJ_NPZ,
        ObjectType::TfRecord => S3DG_OBJ_TFRECORD,
        ObjectType::Hdf5 => S3DG_OBJ_HDF5,
        ObjectType::Raw => S3DG_OBJ_RAW,
    }
}

/// `generate_object` (src/data_gen.rs:29): payload (random layout, or the
/// dgen-contract stream when `use_controlled`) generated straight into its
/// place in the framed object (no `.to_vec()` / `build_raw` copies).  HDF5 is
/// an error, as a reference build without the `hdf5` feature.
pub fn generate_object(cfg: &Config) -> anyhow::Result<bytes::Bytes> {
    let t = object_type_code(&cfg.object_type);
    let mut need = 0u64;
    check(unsafe { s3dg_object_size(t, cfg.elements as u64, cfg.element_size as u64, &mut need) })?;
    let mut out = vec![0u8; need as usize];
    let mut written = 0u64;
    let mode = match cfg.data_gen_mode {
        DataGenMode::Streaming => S3DG_MODE_STREAMING,
        DataGenMode::SinglePass => S3DG_MODE_SINGLE_PASS,
    };
    check(unsafe {
        s3dg_generate_object(t, cfg.elements as u64, cfg.element_size as u64, cfg.use_controlled as c_int,
                             cfg.dedup_factor as u64, cfg.compress_factor as u64, mode, 0, 0,
                             out.as_mut_ptr(), need, &mut written)
    })?;
    out.truncate(written as usize);
    Ok(bytes::Bytes::from(out))
}

// ---- dgen: the dgen-data 0.2.4 surface src/data_gen_alt.rs:14-16 re-exports ----
//
// dgen-data's own bytes are unknown here (the crate is absent: parity unpinned);
// these items generate the build-defined DG1 layout, which
// meets the statistical contract the reference's tests pin (SURVEY Appendix
// B).  Under the `gpu` feature src/data_gen_alt.rs:14-16 becomes
//     pub use crate::gpu_data_gen::{generate_data, generate_data_simple, DataBuffer,
//                                   DataGenerator, GeneratorConfig, NumaMode};
// and src/python_api/python_datagen_api.rs is replaced by
// python_api/python_datagen_api_gpu.rs.

/// `dgen_data::NumaMode`.  Accepted for source compatibility: generation runs
/// on the GPUs' HBM, the host buffer is the caller's.
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub enum NumaMode {
    #[default]
    Auto,
    Force,
    Disabled,
}

/// `dgen_data::GeneratorConfig` (field list as built at
/// src/python_api/python_datagen_api.rs:59-68).  `max_threads`, `numa_mode` and
/// `numa_node` size the CPU pool of the reference and are ignored here;
/// `block_size` must be None or 1 MiB (DG1's dedup unit, src/constants.rs:348).
#[derive(Clone, Debug)]
pub struct GeneratorConfig {
    pub size: usize,
    pub dedup_factor: usize,
    pub compress_factor: usize,
    pub numa_mode: NumaMode,
    pub max_threads: Option<usize>,
    pub numa_node: Option<usize>,
    pub block_size: Option<usize>,
    pub seed: Option<u64>,
}

impl Default for GeneratorConfig {
    fn default() -> Self {
        Self { size: 0, dedup_factor: 1, compress_factor: 1, numa_mode: NumaMode::Auto, max_threads: None,
               numa_node: None, block_size: None, seed: None }
    }
}

const DGEN_BLOCK: usize = 1 << 20;

fn check_block_size(cfg: &GeneratorConfig) -> anyhow::Result<()> {
    match cfg.block_size {
        None | Some(DGEN_BLOCK) => Ok(()),
        Some(b) => anyhow::bail!("s3dlio_amd: block_size {b} unsupported (DG1 uses 1 MiB blocks)"),
    }
}

/// `dgen_data::DataBuffer`: the owned result of `generate_data`.
pub struct DataBuffer {
    data: Vec<u8>,
}

impl DataBuffer {
    pub fn as_slice(&self) -> &[u8] {
        &self.data
    }
    pub fn as_mut_slice(&mut self) -> &mut [u8] {
        &mut self.data
    }
    pub fn as_ptr(&self) -> *const u8 {
        self.data.as_ptr()
    }
    pub fn len(&self) -> usize {
        self.data.len()
    }
    pub fn is_empty(&self) -> bool {
        self.data.is_empty()
    }
    /// Zero-copy hand-off (`Bytes::from(Vec)`), as src/data_gen_alt.rs:57 uses it.
    pub fn into_bytes(self) -> bytes::Bytes {
        bytes::Bytes::from(self.data)
    }
}

/// Fill `buf` in place with a DG1 object of `buf.len()` bytes; `seed` None =
/// time + per-process counter.  The zero-copy write behind the PyO3
/// `generate_into_buffer` (no intermediate DataBuffer, unlike
/// python_datagen_api.rs:179-197).
pub fn try_generate_into(buf: &mut [u8], dedup: usize, compress: usize, seed: Option<u64>) -> anyhow::Result<()> {
    if buf.is_empty() {
        return Ok(());
    }
    check(unsafe {
        s3dg_generate_data(buf.as_mut_ptr(), buf.len() as u64, dedup as u64, compress as u64,
                           seed.is_some() as c_int, seed.unwrap_or(0))
    })
}

/// `dgen_data::generate_data`, fallible form.  Unlike dgen's batch path
/// (src/data_gen_alt.rs:63-64) the seed is honoured, as the reference's tests
/// expect (tests/test_high_speed_data_gen.rs:148-198).
pub fn try_generate_data(config: GeneratorConfig) -> anyhow::Result<DataBuffer> {
    check_block_size(&config)?;
    let mut data = vec![0u8; config.size];
    try_generate_into(&mut data, config.dedup_factor, config.compress_factor, config.seed)?;
    Ok(DataBuffer { data })
}

/// `dgen_data::generate_data(GeneratorConfig) -> DataBuffer`.
pub fn generate_data(config: GeneratorConfig) -> DataBuffer {
    try_generate_data(config).unwrap_or_else(|e| panic!("{e}"))
}

/// `dgen_data::generate_data_simple(size, dedup, compress)`.
pub fn generate_data_simple(size: usize, dedup: usize, compress: usize) -> DataBuffer {
    generate_data(GeneratorConfig { size, dedup_factor: dedup, compress_factor: compress, ..Default::default() })
}

/// `generate_data_with_config` (src/data_gen_alt.rs:56-58), for callers that
/// import it from here; data_gen_alt.rs's own copy works unchanged over the
/// re-exported items.
pub fn generate_data_with_config(config: GeneratorConfig) -> bytes::Bytes {
    generate_data(config).into_bytes()
}

/// `dgen_data::DataGenerator`: one object's positional stream over the
/// library's generator handle (s3dg_gen_*), on one host slot (GPU).  Output
/// does not depend on the chunk sizes passed to `fill_chunk`.
pub struct DataGenerator {
    g: *mut S3dgGen,
}

// The library serialises calls on one handle; a generator may move threads
// (the PyO3 Generator calls it under py.detach).
unsafe impl Send for DataGenerator {}
// Sync: pyo3 ^0.27 (Cargo.toml:99) requires every #[pyclass] to be Sync
// (assert_pyclass_sync), and PyGenerator holds a DataGenerator.  Sound: every
// s3dg_gen_* call that reads or moves the stream position takes the handle's
// own mutex (s3dg_generator.cpp, s3dg_gen::mu), the &self accessors
// (is_complete, position, total_size, seed) read a position the library keeps
// atomic, and the only mutators here take &mut self.
unsafe impl Sync for DataGenerator {}

impl DataGenerator {
    pub fn try_new(config: GeneratorConfig) -> anyhow::Result<Self> {
        check_block_size(&config)?;
        let mut g = std::ptr::null_mut();
        check(unsafe {
            s3dg_gen_create(config.size as u64, config.dedup_factor as u64, config.compress_factor as u64,
                            config.seed.is_some() as c_int, config.seed.unwrap_or(0), &mut g)
        })?;
        Ok(Self { g })
    }
    pub fn new(config: GeneratorConfig) -> Self {
        Self::try_new(config).unwrap_or_else(|e| panic!("{e}"))
    }
    /// Chunk size the PyO3 `Generator` defaults to (python_datagen_api.rs:285).
    pub fn recommended_chunk_size() -> usize {
        32 << 20
    }
    pub fn try_fill_chunk(&mut self, buf: &mut [u8]) -> anyhow::Result<usize> {
        let mut w = 0u64;
        check(unsafe { s3dg_gen_fill_chunk(self.g, buf.as_mut_ptr(), buf.len() as u64, &mut w) })?;
        Ok(w as usize)
    }
    /// Next bytes of the object into `buf`; returns the count (0 when complete).
    pub fn fill_chunk(&mut self, buf: &mut [u8]) -> usize {
        self.try_fill_chunk(buf).unwrap_or_else(|e| panic!("{e}"))
    }
    pub fn is_complete(&self) -> bool {
        unsafe { s3dg_gen_is_complete(self.g) != 0 }
    }
    pub fn reset(&mut self) {
        ok_or_panic(unsafe { s3dg_gen_reset(self.g) });
    }
    pub fn position(&self) -> usize {
        unsafe { s3dg_gen_position(self.g) as usize }
    }
    pub fn total_size(&self) -> usize {
        unsafe { s3dg_gen_total_size(self.g) as usize }
    }
}

impl Drop for DataGenerator {
    fn drop(&mut self) {
        unsafe {
            s3dg_gen_destroy(self.g);
        }
    }
}

// ---- src/data_formats/npz.rs -----------------------------------------------------

/// `generate_npz_bytes_raw` (src/data_formats/npz.rs:322): byte-identical
/// archive; x.npy keystream and its CRC-32 on the GPU, framing on the host.
pub fn generate_npz_bytes_raw(shape: &[usize], dtype_str: &str, num_samples: usize) -> anyhow::Result<Vec<u8>> {
    let dims: Vec<u64> = shape.iter().map(|&d| d as u64).collect();
    let dt = CString::new(dtype_str)?;
    let mut total = 0u64;
    check(unsafe { s3dg_npz_size(dims.as_ptr(), dims.len() as c_int, dt.as_ptr(), num_samples as u64, &mut total) })?;
    let mut ctx = std::ptr::null_mut();
    check(unsafe { s3dg_host_slot_context(-1, &mut ctx) })?;
    let mut out = vec![0u8; total as usize];
    check(unsafe {
        s3dg_npz_build(ctx, dims.as_ptr(), dims.len() as c_int, dt.as_ptr(), num_samples as u64,
                       out.as_mut_ptr(), total)
    })?;
    Ok(out)
}

// integration/rust/src/gpu_data_gen.rs — the reference-side binding a
// s3dlio maintainer adds as `src/gpu_data_gen.rs` (behind a `gpu` cargo
// feature) to put the MI355X generator (libs3dlio_amd.so, include/s3dlio_gpu.h)
// behind s3dlio's own data-generation API.
//
// A REFERENCE PATCH: cargo/rustc are not in this build's image, so this file is
// not compiled here.  Every extern "C" call below is exercised, in the same
// order and with the same arguments, by tests/capi/binding_abi.c (built and run
// by tests/test_capi_binding.py), which is the tested form of this binding.
//
// Public signatures are exactly the reference's (paths relative to the s3dlio
// checkout):
//   fill_controlled_data                 src/data_gen.rs:151
//   generate_random_data                 src/data_gen.rs:102
//   generate_object                      src/data_gen.rs:29
//   generate_controlled_data_streaming   src/data_gen.rs:232
//   DataGenerator / ObjectGen            src/data_gen.rs:253-371
//   generate_controlled_data_alt         src/data_gen_alt.rs:66
//   ObjectGenAlt                         src/data_gen_alt.rs:89-149
//   generate_npz_bytes_raw               src/data_formats/npz.rs:322 (behind the
//                                        PyO3 generate_npz_bytes, python_datagen_api.rs:395)
// The reference functions are infallible except generate_object and
// generate_npz_bytes_raw; here a GPU or HIP failure is a configuration error,
// so the infallible ones panic with the library's message (the reference would
// have no GPU path to fail).

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
    fn s3dg_last_error() -> *const c_char;
}

fn last_error() -> String {
    unsafe { CStr::from_ptr(s3dg_last_error()).to_string_lossy().into_owned() }
}

fn ok_or_panic(rc: c_int) {
    assert!(rc == 0, "s3dlio_amd: {}", last_error());
}

// ---- src/data_gen.rs ---------------------------------------------------------

/// `fill_controlled_data` (src/data_gen.rs:151): same signature, same byte
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
    let rc = unsafe { s3dlio_fill_controlled_data_seeded(buf.as_mut_ptr(), buf.len(), dedup, compress, entropy, p) };
    if rc == 0 { Ok(()) } else { anyhow::bail!("s3dlio_amd: {}", last_error()) }
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
/// dgen-contract stream when `use_controlled`) framed as the object type.
/// HDF5 is an error, as a reference build without the `hdf5` feature.
pub fn generate_object(cfg: &Config) -> anyhow::Result<bytes::Bytes> {
    let t = object_type_code(&cfg.object_type);
    let mut need = 0u64;
    if unsafe { s3dg_object_size(t, cfg.elements as u64, cfg.element_size as u64, &mut need) } != 0 {
        anyhow::bail!("{}", last_error());
    }
    let mut out = vec![0u8; need as usize];
    let mut written = 0u64;
    let mode = match cfg.data_gen_mode {
        DataGenMode::Streaming => S3DG_MODE_STREAMING,
        DataGenMode::SinglePass => S3DG_MODE_SINGLE_PASS,
    };
    let rc = unsafe {
        s3dg_generate_object(t, cfg.elements as u64, cfg.element_size as u64, cfg.use_controlled as c_int,
                             cfg.dedup_factor as u64, cfg.compress_factor as u64, mode, 0, 0,
                             out.as_mut_ptr(), need, &mut written)
    };
    if rc != 0 {
        anyhow::bail!("{}", last_error());
    }
    out.truncate(written as usize);
    Ok(bytes::Bytes::from(out))
}

/// `generate_controlled_data_streaming` (src/data_gen.rs:232).  Generation
/// is positional, so the chunk size changes nothing but the copy granularity.
pub fn generate_controlled_data_streaming(size: usize, dedup: usize, compress: usize,
                                          chunk_size: usize) -> Vec<u8> {
    let gen = DataGenerator::new(None);
    let mut object_gen = gen.begin_object(size, dedup, compress);
    let mut result = Vec::with_capacity(size);
    while !object_gen.is_complete() {
        match object_gen.fill_chunk(chunk_size) {
            Some(chunk) => result.extend_from_slice(&chunk),
            None => break,
        }
    }
    result
}

/// `DataGenerator` (src/data_gen.rs:253-305): an instance entropy, explicit or
/// time + thread-local counter (:271-291); every object begun from it is seeded
/// with that entropy, so repeated `begin_object` calls give identical objects.
pub struct DataGenerator {
    instance_entropy: u64,
}

impl DataGenerator {
    pub fn new(seed: Option<u64>) -> Self {
        let instance_entropy = match seed {
            Some(s) => s,
            None => {
                use std::cell::Cell;
                use std::time::{SystemTime, UNIX_EPOCH};
                thread_local! {
                    static ENTROPY_COUNTER: Cell<u64> = const { Cell::new(0) };
                }
                let base = SystemTime::now().duration_since(UNIX_EPOCH).unwrap_or_default().as_nanos() as u64;
                let counter = ENTROPY_COUNTER.with(|c| {
                    let v = c.get();
                    c.set(v.wrapping_add(1));
                    v
                });
                base.wrapping_add(counter)
            }
        };
        Self { instance_entropy }
    }

    pub fn new_with_seed(seed: u64) -> Self {
        Self::new(Some(seed))
    }

    pub fn begin_object(&self, size: usize, dedup: usize, compress: usize) -> ObjectGen {
        ObjectGen { alt_gen: ObjectGenAlt::new_with_seed(size, dedup, compress, self.instance_entropy) }
    }
}

impl Default for DataGenerator {
    fn default() -> Self {
        Self::new(None)
    }
}

/// `ObjectGen` (src/data_gen.rs:308-371).
pub struct ObjectGen {
    alt_gen: ObjectGenAlt,
}

impl ObjectGen {
    pub fn fill_chunk(&mut self, chunk_size: usize) -> Option<Vec<u8>> {
        assert!(chunk_size > 0, "Chunk size must be greater than 0"); // :328
        let mut buf = vec![0u8; chunk_size];
        let written = self.alt_gen.fill_chunk(&mut buf);
        if written == 0 {
            return None;
        }
        buf.truncate(written);
        Some(buf)
    }
    pub fn is_complete(&self) -> bool {
        self.alt_gen.is_complete()
    }
    pub fn reset(&mut self) {
        self.alt_gen.reset()
    }
    pub fn position(&self) -> usize {
        self.alt_gen.position()
    }
    pub fn total_size(&self) -> usize {
        self.alt_gen.total_size()
    }
    pub fn fill_remaining(&mut self) -> Vec<u8> {
        const CHUNK: usize = 32 * 1024 * 1024; // :360
        let mut result = Vec::with_capacity(self.total_size().saturating_sub(self.position()));
        while !self.is_complete() {
            match self.fill_chunk(CHUNK) {
                Some(c) => result.extend_from_slice(&c),
                None => break,
            }
        }
        result
    }
}

// ---- src/data_gen_alt.rs -----------------------------------------------------

/// `generate_controlled_data_alt` (src/data_gen_alt.rs:66): `.max(1)` on dedup
/// and compress; seeded output is reproducible.
pub fn generate_controlled_data_alt(size: usize, dedup: usize, compress: usize,
                                    seed: Option<u64>) -> bytes::Bytes {
    let mut v = vec![0u8; size];
    if size > 0 {
        ok_or_panic(unsafe {
            s3dg_generate_data(v.as_mut_ptr(), size as u64, dedup.max(1) as u64, compress.max(1) as u64,
                               seed.is_some() as c_int, seed.unwrap_or(0))
        });
    }
    bytes::Bytes::from(v)
}

/// `ObjectGenAlt` (src/data_gen_alt.rs:89-149) over the library's streaming
/// generator (s3dg_gen_*): one host slot (GPU) per generator.
pub struct ObjectGenAlt {
    g: *mut S3dgGen,
}

// the library serialises calls on one generator; a generator may move threads
unsafe impl Send for ObjectGenAlt {}

impl ObjectGenAlt {
    pub fn new(total_size: usize, dedup: usize, compress: usize) -> Self {
        Self::create(total_size, dedup, compress, None)
    }
    pub fn new_with_seed(total_size: usize, dedup: usize, compress: usize, seed: u64) -> Self {
        Self::create(total_size, dedup, compress, Some(seed))
    }
    fn create(total_size: usize, dedup: usize, compress: usize, seed: Option<u64>) -> Self {
        let mut g = std::ptr::null_mut();
        ok_or_panic(unsafe {
            s3dg_gen_create(total_size as u64, dedup.max(1) as u64, compress.max(1) as u64,
                            seed.is_some() as c_int, seed.unwrap_or(0), &mut g)
        });
        Self { g }
    }
    pub fn fill_chunk(&mut self, buf: &mut [u8]) -> usize {
        let mut w = 0u64;
        ok_or_panic(unsafe { s3dg_gen_fill_chunk(self.g, buf.as_mut_ptr(), buf.len() as u64, &mut w) });
        w as usize
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

impl Drop for ObjectGenAlt {
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
    if unsafe { s3dg_npz_size(dims.as_ptr(), dims.len() as c_int, dt.as_ptr(), num_samples as u64, &mut total) } != 0 {
        anyhow::bail!("{}", last_error());
    }
    let mut ctx = std::ptr::null_mut();
    if unsafe { s3dg_host_slot_context(-1, &mut ctx) } != 0 {
        anyhow::bail!("{}", last_error());
    }
    let mut out = vec![0u8; total as usize];
    let rc = unsafe {
        s3dg_npz_build(ctx, dims.as_ptr(), dims.len() as c_int, dt.as_ptr(), num_samples as u64,
                       out.as_mut_ptr(), total)
    };
    if rc != 0 {
        anyhow::bail!("{}", last_error());
    }
    Ok(out)
}

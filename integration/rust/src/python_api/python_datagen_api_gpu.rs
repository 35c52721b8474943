// integration/rust/src/python_api/python_datagen_api_gpu.rs — the PyO3 layer
// of the MI355X generator: under the `gpu` cargo feature it stands in for
// src/python_api/python_datagen_api.rs (same module, same `_pymod` names).
//
// A REFERENCE PATCH: cargo/rustc/pyo3 are not in this build's image, so this
// file is not compiled here.  The C calls it reaches (through
// crate::gpu_data_gen) are made with the same arguments by
// tests/capi/binding_abi.c ("PyO3 ..." checks); the Python-visible behaviour
// (names, defaults, return types, ValueError messages, BytesView) is that of
// the Python mirror s3dlio_amd/datagen.py, tested by tests/test_gpu_datagen.py
// and tests/test_bytesview.py.
//
// Kept from the reference (python_datagen_api.rs line numbers): every
// #[pyfunction] / #[pyclass] signature and default (:49-51, :95-97, :150-152,
// :218, :235, :270-288, :395-397), the two ValueError strings of
// generate_into_buffer (:163-173) and the slightly different one of
// Generator.fill_chunk (:338-342), py.detach around every generation, the
// BytesView return type (python_core_api.rs:306) and the registration list
// (:420-435).
// Changed: the bytes come from the GPU (DG1 layout); a GPU or
// HIP failure raises RuntimeError where dgen-data could not fail;
// generate_into_buffer writes straight into the caller's buffer (the
// reference generates a DataBuffer and copies it, :179-197); `threads` is
// accepted and ignored (no CPU pool).

use pyo3::buffer::PyBuffer;
use pyo3::exceptions::{PyRuntimeError, PyValueError};
use pyo3::prelude::*;

use super::python_core_api::PyBytesView;
use crate::gpu_data_gen::{self as gpu, DataGenerator, GeneratorConfig, NumaMode};
use crate::hardware::{recommended_data_gen_threads, total_cpus};

fn runtime(e: anyhow::Error) -> PyErr {
    PyRuntimeError::new_err(format!("{e:#}"))
}

fn config(size: usize, dedup: usize, compress: usize, threads: Option<usize>, seed: Option<u64>) -> GeneratorConfig {
    GeneratorConfig {
        size,
        dedup_factor: dedup,
        compress_factor: compress,
        numa_mode: NumaMode::Auto,
        max_threads: threads,
        numa_node: None,
        block_size: None,
        seed,
    }
}

/// A new DG1 object of `size` bytes as a read-only zero-copy BytesView.
fn new_view(py: Python<'_>, cfg: GeneratorConfig) -> PyResult<Py<PyBytesView>> {
    let buf = py.detach(|| gpu::try_generate_data(cfg)).map_err(runtime)?;
    Py::new(py, PyBytesView::new(buf.into_bytes()))
}

/// Writable, C-contiguous byte view of a Python buffer, or the reference's
/// ValueError (`contig_msg` differs between the two call sites).
fn writable(py: Python<'_>, obj: &Py<PyAny>, contig_msg: &'static str) -> PyResult<PyBuffer<u8>> {
    let b: PyBuffer<u8> = PyBuffer::get(obj.bind(py))?;
    if b.readonly() {
        return Err(PyValueError::new_err("Buffer must be writable"));
    }
    if !b.is_c_contiguous() {
        return Err(PyValueError::new_err(contig_msg));
    }
    Ok(b)
}

/// generate_data(size, dedup=1, compress=1) -> BytesView.
#[pyfunction]
#[pyo3(signature = (size, dedup=1, compress=1))]
fn generate_data(py: Python<'_>, size: usize, dedup: usize, compress: usize) -> PyResult<Py<PyBytesView>> {
    new_view(py, config(size, dedup, compress, Some(recommended_data_gen_threads(None, None)), None))
}

/// generate_data_with_threads(size, dedup=1, compress=1, threads=None) -> BytesView.
#[pyfunction]
#[pyo3(signature = (size, dedup=1, compress=1, threads=None))]
fn generate_data_with_threads(py: Python<'_>, size: usize, dedup: usize, compress: usize,
                              threads: Option<usize>) -> PyResult<Py<PyBytesView>> {
    let t = threads.unwrap_or_else(|| recommended_data_gen_threads(None, None));
    new_view(py, config(size, dedup, compress, Some(t), None))
}

/// generate_into_buffer(buffer, dedup=1, compress=1, threads=None) -> int:
/// fills the whole buffer in place (one D2H into it, no staging copy).
#[pyfunction]
#[pyo3(signature = (buffer, dedup=1, compress=1, threads=None))]
fn generate_into_buffer(py: Python<'_>, buffer: Py<PyAny>, dedup: usize, compress: usize,
                        threads: Option<usize>) -> PyResult<usize> {
    let _ = threads;
    let b = writable(py, &buffer, "Buffer must be C-contiguous for zero-copy operation")?;
    let n = b.len_bytes();
    let addr = b.buf_ptr() as usize;
    py.detach(|| {
        // SAFETY: `b` holds the buffer export (and so the memory) until it drops
        // after this closure; the GIL-free write is the reference's own pattern
        // (python_datagen_api.rs:347-351).
        let dst = unsafe { std::slice::from_raw_parts_mut(addr as *mut u8, n) };
        gpu::try_generate_into(dst, dedup, compress, None)
    })
    .map_err(runtime)?;
    drop(b);
    Ok(n)
}

/// py_default_data_gen_threads() (exported as in the reference).
#[pyfunction]
fn py_default_data_gen_threads() -> usize {
    recommended_data_gen_threads(None, None)
}

/// py_total_cpus() (exported as in the reference).
#[pyfunction]
fn py_total_cpus() -> usize {
    total_cpus()
}

/// Generator(size, dedup=1, compress=1, threads=None, chunk_size=None, seed=None):
/// a positional DG1 stream over one object, filled chunk by chunk in place.
#[pyclass(name = "Generator")]
struct PyGenerator {
    inner: DataGenerator,
    chunk_size: usize,
}

#[pymethods]
impl PyGenerator {
    #[new]
    #[pyo3(signature = (size, dedup=1, compress=1, threads=None, chunk_size=None, seed=None))]
    fn new(size: usize, dedup: usize, compress: usize, threads: Option<usize>, chunk_size: Option<usize>,
           seed: Option<u64>) -> PyResult<Self> {
        let inner = DataGenerator::try_new(config(size, dedup, compress, threads, seed)).map_err(runtime)?;
        Ok(Self { inner, chunk_size: chunk_size.unwrap_or_else(DataGenerator::recommended_chunk_size) })
    }

    #[getter]
    fn chunk_size(&self) -> usize {
        self.chunk_size
    }

    /// Writes the object's next bytes into `buffer`; returns the count (0 when complete).
    fn fill_chunk(&mut self, py: Python<'_>, buffer: Py<PyAny>) -> PyResult<usize> {
        let b = writable(py, &buffer, "Buffer must be C-contiguous")?;
        let n = b.len_bytes();
        let addr = b.buf_ptr() as usize;
        let inner = &mut self.inner;
        let w = py
            .detach(|| {
                // SAFETY: as in generate_into_buffer.
                let dst = unsafe { std::slice::from_raw_parts_mut(addr as *mut u8, n) };
                inner.try_fill_chunk(dst)
            })
            .map_err(runtime)?;
        drop(b);
        Ok(w)
    }

    fn is_complete(&self) -> bool {
        self.inner.is_complete()
    }

    fn reset(&mut self) {
        self.inner.reset();
    }
}

/// generate_npz_bytes(shape, dtype="<f4", num_samples=1) -> BytesView: the
/// byte-identical archive of generate_npz_bytes_raw (npz.rs:322), x.npy and its
/// CRC-32 on the GPU.
#[pyfunction]
#[pyo3(signature = (shape, dtype="<f4", num_samples=1))]
fn generate_npz_bytes(py: Python<'_>, shape: Vec<usize>, dtype: &str, num_samples: usize)
                      -> PyResult<Py<PyBytesView>> {
    let dt = dtype.to_owned();
    let v = py.detach(|| gpu::generate_npz_bytes_raw(&shape, &dt, num_samples)).map_err(runtime)?;
    Py::new(py, PyBytesView::new(bytes::Bytes::from(v)))
}

/// Same registration as python_datagen_api.rs:420-435, so lib.rs:263-272 is unchanged.
pub fn register_datagen_functions(m: &Bound<'_, PyModule>) -> PyResult<()> {
    m.add_class::<PyGenerator>()?;
    for f in [
        wrap_pyfunction!(generate_data, m)?,
        wrap_pyfunction!(generate_data_with_threads, m)?,
        wrap_pyfunction!(generate_into_buffer, m)?,
        wrap_pyfunction!(generate_npz_bytes, m)?,
        wrap_pyfunction!(py_default_data_gen_threads, m)?,
        wrap_pyfunction!(py_total_cpus, m)?,
    ] {
        m.add_function(f)?;
    }
    Ok(())
}

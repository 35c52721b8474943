/* bytesview.c — the reference's Python `BytesView` (src/python_api/
 * python_core_api.rs:300-462) as a CPython extension type.
 *
 * A read-only, zero-copy byte buffer over host memory the library filled
 * (s3dlio_amd/hostbuf.py).  Semantics kept from the reference:
 *   * buffer protocol: memoryview(bv) / np.frombuffer(bv) share the memory;
 *     a writable request raises BufferError (:354-358);
 *   * len(bv) (:322), bytes(bv) and bv.to_bytes() copy (:327, :442),
 *     bv.memoryview() is zero-copy and keeps bv alive (:429-439),
 *     repr "BytesView(<n> bytes)" (:447-449).
 * The owner object (a numpy array of a pooled mapping) is held through a
 * buffer export for the BytesView's lifetime. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

typedef struct {
    PyObject_HEAD
    Py_buffer src;          /* read-only export of the owner */
    Py_ssize_t shape0;      /* stable shape[0] for consumers' Py_buffer */
    int has_src;
} BytesView;

static int bv_init(BytesView *self, PyObject *args, PyObject *kw) {
    PyObject *owner;
    static char *kwlist[] = {"owner", NULL};
    if (!PyArg_ParseTupleAndKeywords(args, kw, "O", kwlist, &owner)) return -1;
    if (self->has_src) {
        PyBuffer_Release(&self->src);
        self->has_src = 0;
    }
    if (PyObject_GetBuffer(owner, &self->src, PyBUF_SIMPLE) < 0) return -1;
    self->has_src = 1;
    self->shape0 = self->src.len;
    return 0;
}

static void bv_dealloc(BytesView *self) {
    if (self->has_src) PyBuffer_Release(&self->src);
    Py_TYPE(self)->tp_free((PyObject *)self);
}

static int bv_getbuffer(BytesView *self, Py_buffer *view, int flags) {
    static Py_ssize_t unit_stride = 1;
    if (flags & PyBUF_WRITABLE) {
        PyErr_SetString(PyExc_BufferError, "BytesView is read-only and does not support writable buffers");
        view->obj = NULL;
        return -1;
    }
    if (!self->has_src) {
        PyErr_SetString(PyExc_BufferError, "BytesView is not initialised");
        view->obj = NULL;
        return -1;
    }
    view->buf = self->src.buf;
    view->len = self->src.len;
    view->readonly = 1;
    view->itemsize = 1;
    view->ndim = 1;
    view->format = (flags & PyBUF_FORMAT) ? "B" : NULL;
    view->shape = (flags & PyBUF_ND) ? &self->shape0 : NULL;
    view->strides = (flags & PyBUF_STRIDES) ? &unit_stride : NULL;
    view->suboffsets = NULL;
    view->internal = NULL;
    view->obj = (PyObject *)self;
    Py_INCREF(self);
    return 0;
}

static Py_ssize_t bv_len(BytesView *self) { return self->has_src ? self->src.len : 0; }

static PyObject *bv_to_bytes(BytesView *self, PyObject *unused) {
    (void)unused;
    return PyBytes_FromStringAndSize(self->has_src ? (const char *)self->src.buf : "", bv_len(self));
}

static PyObject *bv_memoryview(BytesView *self, PyObject *unused) {
    (void)unused;
    return PyMemoryView_FromObject((PyObject *)self);
}

static PyObject *bv_repr(BytesView *self) {
    return PyUnicode_FromFormat("BytesView(%zd bytes)", bv_len(self));
}

static PyMethodDef bv_methods[] = {
    {"memoryview", (PyCFunction)bv_memoryview, METH_NOARGS, "Zero-copy read-only memoryview."},
    {"to_bytes", (PyCFunction)bv_to_bytes, METH_NOARGS, "Copy into a new bytes object."},
    {"__bytes__", (PyCFunction)bv_to_bytes, METH_NOARGS, "Copy into a new bytes object."},
    {NULL, NULL, 0, NULL},
};

static PyBufferProcs bv_as_buffer = {(getbufferproc)bv_getbuffer, NULL};
static PySequenceMethods bv_as_sequence = {(lenfunc)bv_len};

static PyTypeObject BytesViewType = {
    PyVarObject_HEAD_INIT(NULL, 0)
    .tp_name = "s3dlio_amd.BytesView",
    .tp_basicsize = sizeof(BytesView),
    .tp_dealloc = (destructor)bv_dealloc,
    .tp_repr = (reprfunc)bv_repr,
    .tp_as_sequence = &bv_as_sequence,
    .tp_as_buffer = &bv_as_buffer,
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "Read-only zero-copy byte buffer (s3dlio BytesView).",
    .tp_methods = bv_methods,
    .tp_init = (initproc)bv_init,
    .tp_new = PyType_GenericNew,
};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_bytesview", NULL, -1, NULL};

PyMODINIT_FUNC PyInit__bytesview(void) {
    if (PyType_Ready(&BytesViewType) < 0) return NULL;
    PyObject *m = PyModule_Create(&moddef);
    if (!m) return NULL;
    Py_INCREF(&BytesViewType);
    if (PyModule_AddObject(m, "BytesView", (PyObject *)&BytesViewType) < 0) {
        Py_DECREF(&BytesViewType);
        Py_DECREF(m);
        return NULL;
    }
    return m;
}

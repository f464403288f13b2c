/* gq_pycall.c -- a CPython fast-call entry to gq_mmq_ex, the eager drop-in's launch hop.
 *
 * The reference's callers invoke kernels.mmq_q4_k.mmq_q4_k(A, B, M, N, K) eagerly, one call per
 * MMQ (/root/reference/test/test_mmq_q4_k.py:34); at decode sizes the kernel runs in ~10 us, so
 * the host cost of getting from Python into the C ABI matters.  ctypes spends ~1.5-2 us
 * converting thirteen arguments; this module takes them as METH_FASTCALL integers and calls
 * the same gq_mmq_ex (include/gguf_mmq.h) through a pointer that kernels/_lib.py hands over
 * from the ctypes-loaded libgguf_mmq.so -- so exactly one copy of the HIP library is in play
 * and nothing here links against it or against torch.
 *
 *   bind(address)                  the address of gq_mmq_ex in the loaded library
 *   mmq_ex(type, act, A, B, C, M, N, K, ldb, ldc, ws|None, ws_bytes, stream) -> int status
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

typedef int (*gq_mmq_ex_fn)(int, int, const void *, const void *, void *, int64_t, int64_t, int64_t, int64_t,
                            int64_t, void *, size_t, void *);

static gq_mmq_ex_fn g_mmq_ex;

static PyObject *gq_bind(PyObject *self, PyObject *arg) {
    void *p = PyLong_AsVoidPtr(arg);
    if (p == NULL) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "bind: null gq_mmq_ex address");
        return NULL;
    }
    g_mmq_ex = (gq_mmq_ex_fn)p;
    Py_RETURN_NONE;
}

/* an integer argument (None reads as 0, for the optional workspace pointer) */
static int as_i64(PyObject *o, int64_t *v) {
    if (o == Py_None) { *v = 0; return 0; }
    long long x = PyLong_AsLongLong(o);
    if (x == -1 && PyErr_Occurred()) return -1;
    *v = (int64_t)x;
    return 0;
}

static PyObject *gq_mmq_ex(PyObject *self, PyObject *const *args, Py_ssize_t nargs) {
    if (nargs != 13) {
        PyErr_Format(PyExc_TypeError, "mmq_ex takes 13 arguments (%zd given)", nargs);
        return NULL;
    }
    if (g_mmq_ex == NULL) {
        PyErr_SetString(PyExc_RuntimeError, "mmq_ex: bind() the library first");
        return NULL;
    }
    int64_t v[13];
    for (int i = 0; i < 13; ++i)
        if (as_i64(args[i], &v[i])) return NULL;
    int rc = g_mmq_ex((int)v[0], (int)v[1], (const void *)(intptr_t)v[2], (const void *)(intptr_t)v[3],
                      (void *)(intptr_t)v[4], v[5], v[6], v[7], v[8], v[9], (void *)(intptr_t)v[10],
                      (size_t)v[11], (void *)(intptr_t)v[12]);
    return PyLong_FromLong(rc);
}

static PyMethodDef methods[] = {
    {"bind", (PyCFunction)gq_bind, METH_O, "bind(address of gq_mmq_ex)"},
    {"mmq_ex", (PyCFunction)(void (*)(void))gq_mmq_ex, METH_FASTCALL,
     "mmq_ex(type, act, A, B, C, M, N, K, ldb, ldc, ws, ws_bytes, stream) -> status"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_gqcall", NULL, -1, methods};

PyMODINIT_FUNC PyInit__gqcall(void) { return PyModule_Create(&module); }

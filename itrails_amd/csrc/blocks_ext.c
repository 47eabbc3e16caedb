/* _blocks: the pointer / length scan of a V_lst (read_data.py:94-117: a list of int64 NumPy
 * arrays, one per MAF block) for the host-block entry points of libitrails_hip.so
 * (itr_forward_loglik_blocks, itr_viterbi_blocks).  One pass over the list through NumPy's C
 * API fills caller-provided int64 lengths and uintp data pointers; a Python loop over
 * 5,036 blocks spent 3.6 ms on attribute lookups per wrapper call.  No computation here. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>
#include <stdint.h>

/* scan(V_lst, lens_out, ptrs_out) -> True when every entry is a 1-D C-contiguous native int64
 * array (lens_out[k], ptrs_out[k] filled), False at the first one that is not */
static PyObject* scan(PyObject* self, PyObject* args) {
  PyObject* lst;
  PyArrayObject *lens_out, *ptrs_out;
  (void)self;
  if (!PyArg_ParseTuple(args, "OO!O!", &lst, &PyArray_Type, &lens_out, &PyArray_Type, &ptrs_out))
    return NULL;
  PyObject* seq = PySequence_Fast(lst, "V_lst must be a sequence");
  if (!seq) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  if (PyArray_SIZE(lens_out) < n || PyArray_SIZE(ptrs_out) < n || PyArray_ITEMSIZE(lens_out) != 8 ||
      PyArray_ITEMSIZE(ptrs_out) != 8 || !PyArray_IS_C_CONTIGUOUS(lens_out) ||
      !PyArray_IS_C_CONTIGUOUS(ptrs_out)) {
    Py_DECREF(seq);
    PyErr_SetString(PyExc_ValueError, "output arrays too small or not 8-byte contiguous");
    return NULL;
  }
  PyObject** items = PySequence_Fast_ITEMS(seq);
  int64_t* L = (int64_t*)PyArray_DATA(lens_out);
  uint64_t* P = (uint64_t*)PyArray_DATA(ptrs_out);
  int ok = 1;
  for (Py_ssize_t k = 0; k < n; ++k) {
    PyObject* o = items[k];
    if (!PyArray_Check(o)) { ok = 0; break; }
    PyArrayObject* a = (PyArrayObject*)o;
    PyArray_Descr* d = PyArray_DESCR(a);
    if (PyArray_NDIM(a) != 1 || d->kind != 'i' || PyArray_ITEMSIZE(a) != 8 ||
        !PyArray_ISNOTSWAPPED(a) || !PyArray_IS_C_CONTIGUOUS(a)) { ok = 0; break; }
    L[k] = (int64_t)PyArray_DIM(a, 0);
    P[k] = (uint64_t)(uintptr_t)PyArray_DATA(a);
  }
  Py_DECREF(seq);
  return PyBool_FromLong(ok);
}

static PyMethodDef methods[] = {{"scan", scan, METH_VARARGS, "V_lst lengths and data pointers"},
                                {NULL, NULL, 0, NULL}};
static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_blocks", NULL, -1, methods};

PyMODINIT_FUNC PyInit__blocks(void) {
  import_array();
  return PyModule_Create(&mod);
}

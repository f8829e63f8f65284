// Host side of the drop-in's general path: the (L, K) peer-pointer table of
// aggregate_models (reference aggregator/aggregation.py:25-28 reads
// received_models[j]["model"][key] for every key of self.model.state_dict()
// and every update j).  With plain dicts of tensors -- what the reference's
// listener appends after pickle.loads (node/node.py:135-141) -- the Python
// loop cost ~0.5 us per tensor in dict lookups and dtype / device / layout
// getters: 1.9 ms per call for ResNet-18 x 64 updates, 3.7x the kernel.  This
// walks the same lists in C (CPython dict lookups, ATen getters) and writes
// the table straight into the caller's buffer.
//
// gather_peer_table(received, keys, numels, device, out) -> int
//   received : list of update records; record["model"][key] is the tensor
//              (the reference's lookups, KeyError on a missing one)
//   keys     : list of L state_dict keys; numels: L element counts
//   device   : CUDA device index of the model
//   out      : writable buffer of L*K uint64, row-major [l][j]
// Returns 0 with out filled when every tensor is fp32, contiguous, on
// `device` with numels[l] elements; 1 (out partially written, nothing
// raised) when some tensor needs the Python path's exact diagnosis or
// widening (a sparse or other non-strided tensor included: its layout is
// checked before any strided-only getter); raises what the reference's
// lookups raise (KeyError, TypeError), and RuntimeError if an ATen getter
// throws -- no C++ exception unwinds through this CPython function.
#include <Python.h>

#include <ATen/core/Tensor.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>
#include <exception>
#include <vector>

namespace {

PyObject* g_model_key = nullptr;  // interned "model"

// record[key] with the reference's semantics: exact dicts through the dict
// API, any other mapping through __getitem__; a new reference or nullptr.
PyObject* get_item(PyObject* mapping, PyObject* key) {
  if (PyDict_CheckExact(mapping)) {
    PyObject* v = PyDict_GetItemWithError(mapping, key);
    if (v) {
      Py_INCREF(v);
      return v;
    }
    if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, key);
    return nullptr;
  }
  return PyObject_GetItem(mapping, key);
}

// Py_buffer released on every exit path (the C++ exception path included).
struct BufferGuard {
  Py_buffer* b;
  ~BufferGuard() { PyBuffer_Release(b); }
};

// status 0: x is a dense fp32 tensor on `device` with n elements.  The layout
// is checked before any getter that only strided tensors implement
// (is_contiguous throws c10::Error on a sparse tensor).
int vouch(const at::Tensor& x, int device, int64_t n) {
  if (x.layout() != at::kStrided || x.scalar_type() != at::kFloat || !x.is_cuda() || x.get_device() != device)
    return 1;
  return (x.numel() == n && x.is_contiguous()) ? 0 : 1;
}

PyObject* gather_peer_table_impl(PyObject* received, PyObject* keys, PyObject* numels_obj, int device,
                                 Py_buffer* out) {
  const Py_ssize_t K = PyList_GET_SIZE(received), L = PyList_GET_SIZE(keys);
  if (out->len < static_cast<Py_ssize_t>(sizeof(uint64_t)) * L * K || PyList_GET_SIZE(numels_obj) != L) {
    PyErr_SetString(PyExc_ValueError, "gather_peer_table: buffer / numels do not match L x K");
    return nullptr;
  }
  int status = 0;
  std::vector<int64_t> numels(static_cast<size_t>(L));
  for (Py_ssize_t l = 0; l < L; ++l) {
    numels[l] = PyLong_AsLongLong(PyList_GET_ITEM(numels_obj, l));
    if (numels[l] == -1 && PyErr_Occurred()) return nullptr;
  }
  uint64_t* table = static_cast<uint64_t*>(out->buf);
  for (Py_ssize_t j = 0; j < K && status == 0; ++j) {
    PyObject* model = get_item(PyList_GET_ITEM(received, j), g_model_key);
    if (!model) return nullptr;
    for (Py_ssize_t l = 0; l < L; ++l) {
      PyObject* t = get_item(model, PyList_GET_ITEM(keys, l));
      if (!t) {
        Py_DECREF(model);
        return nullptr;
      }
      if (!THPVariable_Check(t)) {
        Py_DECREF(t);
        status = 1;  // not a tensor: the Python path reports it the reference's way
        break;
      }
      int bad;
      try {
        const at::Tensor& x = THPVariable_Unpack(t);
        bad = vouch(x, device, numels[l]);
        if (!bad) table[l * K + j] = reinterpret_cast<uint64_t>(x.data_ptr());
      } catch (const std::exception& e) {  // an ATen getter threw: a Python error, never std::terminate
        Py_DECREF(t);
        Py_DECREF(model);
        PyErr_Format(PyExc_RuntimeError, "gather_peer_table: %s", e.what());
        return nullptr;
      }
      Py_DECREF(t);
      if (bad) {
        status = 1;
        break;
      }
    }
    Py_DECREF(model);
  }
  return PyLong_FromLong(status);
}

PyObject* gather_peer_table(PyObject*, PyObject* args) {
  PyObject *received, *keys, *numels_obj;
  int device;
  Py_buffer out;
  if (!PyArg_ParseTuple(args, "O!O!O!iw*", &PyList_Type, &received, &PyList_Type, &keys, &PyList_Type,
                        &numels_obj, &device, &out))
    return nullptr;
  BufferGuard guard{&out};
  return gather_peer_table_impl(received, keys, numels_obj, device, &out);
}

// fill_chunk_list(nch, out) -> C
//   nch : buffer of L int64, key l's 1024-element chunks (0: not chunked)
//   out : writable buffer of 2*M int64, M a multiple of 8 >= the chunk total
// Writes the split kernel's chunk list (include/p2pdl.h
// p2p_fedavg_split_chunks_f32: (seg, c0) pairs, key order, the rest (-1, 0))
// and returns the chunk total C; -1 when it exceeds M.  numpy's repeat /
// arange / strided stores took ~90 us for ResNet-18's 11,448 chunks.
PyObject* fill_chunk_list(PyObject*, PyObject* args) {
  Py_buffer nch, out;
  if (!PyArg_ParseTuple(args, "y*w*", &nch, &out)) return nullptr;
  BufferGuard g1{&nch}, g2{&out};
  const int64_t* n = static_cast<const int64_t*>(nch.buf);
  const int64_t L = nch.len / 8, M = out.len / 16;
  int64_t* o = static_cast<int64_t*>(out.buf);
  int64_t c = 0;
  for (int64_t l = 0; l < L; ++l) {
    if (n[l] < 0 || n[l] > M - c) return PyLong_FromLongLong(-1);
    for (int64_t j = 0; j < n[l]; ++j, ++c) {
      o[2 * c] = l;
      o[2 * c + 1] = j * 1024;
    }
  }
  for (int64_t j = c; j < M; ++j) {
    o[2 * j] = -1;
    o[2 * j + 1] = 0;
  }
  return PyLong_FromLongLong(c);
}

PyMethodDef methods[] = {
    {"gather_peer_table", gather_peer_table, METH_VARARGS,
     "gather_peer_table(received, keys, numels, device, out) -> 0 (table filled) or 1 (use the Python path)"},
    {"fill_chunk_list", fill_chunk_list, METH_VARARGS,
     "fill_chunk_list(nch int64[L], out int64[2M]) -> chunk total, the (seg, c0) list padded with (-1, 0)"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_host_tables", nullptr, -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__host_tables(void) {
  g_model_key = PyUnicode_InternFromString("model");
  if (!g_model_key) return nullptr;
  return PyModule_Create(&module);
}

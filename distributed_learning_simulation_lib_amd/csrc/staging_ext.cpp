// staging_ext.cpp — host-side staging of one client update for the plugin path (a torch C++
// extension, CPU code only; the HIP library's C ABI stays torch-free).
//
// FedAVGAlgorithm.process_worker_data (fed_avg_algorithm.py:20-64) walks the update's tensors
// once per arrival: per tensor the default hooks take the message's weight (:66-69), add it to
// the per-name total in arrival order (:59-62) and release the payload (:64); the GPU fold needs
// each tensor's device pointer. In Python that walk costs ~0.9 us per tensor (attribute calls on
// torch tensors); here it is ~50 ns. stage_resident() either stages the whole update or changes
// nothing and returns None, so the caller can take its general path (host tensors, mixed dtypes,
// quantised records, a changed shape, a name the layout does not know, ...).
// The same module serves PersonalizedFedAVG's plugin: resident_row() (an arrival in layout order),
// row_pointers() (the checks + pointer pass of a client / output row) and views() (the M x T
// per-receiver result tensors as views of flat buffers).
#include <torch/extension.h>

#include <cstdint>
#include <vector>

namespace {

// 0 fp32, 1 fp16, 2 bf16, 3 fp64 (the kernel input dtypes), -1 other
int dtype_code(c10::ScalarType st) {
  switch (st) {
    case c10::ScalarType::Float: return 0;
    case c10::ScalarType::Half: return 1;
    case c10::ScalarType::BFloat16: return 2;
    case c10::ScalarType::Double: return 3;
    default: return -1;
  }
}

bool same_shape(const at::Tensor& t, PyObject* shape) {
  if (!PyTuple_Check(shape)) return false;
  const Py_ssize_t nd = PyTuple_GET_SIZE(shape);
  const auto sizes = t.sizes();
  if (static_cast<Py_ssize_t>(sizes.size()) != nd) return false;
  for (Py_ssize_t d = 0; d < nd; ++d) {
    const long long v = PyLong_AsLongLong(PyTuple_GET_ITEM(shape, d));
    if (v != sizes[d]) return false;
  }
  return true;
}

// stage_resident(params, index, shapes, device_index, totals, weight)
//   params: dict name -> tensor (the update, in arrival order of its keys)
//   index:  dict name -> native segment (-1: a zero-element tensor of the layout)
//   shapes: list of the native segments' shapes (tuples)
//   totals: dict name -> running total (updated in place, :59-62), weight: int / float
//   device_index: the GPU the tensors must already be on, or -1: host tensors (the pinned
//   ingest then packs them from the returned pointers)
// Returns (ptrs, numels, weights, dtype_code, keep) or None (nothing changed).
py::object stage_resident(py::dict params, py::dict index, py::list shapes, int64_t device_index, py::dict totals,
                          py::object weight) {
  const Py_ssize_t T = PyList_GET_SIZE(shapes.ptr());
  const double w = PyFloat_AsDouble(weight.ptr());
  if (PyErr_Occurred()) {
    PyErr_Clear();
    return py::none();
  }
  std::vector<int64_t> ptrs(T, 0), numels(T, -1);
  std::vector<PyObject*> held(T, nullptr);
  int code = -2;  // no present tensor yet
  PyObject *key, *value;
  Py_ssize_t pos = 0;
  // pass 1: checks only (nothing is changed unless the whole update qualifies)
  while (PyDict_Next(params.ptr(), &pos, &key, &value)) {
    PyObject* seg_obj = PyDict_GetItem(index.ptr(), key);  // borrowed
    if (seg_obj == nullptr) return py::none();              // a name the layout does not know
    const long long seg = PyLong_AsLongLong(seg_obj);
    if (!THPVariable_Check(value)) return py::none();
    const at::Tensor& t = THPVariable_Unpack(value);
    if (seg < 0) {  // a zero-element tensor of the layout: no segment, only its total
      if (t.numel() != 0) return py::none();
      continue;
    }
    if (seg >= T || held[seg] != nullptr) return py::none();
    if (!t.is_contiguous()) return py::none();
    if (device_index >= 0 ? (!t.is_cuda() || t.get_device() != device_index) : !t.is_cpu()) return py::none();
    const int c = dtype_code(t.scalar_type());
    if (c < 0 || (code != -2 && c != code)) return py::none();
    code = c;
    if (!same_shape(t, PyList_GET_ITEM(shapes.ptr(), seg))) return py::none();
    ptrs[seg] = reinterpret_cast<int64_t>(t.data_ptr());
    numels[seg] = t.numel();
    held[seg] = value;
  }
  if (code < 0) return py::none();
  // pass 2: the default hooks' bookkeeping, in the update's key order
  pos = 0;
  while (PyDict_Next(params.ptr(), &pos, &key, &value)) {
    PyObject* cur = PyDict_GetItem(totals.ptr(), key);  // borrowed
    if (cur == nullptr) {
      if (PyDict_SetItem(totals.ptr(), key, weight.ptr()) != 0) throw py::error_already_set();
    } else {
      PyObject* sum = PyNumber_InPlaceAdd(cur, weight.ptr());  // `total += weight`
      if (sum == nullptr) throw py::error_already_set();
      const int rc = PyDict_SetItem(totals.ptr(), key, sum);
      Py_DECREF(sum);
      if (rc != 0) throw py::error_already_set();
    }
  }
  py::list out_ptrs(T), out_numels(T), out_weights(T), keep;
  for (Py_ssize_t s = 0; s < T; ++s) {
    out_ptrs[s] = py::int_(ptrs[s]);
    out_numels[s] = py::int_(numels[s]);
    out_weights[s] = py::float_(held[s] ? w : 0.0);
    if (held[s]) keep.append(py::reinterpret_borrow<py::object>(held[s]));
  }
  return py::make_tuple(out_ptrs, out_numels, out_weights, code, keep);
}

// resident_row(params, index, shapes, device_index) — PersonalizedFedAVG's arrival staging
// (personalized_aggregation_algorithm.py:23-43 keeps the update; the kernel reads it in place):
//   index: dict name -> layout position, shapes: list of the layout's shapes (tuples)
// Returns (row, dtype_code): the update's tensors in layout order (None where absent), or None
// when anything needs the general path (an unknown name, a host tensor, another device, a
// non-contiguous tensor, a second dtype, a changed shape).
py::object resident_row(py::dict params, py::dict index, py::list shapes, int64_t device_index) {
  const Py_ssize_t L = PyList_GET_SIZE(shapes.ptr());
  std::vector<PyObject*> row(L, nullptr);
  int code = -2;
  PyObject *key, *value;
  Py_ssize_t pos = 0;
  while (PyDict_Next(params.ptr(), &pos, &key, &value)) {
    PyObject* at_obj = PyDict_GetItem(index.ptr(), key);
    if (at_obj == nullptr) return py::none();
    const long long i = PyLong_AsLongLong(at_obj);
    if (i < 0 || i >= L || row[i] != nullptr || !THPVariable_Check(value)) return py::none();
    const at::Tensor& t = THPVariable_Unpack(value);
    if (!t.is_cuda() || t.get_device() != device_index || !t.is_contiguous()) return py::none();
    const int c = dtype_code(t.scalar_type());
    if (c < 0 || (code != -2 && c != code)) return py::none();
    code = c;
    if (!same_shape(t, PyList_GET_ITEM(shapes.ptr(), i))) return py::none();
    row[i] = value;
  }
  if (code < 0) return py::none();
  py::list out(L);
  for (Py_ssize_t i = 0; i < L; ++i)
    out[i] = row[i] ? py::reinterpret_borrow<py::object>(row[i]) : py::none();
  return py::make_tuple(out, code);
}

// row_pointers(row, numels, device_index, dtype_code) — the validation + pointer pass of a client
// (or output) row: every present tensor on the device, of the dtype, of numels[t] elements and
// contiguous. Returns the pointers (0 for None), or None if any entry fails (the caller then
// raises its own error naming it).
py::object row_pointers(py::list row, py::list numels, int64_t device_index, int code) {
  const Py_ssize_t T = PyList_GET_SIZE(row.ptr());
  if (PyList_GET_SIZE(numels.ptr()) != T) return py::none();
  py::list out(T);
  for (Py_ssize_t t = 0; t < T; ++t) {
    PyObject* x = PyList_GET_ITEM(row.ptr(), t);
    if (x == Py_None) {
      out[t] = py::int_(0);
      continue;
    }
    if (!THPVariable_Check(x)) return py::none();
    const at::Tensor& v = THPVariable_Unpack(x);
    if (!v.is_cuda() || v.get_device() != device_index || dtype_code(v.scalar_type()) != code ||
        v.numel() != PyLong_AsLongLong(PyList_GET_ITEM(numels.ptr(), t)) || !v.is_contiguous())
      return py::none();
    out[t] = py::int_(reinterpret_cast<int64_t>(v.data_ptr()));
  }
  return out;
}

// views(flat, offsets, shapes) — contiguous views of a flat buffer: element offsets[t], shape
// shapes[t] (the per-receiver result dicts of PersonalizedFedAVG: M x T tensors per round).
py::list views(const at::Tensor& flat, py::list offsets, py::list shapes) {
  const Py_ssize_t T = PyList_GET_SIZE(shapes.ptr());
  if (PyList_GET_SIZE(offsets.ptr()) != T) throw std::invalid_argument("offsets and shapes differ in length");
  if (!flat.is_contiguous() || flat.dim() != 1) throw std::invalid_argument("views of a flat contiguous buffer");
  const int64_t n = flat.numel();
  py::list out(T);
  std::vector<int64_t> size, stride;
  for (Py_ssize_t t = 0; t < T; ++t) {
    PyObject* shape = PyList_GET_ITEM(shapes.ptr(), t);
    if (!PyTuple_Check(shape)) throw std::invalid_argument("shapes must be tuples");
    const Py_ssize_t nd = PyTuple_GET_SIZE(shape);
    size.resize(nd);
    stride.resize(nd);
    int64_t numel = 1;
    for (Py_ssize_t d = nd - 1; d >= 0; --d) {
      size[d] = PyLong_AsLongLong(PyTuple_GET_ITEM(shape, d));
      stride[d] = numel;
      numel *= size[d];
    }
    const int64_t off = PyLong_AsLongLong(PyList_GET_ITEM(offsets.ptr(), t));
    if (off < 0 || off + numel > n) throw std::out_of_range("view outside the buffer");
    out[t] = py::reinterpret_steal<py::object>(
        THPVariable_Wrap(flat.as_strided(size, stride, flat.storage_offset() + off)));
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "host-side staging of plugin updates (see staging_ext.cpp)";
  m.def("stage_resident", &stage_resident);
  m.def("resident_row", &resident_row);
  m.def("row_pointers", &row_pointers);
  m.def("views", &views);
}

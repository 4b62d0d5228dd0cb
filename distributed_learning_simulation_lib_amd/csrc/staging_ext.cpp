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
#include <map>
#include <mutex>
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

// The layout's shapes as native integers. A caller passes the same shapes list (one per layout,
// never mutated) with every arrival; reading its T tuples back from Python objects cost more
// than the rest of an arrival's checks, so the last few lists seen are parsed once and kept. The
// cache holds a reference to each list it keeps (its identity cannot be reused while cached) and
// is only touched under the GIL.
struct ShapeSet {
  PyObject* src = nullptr;  // deliberately never released at exit (no Python calls after finalisation)
  bool ok = false;
  std::vector<int32_t> off;
  std::vector<int64_t> dims;
  bool matches(const at::Tensor& t, int64_t seg) const {
    const auto sizes = t.sizes();
    const int32_t b = off[seg], e = off[seg + 1];
    if (static_cast<int64_t>(sizes.size()) != e - b) return false;
    for (int32_t d = b; d < e; ++d)
      if (dims[d] != sizes[d - b]) return false;
    return true;
  }
};

class ShapeCache {
 public:
  // the parsed set of ``shapes`` (a list of tuples of ints), or nullptr when it is not one
  const ShapeSet* get(PyObject* shapes) {
    for (const ShapeSet& s : sets_)
      if (s.src == shapes) return s.ok ? &s : nullptr;
    ShapeSet& s = sets_[next_];
    next_ = (next_ + 1) % kSets;
    Py_XDECREF(s.src);
    Py_INCREF(shapes);
    s.src = shapes;
    s.ok = parse(shapes, s);
    return s.ok ? &s : nullptr;
  }

 private:
  static bool parse(PyObject* shapes, ShapeSet& s) {
    s.off.clear();
    s.dims.clear();
    if (!PyList_Check(shapes)) return false;
    const Py_ssize_t T = PyList_GET_SIZE(shapes);
    s.off.reserve(T + 1);
    for (Py_ssize_t i = 0; i < T; ++i) {
      PyObject* sh = PyList_GET_ITEM(shapes, i);
      s.off.push_back(static_cast<int32_t>(s.dims.size()));
      if (!PyTuple_Check(sh)) return false;
      for (Py_ssize_t d = 0; d < PyTuple_GET_SIZE(sh); ++d) {
        const long long v = PyLong_AsLongLong(PyTuple_GET_ITEM(sh, d));
        if (v == -1 && PyErr_Occurred()) {
          PyErr_Clear();
          return false;
        }
        s.dims.push_back(v);
      }
    }
    s.off.push_back(static_cast<int32_t>(s.dims.size()));
    return true;
  }
  static constexpr int kSets = 4;  // the staging maps and result geometry of a layout or two
  ShapeSet sets_[kSets];
  int next_ = 0;
};
ShapeCache g_shapes;

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
  const ShapeSet* shp = g_shapes.get(shapes.ptr());
  if (shp == nullptr) return py::none();
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
    if (!shp->matches(t, seg)) return py::none();
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
// Returns (row, dtype_code, pointers): the update's tensors in layout order (None where absent)
// and their device addresses (uint64 bytes, 0 where absent), or None
// when anything needs the general path (an unknown name, a host tensor, another device, a
// non-contiguous tensor, a second dtype, a changed shape).
py::object resident_row(py::dict params, py::dict index, py::list shapes, int64_t device_index) {
  const Py_ssize_t L = PyList_GET_SIZE(shapes.ptr());
  const ShapeSet* shp = g_shapes.get(shapes.ptr());
  if (shp == nullptr) return py::none();
  std::vector<PyObject*> row(L, nullptr);
  std::vector<uint64_t> ptrs(L, 0);
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
    if (!shp->matches(t, i)) return py::none();
    row[i] = value;
    ptrs[i] = reinterpret_cast<uint64_t>(t.data_ptr());
  }
  if (code < 0) return py::none();
  py::list out(L);
  for (Py_ssize_t i = 0; i < L; ++i)
    out[i] = row[i] ? py::reinterpret_borrow<py::object>(row[i]) : py::none();
  return py::make_tuple(out, code,
                        py::bytes(reinterpret_cast<const char*>(ptrs.data()), ptrs.size() * sizeof(uint64_t)));
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

// unobserved(flat, views, offsets, shapes) — true when the result buffer of an earlier round can be
// written again without anyone seeing it change: ``views`` (made by views() below, held by the
// caller's pool list) are the only tensors on the buffer's storage (storage use count = 1 + the
// views), nothing else references them (the list's own reference, no C++ holder, no Python
// attributes, no autograd state, no names) and each still has the geometry views() gave it.
// Anything else — a result the caller kept, a view of a result, its storage object, an in-place
// reshape — answers false and the caller allocates a fresh buffer, as every round did before.
//
// Sharing a storage with another process leaves every count above unchanged: torch.multiprocessing
// swaps the storage's DataPtr for one whose deleter parks the block in its IPC limbo (CUDA tensors:
// CudaIPCSentData) or moves it to shared memory (host tensors), so the buffer must also still carry
// the deleter of the allocator that made it — the one a fresh allocation with its options gets.
bool allocator_owned(const at::Tensor& flat) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, c10::DeleterFnPtr> native;  // (device type, index) -> deleter
  const std::pair<int, int> key{static_cast<int>(flat.device().type()), static_cast<int>(flat.device().index())};
  c10::DeleterFnPtr want = nullptr;
  {
    std::lock_guard<std::mutex> lock(mu);
    auto it = native.find(key);
    if (it != native.end()) want = it->second;
  }
  if (want == nullptr) {
    const at::Tensor probe = at::empty({1}, flat.options());
    want = probe.storage().data_ptr().get_deleter();
    std::lock_guard<std::mutex> lock(mu);
    native[key] = want;
  }
  return want != nullptr && flat.storage().data_ptr().get_deleter() == want;
}

// foreign(t) — t's memory was not allocated by this process's allocator: a tensor received from
// another process through torch.multiprocessing (CUDA IPC: the sender holds a context on this GPU,
// e.g. a worker training there), or external memory. FedAVGAlgorithm then keeps its dynamic wave
// off for the round (the wave would hold the register file while that process computes).
bool foreign(const at::Tensor& t) { return t.has_storage() && t.storage().data() != nullptr && !allocator_owned(t); }

bool unobserved(const at::Tensor& flat, py::list views, py::list offsets, py::list shapes) {
  const Py_ssize_t T = PyList_GET_SIZE(views.ptr());
  const ShapeSet* shp = g_shapes.get(shapes.ptr());
  if (shp == nullptr || PyList_GET_SIZE(shapes.ptr()) != T || PyList_GET_SIZE(offsets.ptr()) != T ||
      !flat.has_storage() || flat.dim() != 1 || !flat.is_contiguous())
    return false;
  const c10::Storage& st = flat.storage();
  if (st.use_count() != 1 + static_cast<int64_t>(T)) return false;
  if (!allocator_owned(flat)) return false;
  const char* base = static_cast<const char*>(st.data()) + flat.storage_offset() * flat.itemsize();
  for (Py_ssize_t t = 0; t < T; ++t) {
    PyObject* o = PyList_GET_ITEM(views.ptr(), t);
    if (Py_REFCNT(o) != 1 || !THPVariable_Check(o)) return false;
    PyObject** dict = _PyObject_GetDictPtr(o);
    if (dict != nullptr && *dict != nullptr && PyDict_Size(*dict) != 0) return false;
    const at::Tensor& v = THPVariable_Unpack(o);
    if (v.use_count() != 1 || v.requires_grad() || v.has_names() || !v.is_contiguous() ||
        v.scalar_type() != flat.scalar_type() || !v.has_storage() || !v.storage().is_alias_of(st))
      return false;
    const int64_t off = PyLong_AsLongLong(PyList_GET_ITEM(offsets.ptr(), t));
    if (static_cast<const char*>(v.const_data_ptr()) != base + off * flat.itemsize()) return false;
    if (!shp->matches(v, t)) return false;
  }
  return true;
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

// Rows — the client table of one wave, held natively ([num_clients][T] device pointers, fp64
// weights, element counts; references to the staged tensors). FedAVGAlgorithm appends one update
// per arrival with append(): one pass over the update's dict that checks every tensor (known name,
// contiguous, on the device, one kernel dtype, the layout's shape) and writes its row straight
// into the table — no Python list per update, no second pass at launch time (the arrays are
// already contiguous). The per-name totals (fed_avg_algorithm.py:59-62) stay with the caller:
// append() reports whether the update carried every name of the layout, so the caller can keep
// one running total for all names while every update is complete.
class Rows {
 public:
  Rows(int64_t T, int64_t device_index) : T_(T), dev_(device_index) {
    if (T < 1) throw std::invalid_argument("a table needs at least one segment");
  }
  Rows(const Rows&) = delete;
  Rows& operator=(const Rows&) = delete;
  ~Rows() {
    for (PyObject* o : keep_) Py_DECREF(o);  // pybind11 destroys the holder with the GIL held
  }

  // append(params, index, shapes, weight, want_code) -> int
  //   >= 0: staged; the low 4 bits are the dtype code, bit 4 (16) is set when the update carried
  //         every name of ``index`` (a complete update)
  //   -1:   nothing changed — the update needs the general path
  //   -2 - c: nothing changed — a valid update of dtype code c, but the table holds ``want_code``
  //   want_code: the table's dtype code, or -1 when the table is still empty
  int append(py::dict params, py::dict index, py::list shapes, py::object weight, int want_code) {
    const double w = PyFloat_AsDouble(weight.ptr());
    if (PyErr_Occurred()) {
      PyErr_Clear();
      return -1;
    }
    if (PyList_GET_SIZE(shapes.ptr()) != T_) return -1;
    const ShapeSet* shp = g_shapes.get(shapes.ptr());
    if (shp == nullptr) return -1;
    const size_t base = ptrs_.size();
    ptrs_.resize(base + T_, 0);
    numels_.resize(base + T_, -1);
    uint64_t* p = ptrs_.data() + base;
    int64_t* n = numels_.data() + base;
    const size_t kbase = keep_.size();
    keep_.reserve(kbase + T_);
    int code = -2;
    Py_ssize_t seen = 0;
    PyObject *key, *value;
    Py_ssize_t pos = 0;
    auto rollback = [&](int rc) {
      ptrs_.resize(base);
      numels_.resize(base);
      for (size_t i = kbase; i < keep_.size(); ++i) Py_DECREF(keep_[i]);
      keep_.resize(kbase);
      return rc;
    };
    while (PyDict_Next(params.ptr(), &pos, &key, &value)) {
      PyObject* seg_obj = PyDict_GetItem(index.ptr(), key);  // borrowed
      if (seg_obj == nullptr) return rollback(-1);           // a name the layout does not know
      ++seen;
      const long long seg = PyLong_AsLongLong(seg_obj);
      if (!THPVariable_Check(value)) return rollback(-1);
      const at::Tensor& t = THPVariable_Unpack(value);
      if (seg < 0) {  // a zero-element tensor of the layout: no segment
        if (t.numel() != 0) return rollback(-1);
        continue;
      }
      if (seg >= T_ || n[seg] >= 0) return rollback(-1);
      if (!t.is_cuda() || t.get_device() != dev_ || !t.is_contiguous()) return rollback(-1);
      const int c = dtype_code(t.scalar_type());
      if (c < 0 || (code != -2 && c != code)) return rollback(-1);
      code = c;
      if (!shp->matches(t, seg)) return rollback(-1);
      p[seg] = reinterpret_cast<uint64_t>(t.data_ptr());
      n[seg] = t.numel();
      // the tensor's Python object keeps it alive until the table is dropped (a plain reference
      // count, not the atomic one of an at::Tensor copy)
      Py_INCREF(value);
      keep_.push_back(value);
    }
    if (code < 0) return rollback(-1);
    if (want_code >= 0 && code != want_code) return rollback(-2 - code);
    if (esize_ == 0) esize_ = esize_of(code);
    weights_.resize(base + T_);
    double* wr = weights_.data() + base;
    for (int64_t s = 0; s < T_; ++s) wr[s] = n[s] >= 0 ? w : 0.0;
    ++rows_;
    const bool complete = seen == PyDict_Size(index.ptr());
    return code | (complete ? 16 : 0);
  }

  // append_row(ptrs, weights, numels, esize, keep): a row the caller has checked (the general
  // staging path, host updates packed by the pinned ingest); numels[s] == -1 marks an absent entry
  void append_row(py::list ptrs, py::list weights, py::list numels, int64_t esize, py::list keep) {
    if (PyList_GET_SIZE(ptrs.ptr()) != T_ || PyList_GET_SIZE(weights.ptr()) != T_ ||
        PyList_GET_SIZE(numels.ptr()) != T_)
      throw std::invalid_argument("client row does not match the layout");
    if (esize_ != 0 && esize != esize_) throw std::invalid_argument("a row of another element size");
    const size_t base = ptrs_.size();
    std::vector<uint64_t> p(T_);
    std::vector<double> wr(T_);
    std::vector<int64_t> nr(T_);
    for (int64_t s = 0; s < T_; ++s) {
      p[s] = PyLong_AsUnsignedLongLongMask(PyList_GET_ITEM(ptrs.ptr(), s));
      wr[s] = PyFloat_AsDouble(PyList_GET_ITEM(weights.ptr(), s));
      nr[s] = PyLong_AsLongLong(PyList_GET_ITEM(numels.ptr(), s));
    }
    if (PyErr_Occurred()) throw py::error_already_set();
    ptrs_.insert(ptrs_.end(), p.begin(), p.end());
    weights_.insert(weights_.end(), wr.begin(), wr.end());
    numels_.insert(numels_.end(), nr.begin(), nr.end());
    (void)base;
    for (auto item : keep) extra_keep_.push_back(py::reinterpret_borrow<py::object>(item));
    esize_ = esize;
    ++rows_;
  }

  // validate(numels, esize, device_index): every present entry has numels[s] elements of esize
  // bytes on the device. Returns "" or a message naming the first bad entry.
  std::string validate(py::list numels, int64_t esize, int64_t device_index) const {
    if (PyList_GET_SIZE(numels.ptr()) != T_) return "the layout does not match the table";
    std::vector<int64_t> want(T_);
    for (int64_t s = 0; s < T_; ++s) want[s] = PyLong_AsLongLong(PyList_GET_ITEM(numels.ptr(), s));
    if (rows_ && (esize != esize_ || device_index != dev_))
      return "rows of " + std::to_string(esize_) + "-byte elements on device " + std::to_string(dev_) +
             "; the input format needs " + std::to_string(esize) + " bytes on device " + std::to_string(device_index);
    for (int64_t k = 0; k < rows_; ++k)
      for (int64_t s = 0; s < T_; ++s) {
        const int64_t have = numels_[k * T_ + s];
        if (have >= 0 && have != want[s])
          return "client " + std::to_string(k) + ", tensor " + std::to_string(s) + ": " + std::to_string(have) +
                 " elements; the layout needs " + std::to_string(want[s]);
      }
    return "";
  }

  py::bytes ptr_bytes() const {
    return py::bytes(reinterpret_cast<const char*>(ptrs_.data()), ptrs_.size() * sizeof(uint64_t));
  }
  py::bytes weight_bytes() const {
    return py::bytes(reinterpret_cast<const char*>(weights_.data()), weights_.size() * sizeof(double));
  }
  py::bytes numel_bytes() const {
    return py::bytes(reinterpret_cast<const char*>(numels_.data()), numels_.size() * sizeof(int64_t));
  }
  // host addresses of the [clients][segments] pointer / weight arrays, valid until the next append
  // (what FedAvgContext hands the C ABI, without a copy into Python objects)
  uint64_t ptr_addr() const { return reinterpret_cast<uint64_t>(ptrs_.data()); }
  uint64_t weight_addr() const { return reinterpret_cast<uint64_t>(weights_.data()); }
  int64_t num_clients() const { return rows_; }
  int64_t num_segments() const { return T_; }
  int64_t esize() const { return esize_; }

 private:
  static int64_t esize_of(int code) { return code == 3 ? 8 : (code == 0 ? 4 : 2); }
  int64_t T_, dev_;
  int64_t rows_ = 0, esize_ = 0;
  std::vector<uint64_t> ptrs_;
  std::vector<double> weights_;
  std::vector<int64_t> numels_;
  std::vector<PyObject*> keep_;       // owned references: the staged tensors outlive the table's launches
  std::vector<py::object> extra_keep_;
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "host-side staging of plugin updates (see staging_ext.cpp)";
  py::class_<Rows>(m, "Rows")
      .def(py::init<int64_t, int64_t>())
      .def("append", &Rows::append)
      .def("append_row", &Rows::append_row)
      .def("validate", &Rows::validate)
      .def("ptr_bytes", &Rows::ptr_bytes)
      .def("weight_bytes", &Rows::weight_bytes)
      .def("numel_bytes", &Rows::numel_bytes)
      .def("ptr_addr", &Rows::ptr_addr)
      .def("weight_addr", &Rows::weight_addr)
      .def_property_readonly("num_clients", &Rows::num_clients)
      .def_property_readonly("num_segments", &Rows::num_segments)
      .def_property_readonly("esize", &Rows::esize);
  m.def("stage_resident", &stage_resident);
  m.def("resident_row", &resident_row);
  m.def("row_pointers", &row_pointers);
  m.def("views", &views);
  m.def("unobserved", &unobserved);
  m.def("foreign", &foreign);
}

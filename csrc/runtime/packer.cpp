// Native Row -> column packer (the boxed conversion path).
//
// The reference converts Spark Rows cell by cell into java.nio buffers through
// a per-type TensorConverter (reference:
// src/main/scala/org/tensorframes/impl/datatypes.scala:114-127 appendRaw /
// append for cell rank 0/1/2, driven by DataOps.convertFast0,
// src/main/scala/org/tensorframes/impl/DataOps.scala:63-81). Here the rows
// are Python tuples (our Row is a tuple subclass); one C++ pass reads column
// `col` of rows [begin, end) straight from the tuple slots and writes a
// contiguous tensor, with no intermediate Python list or numpy object array.
// Cells of rank 0, 1 (lists/tuples) and 2 (lists of lists) are packed when
// every cell of the slice has the same shape; anything else (ragged cells,
// ndarray cells, strings) returns None and the caller keeps its generic path.
#include <torch/extension.h>
#include <pybind11/numpy.h>

#include <cstring>
#include <limits>

#include "../common.h"
#include "../ir/graph.h"

namespace py = pybind11;

namespace tfa {
namespace {

enum class Slot { F64, F32, I32, I64, U8 };

// status: 0 ok, 1 unsupported (fall back), 2 null cell (error)
template <typename T>
inline int put_scalar(PyObject* o, T* dst) {
  if (o == Py_None) return 2;
  if constexpr (std::is_floating_point<T>::value) {
    if (PyFloat_CheckExact(o)) {
      *dst = static_cast<T>(PyFloat_AS_DOUBLE(o));
      return 0;
    }
    if (PyLong_Check(o) && !PyBool_Check(o)) {
      double v = PyLong_AsDouble(o);
      if (v == -1.0 && PyErr_Occurred()) { PyErr_Clear(); return 1; }
      *dst = static_cast<T>(v);
      return 0;
    }
    if (PyFloat_Check(o)) {  // numpy float64 and other float subclasses
      *dst = static_cast<T>(PyFloat_AsDouble(o));
      return 0;
    }
    return 1;
  } else {
    if (PyLong_Check(o) && !PyBool_Check(o)) {
      int overflow = 0;
      long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
      if (overflow || (v == -1 && PyErr_Occurred())) { PyErr_Clear(); return 1; }
      // out of the column type's range: the generic path reports it
      if (v < (long long)std::numeric_limits<T>::lowest() || v > (long long)std::numeric_limits<T>::max()) return 1;
      *dst = static_cast<T>(v);
      return 0;
    }
    return 1;
  }
}

// cell shape of a value: rank 0 scalars, rank 1/2 lists or tuples (no ndarray)
bool cell_shape(PyObject* v, std::vector<int64_t>* shape) {
  shape->clear();
  if (PyList_Check(v) || (PyTuple_Check(v))) {
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(v);
    shape->push_back(n);
    if (n == 0) return true;
    PyObject* f = PySequence_Fast_GET_ITEM(v, 0);
    if (PyList_Check(f) || PyTuple_Check(f)) {
      shape->push_back(PySequence_Fast_GET_SIZE(f));
      PyObject* g = PySequence_Fast_GET_SIZE(f) ? PySequence_Fast_GET_ITEM(f, 0) : nullptr;
      if (g && (PyList_Check(g) || PyTuple_Check(g))) return false;  // rank > 2: not a supported cell
    }
    return true;
  }
  return PyFloat_Check(v) || PyLong_Check(v);
}

template <typename T>
int pack_typed(PyObject* rows, Py_ssize_t col, Py_ssize_t ncols, Py_ssize_t b, Py_ssize_t e,
               const std::vector<int64_t>& shape, T* out) {
  const int rank = static_cast<int>(shape.size());
  const int64_t inner0 = rank >= 1 ? shape[0] : 1, inner1 = rank >= 2 ? shape[1] : 1;
  const int64_t cell = inner0 * inner1;
  for (Py_ssize_t r = b; r < e; ++r) {
    PyObject* row = PyList_GET_ITEM(rows, r);
    if (!PyTuple_Check(row)) return 1;  // lists etc.: the generic path normalises them
    if (PyTuple_GET_SIZE(row) != ncols) return 3;
    PyObject* v = PyTuple_GET_ITEM(row, col);
    T* dst = out + (r - b) * cell;
    if (rank == 0) {
      int st = put_scalar<T>(v, dst);
      if (st) return st;
      continue;
    }
    if (v == Py_None) return 2;
    if (!(PyList_Check(v) || PyTuple_Check(v)) || PySequence_Fast_GET_SIZE(v) != inner0) return 1;
    PyObject** items = PySequence_Fast_ITEMS(v);
    for (int64_t i = 0; i < inner0; ++i) {
      if (rank == 1) {
        int st = put_scalar<T>(items[i], dst + i);
        if (st) return st == 2 ? 2 : 1;
      } else {
        PyObject* w = items[i];
        if (!(PyList_Check(w) || PyTuple_Check(w)) || PySequence_Fast_GET_SIZE(w) != inner1) return 1;
        PyObject** it2 = PySequence_Fast_ITEMS(w);
        for (int64_t j = 0; j < inner1; ++j) {
          int st = put_scalar<T>(it2[j], dst + i * inner1 + j);
          if (st) return st == 2 ? 2 : 1;
        }
      }
    }
  }
  return 0;
}

}  // namespace

// rows: list of tuples (Row is a tuple subclass), every one with `ncols`
// fields. Returns a tensor [end - begin, *cell] of dtype `tf_dtype`, or None
// when the slice needs the generic path. Raises ValueError on a null cell or a
// row of the wrong width.
py::object pack_column(py::list rows, int64_t col, int64_t ncols, int64_t begin, int64_t end, int tf_dtype) {
  PyObject* lst = rows.ptr();
  const Py_ssize_t n = PyList_GET_SIZE(lst);
  TFA_CHECK(begin >= 0 && end <= n && begin <= end, "pack_column: bad row range");
  TFA_CHECK(col >= 0 && col < ncols, "pack_column: bad column");
  const DType dt = static_cast<DType>(tf_dtype);
  at::ScalarType st;
  switch (dt) {
    case DType::F64: st = at::kDouble; break;
    case DType::F32: st = at::kFloat; break;
    case DType::I32: st = at::kInt; break;
    case DType::I64: st = at::kLong; break;
    default: return py::none();
  }
  std::vector<int64_t> shape;
  if (end > begin) {
    PyObject* row0 = PyList_GET_ITEM(lst, begin);
    if (!PyTuple_Check(row0) || PyTuple_GET_SIZE(row0) != ncols) return py::none();
    PyObject* v0 = PyTuple_GET_ITEM(row0, col);
    if (v0 == Py_None) throw py::value_error("null cell");
    if (!cell_shape(v0, &shape)) return py::none();
  }
  std::vector<int64_t> sizes{end - begin};
  sizes.insert(sizes.end(), shape.begin(), shape.end());
  at::Tensor out = at::empty(sizes, at::TensorOptions().dtype(st));
  if (end == begin) return py::cast(out);
  int status = 0;
  switch (dt) {
    case DType::F64: status = pack_typed<double>(lst, col, ncols, begin, end, shape, out.data_ptr<double>()); break;
    case DType::F32: status = pack_typed<float>(lst, col, ncols, begin, end, shape, out.data_ptr<float>()); break;
    case DType::I32: status = pack_typed<int32_t>(lst, col, ncols, begin, end, shape, out.data_ptr<int32_t>()); break;
    case DType::I64: status = pack_typed<int64_t>(lst, col, ncols, begin, end, shape, out.data_ptr<int64_t>()); break;
    default: return py::none();
  }
  if (status == 2) throw py::value_error("null cell");
  if (status == 3) throw py::value_error("row of the wrong width");
  if (status != 0) return py::none();
  return py::cast(out);
}

// ------------------------------------------------------------------ columns -> Rows
// The reverse direction, the reference's convertBack (reference:
// src/main/scala/org/tensorframes/impl/DataOps.scala:20-61 convertBackFast0,
// one GenericRow per row from the reshaped column buffers). Dense columns
// arrive as numpy arrays [rows, *cell] and are read straight from their
// buffers: rank-0 cells become Python scalars, higher ranks nested lists (a
// Spark array column). Other columns arrive as lists of ready values. Each
// Row is allocated directly as an instance of the (tuple-subclass) row type
// and its slots filled in place: no intermediate tuple, zip or per-row dict.
namespace {

enum class Kind { F32, F64, I8, I16, I32, I64, U8, U16, U32, U64, BOOL, LIST };

struct ColView {
  Kind kind = Kind::LIST;
  const char* ptr = nullptr;
  std::vector<int64_t> shape;    // cell dims
  std::vector<int64_t> strides;  // bytes: [row, cell dims...]
  PyObject* list = nullptr;
};

inline PyObject* scalar_at(Kind k, const char* p) {
  switch (k) {
    case Kind::F32: return PyFloat_FromDouble(*reinterpret_cast<const float*>(p));
    case Kind::F64: return PyFloat_FromDouble(*reinterpret_cast<const double*>(p));
    case Kind::I8: return PyLong_FromLong(*reinterpret_cast<const int8_t*>(p));
    case Kind::I16: return PyLong_FromLong(*reinterpret_cast<const int16_t*>(p));
    case Kind::I32: return PyLong_FromLong(*reinterpret_cast<const int32_t*>(p));
    case Kind::I64: return PyLong_FromLongLong(*reinterpret_cast<const int64_t*>(p));
    case Kind::U8: return PyLong_FromLong(*reinterpret_cast<const uint8_t*>(p));
    case Kind::U16: return PyLong_FromLong(*reinterpret_cast<const uint16_t*>(p));
    case Kind::U32: return PyLong_FromUnsignedLong(*reinterpret_cast<const uint32_t*>(p));
    case Kind::U64: return PyLong_FromUnsignedLongLong(*reinterpret_cast<const uint64_t*>(p));
    case Kind::BOOL: return PyBool_FromLong(*reinterpret_cast<const bool*>(p));
    default: return nullptr;
  }
}

// nested list of the cell at p over dims [d, rank)
PyObject* cell_list(const ColView& c, const char* p, size_t d) {
  if (d == c.shape.size()) return scalar_at(c.kind, p);
  const int64_t n = c.shape[d];
  PyObject* l = PyList_New(n);
  if (!l) return nullptr;
  for (int64_t i = 0; i < n; ++i) {
    PyObject* v = cell_list(c, p + i * c.strides[d + 1], d + 1);
    if (!v) {
      Py_DECREF(l);
      return nullptr;
    }
    PyList_SET_ITEM(l, i, v);
  }
  return l;
}

Kind kind_of(const py::dtype& dt) {
  const char k = dt.kind();
  const ssize_t sz = dt.itemsize();
  if (k == 'f') return sz == 4 ? Kind::F32 : sz == 8 ? Kind::F64 : Kind::LIST;
  if (k == 'i') return sz == 1 ? Kind::I8 : sz == 2 ? Kind::I16 : sz == 4 ? Kind::I32 : sz == 8 ? Kind::I64 : Kind::LIST;
  if (k == 'u') return sz == 1 ? Kind::U8 : sz == 2 ? Kind::U16 : sz == 4 ? Kind::U32 : sz == 8 ? Kind::U64 : Kind::LIST;
  if (k == 'b') return Kind::BOOL;
  return Kind::LIST;
}

}  // namespace

// Fills out[at, at + nrows) with rows of one segment. cols[j]: numpy array
// [nrows, *cell] (numeric/bool) or a list of nrows values.
void fill_rows(PyTypeObject* tp, py::list cols, int64_t nrows, PyObject* out, int64_t at) {
  const Py_ssize_t ncols = PyList_GET_SIZE(cols.ptr());
  std::vector<ColView> views(ncols);
  std::vector<py::object> keep;  // arrays stay alive while their buffers are read
  for (Py_ssize_t j = 0; j < ncols; ++j) {
    py::handle c = PyList_GET_ITEM(cols.ptr(), j);
    ColView& v = views[j];
    if (PyList_Check(c.ptr())) {
      TFA_CHECK(PyList_GET_SIZE(c.ptr()) == nrows, "build_rows: column ", j, " has ", PyList_GET_SIZE(c.ptr()),
                " values for ", nrows, " rows");
      v.list = c.ptr();
      continue;
    }
    TFA_CHECK(py::isinstance<py::array>(c), "build_rows: column ", j, " must be a numpy array or a list");
    py::array a = py::reinterpret_borrow<py::array>(c);
    v.kind = kind_of(a.dtype());
    TFA_CHECK(v.kind != Kind::LIST, "build_rows: unsupported array dtype in column ", j);
    TFA_CHECK(a.ndim() >= 1 && a.shape(0) == nrows, "build_rows: column ", j, " has the wrong row count");
    v.ptr = static_cast<const char*>(a.data());
    for (ssize_t d = 0; d < a.ndim(); ++d) {
      if (d) v.shape.push_back(a.shape(d));
      v.strides.push_back(a.strides(d));
    }
    keep.push_back(a);
  }
  for (int64_t r = 0; r < nrows; ++r) {
    PyObject* row = tp->tp_alloc(tp, ncols);
    if (!row) throw py::error_already_set();
    PyList_SET_ITEM(out, at + r, row);  // owned by the list from here (errors free it with the list)
    for (Py_ssize_t j = 0; j < ncols; ++j) {
      const ColView& v = views[j];
      PyObject* val;
      if (v.list) {
        val = PyList_GET_ITEM(v.list, r);
        Py_INCREF(val);
      } else {
        const char* p = v.ptr + r * v.strides[0];
        val = v.shape.empty() ? scalar_at(v.kind, p) : cell_list(v, p, 0);
        if (!val) throw py::error_already_set();
      }
      PyTuple_SET_ITEM(row, j, val);
    }
  }
}

// segments: [(nrows, cols)] in output order -> one list of row_type
// instances (a tuple subclass), built in one pass over all segments
py::list build_rows(py::object row_type, py::list segments) {
  PyObject* tp_obj = row_type.ptr();
  TFA_CHECK(PyType_Check(tp_obj) && PyType_IsSubtype(reinterpret_cast<PyTypeObject*>(tp_obj), &PyTuple_Type),
            "build_rows: row type must be a tuple subclass");
  PyTypeObject* tp = reinterpret_cast<PyTypeObject*>(tp_obj);
  int64_t total = 0;
  for (auto seg : segments) total += seg.cast<py::tuple>()[0].cast<int64_t>();
  PyObject* out = PyList_New(total);
  if (!out) throw py::error_already_set();
  py::list result = py::reinterpret_steal<py::list>(out);
  int64_t at = 0;
  for (auto seg : segments) {
    py::tuple t = seg.cast<py::tuple>();
    const int64_t n = t[0].cast<int64_t>();
    fill_rows(tp, t[1].cast<py::list>(), n, out, at);
    at += n;
  }
  return result;
}

void register_packer(py::module& m) {
  m.def("pack_column", &pack_column, py::arg("rows"), py::arg("col"), py::arg("ncols"), py::arg("begin"),
        py::arg("end"), py::arg("tf_dtype"),
        "column `col` of rows[begin:end] (tuples) -> contiguous tensor, or None for the generic path");
  m.def("build_rows", &build_rows, py::arg("row_type"), py::arg("segments"),
        "[(nrows, columns)] (numpy arrays [rows, *cell] or value lists) -> one list of row_type instances");
}

}  // namespace tfa

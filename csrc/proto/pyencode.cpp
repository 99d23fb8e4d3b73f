// Native GraphDef node encoder for the Python DSL.
//
// The DSL (tensorframes_amd/graph/dsl.py) keeps nodes as small Python
// objects (graph/proto.py NodeDef / AttrValue / TensorProto) and serialises
// them to protobuf wire format before every analyze / map_blocks call. Graphs
// rebuilt per iteration (the reference K-Means demo rebuilds both graphs with
// new centres every step: src/main/python/tensorframes_snippets/kmeans_demo.py:68-168)
// spent about a quarter of their host time in the pure-Python encoder; this
// file produces byte-identical output in one C++ pass over the node objects.
// proto.py stays the reference encoder (and the fallback for anything this
// one does not cover: it raises, and the caller re-encodes in Python).
#include <torch/extension.h>

#include <cstring>
#include <string>

#include "../common.h"

namespace py = pybind11;

namespace tfa {
namespace {

struct Unsupported {};

// TF DataType enum values used by the typed `*_val` single-element rule
enum : int { DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_UINT8 = 4, DT_INT16 = 5, DT_INT8 = 6, DT_STRING = 7,
             DT_INT64 = 9, DT_BOOL = 10, DT_BFLOAT16 = 14, DT_UINT16 = 17, DT_HALF = 19, DT_UINT32 = 22,
             DT_UINT64 = 23 };

inline void varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o.push_back(static_cast<char>(v));
}
inline void key(std::string& o, int field, int wt) { varint(o, (static_cast<uint64_t>(field) << 3) | wt); }
inline void ld(std::string& o, int field, const std::string& payload) {
  key(o, field, 2);
  varint(o, payload.size());
  o += payload;
}
inline void ld(std::string& o, int field, const char* p, size_t n) {
  key(o, field, 2);
  varint(o, n);
  o.append(p, n);
}

// interned attribute names
struct Names {
  py::object name, op, input, device, attr, kind, value, dtype, shape, content, strings, dims, unknown_rank;
  Names()
      : name(py::str("name")), op(py::str("op")), input(py::str("input")), device(py::str("device")),
        attr(py::str("attr")), kind(py::str("kind")), value(py::str("value")), dtype(py::str("dtype")),
        shape(py::str("shape")), content(py::str("content")), strings(py::str("strings")), dims(py::str("dims")),
        unknown_rank(py::str("unknown_rank")) {}
};
Names& names() {
  static Names* n = new Names();  // lives for the process (no teardown-order issues)
  return *n;
}

inline py::object get(py::handle o, const py::object& nm) { return py::reinterpret_steal<py::object>(
    PyObject_GetAttr(o.ptr(), nm.ptr())) ; }

std::string str_bytes(py::handle v) {
  if (PyBytes_Check(v.ptr())) return std::string(PyBytes_AS_STRING(v.ptr()), PyBytes_GET_SIZE(v.ptr()));
  if (PyUnicode_Check(v.ptr())) {
    Py_ssize_t n = 0;
    const char* s = PyUnicode_AsUTF8AndSize(v.ptr(), &n);
    if (!s) throw py::error_already_set();
    return std::string(s, n);
  }
  throw Unsupported{};
}

int64_t as_i64(py::handle v) {
  if (!PyLong_Check(v.ptr())) throw Unsupported{};
  int overflow = 0;
  long long x = PyLong_AsLongLongAndOverflow(v.ptr(), &overflow);
  if (overflow) throw Unsupported{};
  return x;
}

void enc_shape_dims(std::string& o, const std::vector<int64_t>& dims, bool unknown) {
  if (unknown) {
    key(o, 3, 0);
    varint(o, 1);
    return;
  }
  for (int64_t d : dims) {
    std::string dim;
    if (d != 0) {
      key(dim, 1, 0);
      varint(dim, static_cast<uint64_t>(d));
    }
    ld(o, 2, dim);
  }
}

void enc_shape(std::string& o, py::handle s) {
  Names& N = names();
  bool unknown = PyObject_IsTrue(get(s, N.unknown_rank).ptr()) == 1;
  std::vector<int64_t> dims;
  if (!unknown)
    for (auto d : get(s, N.dims)) dims.push_back(as_i64(d));
  enc_shape_dims(o, dims, unknown);
}

void typed_val(std::string& o, int dt, const char* p, size_t n) {
  auto need = [&](size_t k) {
    if (n < k) throw Unsupported{};
  };
  switch (dt) {
    case DT_FLOAT: need(4); ld(o, 5, p, 4); return;
    case DT_DOUBLE: need(8); ld(o, 6, p, 8); return;
    case DT_INT64: {
      need(8); int64_t v; std::memcpy(&v, p, 8);
      std::string s; varint(s, static_cast<uint64_t>(v)); ld(o, 10, s); return;
    }
    case DT_BOOL: {
      need(1); std::string s; varint(s, p[0] ? 1 : 0); ld(o, 11, s); return;
    }
    case DT_HALF: {
      need(2); uint16_t v; std::memcpy(&v, p, 2);
      std::string s; varint(s, v); ld(o, 13, s); return;
    }
    default: break;
  }
  int64_t v;
  switch (dt) {
    case DT_INT32: { need(4); int32_t x; std::memcpy(&x, p, 4); v = x; break; }
    case DT_UINT8: { need(1); v = static_cast<uint8_t>(p[0]); break; }
    case DT_INT16: { need(2); int16_t x; std::memcpy(&x, p, 2); v = x; break; }
    case DT_INT8: { need(1); v = static_cast<int8_t>(p[0]); break; }
    case DT_UINT16: { need(2); uint16_t x; std::memcpy(&x, p, 2); v = x; break; }
    case DT_UINT32: { need(4); uint32_t x; std::memcpy(&x, p, 4); v = x; break; }
    default: throw Unsupported{};  // uint64 / complex / ...: the Python encoder decides
  }
  std::string s;
  varint(s, static_cast<uint64_t>(v));
  ld(o, 7, s);
}

void enc_tensor(std::string& o, py::handle t) {
  Names& N = names();
  int dt = static_cast<int>(as_i64(get(t, N.dtype)));
  std::vector<int64_t> shape;
  int64_t numel = 1;
  for (auto d : get(t, N.shape)) {
    shape.push_back(as_i64(d));
    numel *= shape.back();
  }
  key(o, 1, 0);
  varint(o, static_cast<uint64_t>(dt));
  std::string sh;
  enc_shape_dims(sh, shape, false);
  ld(o, 2, sh);
  if (dt == DT_STRING) {
    py::object strs = get(t, N.strings);
    if (!strs.is_none())
      for (auto s : strs) ld(o, 8, str_bytes(s));
    return;
  }
  py::object content = get(t, N.content);
  if (!PyBytes_Check(content.ptr())) throw Unsupported{};
  const char* p = PyBytes_AS_STRING(content.ptr());
  size_t n = PyBytes_GET_SIZE(content.ptr());
  if (numel == 1 && dt != DT_BFLOAT16) {
    typed_val(o, dt, p, n);
  } else if (numel > 1) {
    ld(o, 4, p, n);
  }
}

void enc_list(std::string& o, py::handle l) {
  if (!PyDict_Check(l.ptr())) throw Unsupported{};
  py::dict d = py::reinterpret_borrow<py::dict>(l);
  auto field = [&](const char* k) -> py::object {
    PyObject* v = PyDict_GetItemString(d.ptr(), k);
    return v ? py::reinterpret_borrow<py::object>(v) : py::object();
  };
  auto nonempty = [](const py::object& v) { return v && PyObject_IsTrue(v.ptr()) == 1; };
  for (auto k : d) {
    std::string ks = str_bytes(k.first);
    if (ks != "s" && ks != "i" && ks != "f" && ks != "b" && ks != "type" && ks != "shape" && ks != "tensor")
      throw Unsupported{};
  }
  if (py::object v = field("s"))
    for (auto s : v) ld(o, 2, str_bytes(s));
  if (py::object v = field("i"); nonempty(v)) {
    std::string p;
    for (auto x : v) varint(p, static_cast<uint64_t>(as_i64(x)));
    ld(o, 3, p);
  }
  if (py::object v = field("f"); nonempty(v)) {
    std::string p;
    for (auto x : v) {
      float f = static_cast<float>(PyFloat_AsDouble(x.ptr()));
      if (PyErr_Occurred()) throw py::error_already_set();
      p.append(reinterpret_cast<const char*>(&f), 4);
    }
    ld(o, 4, p);
  }
  if (py::object v = field("b"); nonempty(v)) {
    std::string p;
    for (auto x : v) varint(p, PyObject_IsTrue(x.ptr()) == 1 ? 1 : 0);
    ld(o, 5, p);
  }
  if (py::object v = field("type"); nonempty(v)) {
    std::string p;
    for (auto x : v) varint(p, static_cast<uint64_t>(as_i64(x)));
    ld(o, 6, p);
  }
  if (py::object v = field("shape"))
    for (auto s : v) {
      std::string p;
      enc_shape(p, s);
      ld(o, 7, p);
    }
  if (py::object v = field("tensor"))
    for (auto t : v) {
      std::string p;
      enc_tensor(p, t);
      ld(o, 8, p);
    }
}

void enc_attr(std::string& o, py::handle a) {
  Names& N = names();
  std::string k = str_bytes(get(a, N.kind));
  py::object v = get(a, N.value);
  if (k == "list") {
    std::string p;
    enc_list(p, v);
    ld(o, 1, p);
  } else if (k == "s") {
    ld(o, 2, str_bytes(v));
  } else if (k == "i") {
    key(o, 3, 0);
    varint(o, static_cast<uint64_t>(as_i64(v)));
  } else if (k == "f") {
    float f = static_cast<float>(PyFloat_AsDouble(v.ptr()));
    if (PyErr_Occurred()) throw py::error_already_set();
    key(o, 4, 5);
    o.append(reinterpret_cast<const char*>(&f), 4);
  } else if (k == "b") {
    key(o, 5, 0);
    varint(o, PyObject_IsTrue(v.ptr()) == 1 ? 1 : 0);
  } else if (k == "type") {
    key(o, 6, 0);
    varint(o, static_cast<uint64_t>(as_i64(v)));
  } else if (k == "shape") {
    std::string p;
    enc_shape(p, v);
    ld(o, 7, p);
  } else if (k == "tensor") {
    std::string p;
    enc_tensor(p, v);
    ld(o, 8, p);
  } else if (k == "placeholder") {
    ld(o, 9, str_bytes(v));
  } else if (k == "func") {
    std::string p;
    ld(p, 1, str_bytes(v));
    ld(o, 10, p);
  } else {
    throw Unsupported{};
  }
}

// One node as a GraphDef `node` field (field 1). `view_limit` >= 0: Consts of
// more than that many elements are written as Placeholders of the same
// dtype/shape (the light view used for shape inference, dsl.Graph._view_node).
void enc_node(std::string& out, py::handle n, int64_t view_limit) {
  Names& N = names();
  std::string name = str_bytes(get(n, N.name));
  std::string op = str_bytes(get(n, N.op));
  py::object attr = get(n, N.attr);
  if (!PyDict_Check(attr.ptr())) throw Unsupported{};
  std::string body;
  if (view_limit >= 0 && op == "Const") {
    PyObject* a = PyDict_GetItemString(attr.ptr(), "value");
    if (a) {
      py::handle av(a);
      if (str_bytes(get(av, N.kind)) == "tensor") {
        py::object t = get(av, N.value);
        std::vector<int64_t> shape;
        int64_t numel = 1;
        for (auto d : get(t, N.shape)) {
          shape.push_back(as_i64(d));
          numel *= shape.back();
        }
        if (!shape.empty() && numel > view_limit) {
          ld(body, 1, name);
          ld(body, 2, std::string("Placeholder"));
          std::string e, v;
          key(v, 6, 0);
          varint(v, static_cast<uint64_t>(as_i64(get(t, N.dtype))));
          ld(e, 1, std::string("dtype"));
          ld(e, 2, v);
          ld(body, 5, e);
          std::string sh, sv, e2;
          enc_shape_dims(sh, shape, false);
          ld(sv, 7, sh);
          ld(e2, 1, std::string("shape"));
          ld(e2, 2, sv);
          ld(body, 5, e2);
          ld(out, 1, body);
          return;
        }
      }
    }
  }
  ld(body, 1, name);
  ld(body, 2, op);
  for (auto i : get(n, N.input)) ld(body, 3, str_bytes(i));
  std::string dev = str_bytes(get(n, N.device));
  if (!dev.empty()) ld(body, 4, dev);
  std::vector<std::pair<std::string, py::handle>> attrs;
  PyObject *k, *v;
  Py_ssize_t pos = 0;
  while (PyDict_Next(attr.ptr(), &pos, &k, &v)) attrs.emplace_back(str_bytes(k), v);
  std::sort(attrs.begin(), attrs.end(), [](auto& a, auto& b) { return a.first < b.first; });
  for (auto& [an, av] : attrs) {
    std::string val, entry;
    enc_attr(val, av);
    ld(entry, 1, an);
    ld(entry, 2, val);
    ld(body, 5, entry);
  }
  ld(out, 1, body);
}

// [bytes | None] per node: None where this encoder does not cover a value
// (the caller encodes that node with graph/proto.py).
py::list encode_nodes(py::sequence nodes, int64_t view_limit) {
  py::list res;
  std::string buf;
  for (auto n : nodes) {
    buf.clear();
    try {
      enc_node(buf, n, view_limit);
      res.append(py::bytes(buf));
    } catch (const Unsupported&) {
      res.append(py::none());
    }
  }
  return res;
}

}  // namespace

void register_pyencode(py::module& m) {
  m.def("encode_nodes", &encode_nodes, py::arg("nodes"), py::arg("view_limit") = -1,
        "GraphDef `node` fields (protobuf wire format) of DSL NodeDef objects, byte-identical to "
        "graph/proto.py; None for a node holding a value this encoder does not cover.");
}

}  // namespace tfa

// Protobuf wire-format codec for the GraphDef subset (see graphdef.h).
#include "graphdef.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string_view>

namespace tfa {

int64_t max_constant_bytes() {
  static const int64_t cap = [] {
    const char* e = std::getenv("TFA_MAX_CONST_BYTES");
    return e ? std::max<int64_t>(1, std::atoll(e)) : (int64_t(1) << 36);
  }();
  return cap;
}

const char* dtype_name(DType d) {
  switch (d) {
    case DType::F32: return "float32";
    case DType::F64: return "float64";
    case DType::I32: return "int32";
    case DType::U8: return "uint8";
    case DType::I16: return "int16";
    case DType::I8: return "int8";
    case DType::STRING: return "string";
    case DType::C64: return "complex64";
    case DType::I64: return "int64";
    case DType::BOOL: return "bool";
    case DType::BF16: return "bfloat16";
    case DType::F16: return "float16";
    default: return "invalid";
  }
}

int64_t dtype_size(DType d) {
  switch (d) {
    case DType::F32: case DType::I32: return 4;
    case DType::F64: case DType::I64: case DType::C64: return 8;
    case DType::U8: case DType::I8: case DType::BOOL: return 1;
    case DType::I16: case DType::BF16: case DType::F16: return 2;
    default: return 0;
  }
}

bool dtype_is_float(DType d) {
  return d == DType::F32 || d == DType::F64 || d == DType::F16 || d == DType::BF16;
}
bool dtype_is_int(DType d) {
  return d == DType::I32 || d == DType::I64 || d == DType::I16 || d == DType::I8 || d == DType::U8;
}

std::string Shape::str() const {
  if (unknown_rank) return "<unknown>";
  std::string s = "[";
  for (size_t i = 0; i < dims.size(); ++i) {
    if (i) s += ",";
    s += dims[i] < 0 ? std::string("?") : std::to_string(dims[i]);
  }
  return s + "]";
}

double HostTensor::get_f(int64_t i) const {
  switch (dtype) {
    case DType::F32: return as<float>()[i];
    case DType::F64: return as<double>()[i];
    case DType::I32: return as<int32_t>()[i];
    case DType::I64: return static_cast<double>(as<int64_t>()[i]);
    case DType::I16: return as<int16_t>()[i];
    case DType::I8: return as<int8_t>()[i];
    case DType::U8: return as<uint8_t>()[i];
    case DType::BOOL: return as<uint8_t>()[i] ? 1.0 : 0.0;
    default: TFA_CHECK(false, "cannot read element of dtype ", dtype_name(dtype));
  }
  return 0;
}

int64_t HostTensor::get_i(int64_t i) const {
  switch (dtype) {
    case DType::I32: return as<int32_t>()[i];
    case DType::I64: return as<int64_t>()[i];
    case DType::I16: return as<int16_t>()[i];
    case DType::I8: return as<int8_t>()[i];
    case DType::U8: return as<uint8_t>()[i];
    case DType::BOOL: return as<uint8_t>()[i];
    case DType::F32: return static_cast<int64_t>(as<float>()[i]);
    case DType::F64: return static_cast<int64_t>(as<double>()[i]);
    default: TFA_CHECK(false, "cannot read element of dtype ", dtype_name(dtype));
  }
  return 0;
}

namespace {

// ---------------------------------------------------------------- reader
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const void* data, size_t n)
      : p(static_cast<const uint8_t*>(data)), end(static_cast<const uint8_t*>(data) + n) {}
  explicit Reader(std::string_view s) : Reader(s.data(), s.size()) {}
  bool done() const { return p >= end; }

  uint64_t varint() {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      TFA_CHECK(p < end, "protobuf: truncated varint");
      uint8_t b = *p++;
      v |= static_cast<uint64_t>(b & 0x7f) << shift;
      if (!(b & 0x80)) break;
      shift += 7;
      TFA_CHECK(shift < 64, "protobuf: varint too long");
    }
    return v;
  }
  uint32_t fixed32() {
    TFA_CHECK(end - p >= 4, "protobuf: truncated fixed32");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    TFA_CHECK(end - p >= 8, "protobuf: truncated fixed64");
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  // a view into the source buffer: nested messages (and weights) are not copied
  std::string_view bytes() {
    uint64_t n = varint();
    TFA_CHECK(static_cast<uint64_t>(end - p) >= n, "protobuf: truncated length-delimited field");
    std::string_view s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: fixed64(); break;
      case 2: bytes(); break;
      case 5: fixed32(); break;
      default: TFA_CHECK(false, "protobuf: unsupported wire type ", wt);
    }
  }
};

// Repeated scalar fields may arrive packed (wire type 2) or one-by-one.
template <typename F>
void read_repeated(Reader& r, int wt, F&& one) {
  if (wt == 2) {
    std::string_view payload = r.bytes();
    Reader sub(payload);
    // wire type of the elements is implied by the callback
    while (!sub.done()) one(sub, /*packed=*/true);
  } else {
    one(r, /*packed=*/false);
  }
}

Shape decode_shape(std::string_view bytes) {
  Shape s;
  Reader r(bytes);
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
    if (field == 2 && wt == 2) {
      std::string_view dim = r.bytes();
      Reader d(dim);
      int64_t size = 0;
      while (!d.done()) {
        uint64_t k = d.varint();
        int f = static_cast<int>(k >> 3), w = static_cast<int>(k & 7);
        if (f == 1 && w == 0)
          size = static_cast<int64_t>(d.varint());
        else
          d.skip(w);
      }
      TFA_CHECK(size >= -1, "TensorShapeProto: invalid dim size ", size);
      s.dims.push_back(size);
    } else if (field == 3 && wt == 0) {
      s.unknown_rank = r.varint() != 0;
    } else {
      r.skip(wt);
    }
  }
  if (s.unknown_rank) s.dims.clear();
  return s;
}

template <typename T>
void append_pod(std::vector<uint8_t>& out, T v) {
  size_t n = out.size();
  out.resize(n + sizeof(T));
  std::memcpy(out.data() + n, &v, sizeof(T));
}

HostTensor decode_tensor(std::string_view bytes) {
  HostTensor t;
  Reader r(bytes);
  std::string_view content;
  bool has_content = false;
  std::vector<uint8_t> vals;  // typed values, in the element type
  int64_t nvals = 0;
  std::vector<std::string> svals;
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
    switch (field) {
      case 1: t.dtype = static_cast<DType>(r.varint()); break;
      case 2: t.shape = decode_shape(r.bytes()); break;
      case 4: content = r.bytes(); has_content = true; break;
      case 5:  // float_val
        read_repeated(r, wt, [&](Reader& q, bool) {
          uint32_t u = q.fixed32();
          float f;
          std::memcpy(&f, &u, 4);
          append_pod(vals, f);
          ++nvals;
        });
        break;
      case 6:  // double_val
        read_repeated(r, wt, [&](Reader& q, bool) {
          uint64_t u = q.fixed64();
          double d;
          std::memcpy(&d, &u, 8);
          append_pod(vals, d);
          ++nvals;
        });
        break;
      case 7:   // int_val (int32, int16, int8, uint8)
      case 13:  // half_val (f16/bf16 bit patterns)
        read_repeated(r, wt, [&](Reader& q, bool) {
          append_pod(vals, static_cast<int64_t>(static_cast<int32_t>(q.varint())));
          ++nvals;
        });
        break;
      case 10:  // int64_val
        read_repeated(r, wt, [&](Reader& q, bool) {
          append_pod(vals, static_cast<int64_t>(q.varint()));
          ++nvals;
        });
        break;
      case 11:  // bool_val
        read_repeated(r, wt, [&](Reader& q, bool) {
          append_pod(vals, static_cast<int64_t>(q.varint() != 0));
          ++nvals;
        });
        break;
      case 8: svals.emplace_back(r.bytes()); break;
      default: r.skip(wt);
    }
  }
  TFA_CHECK(!t.shape.unknown_rank, "TensorProto with unknown rank");
  TFA_CHECK(t.shape.fully_known(), "TensorProto with unknown dims ", t.shape.str());
  // overflow-checked element count, bounded: a few bytes of typed *_val can
  // expand (fill rule) to a huge constant, so untrusted input is capped
  int64_t n = 1;
  const int64_t cap = max_constant_bytes();
  for (int64_t d : t.shape.dims) {
    TFA_CHECK(d == 0 || n <= cap / d, "TensorProto shape ", t.shape.str(), " exceeds the constant size limit (",
              cap, " bytes; TFA_MAX_CONST_BYTES)");
    n *= d;
  }
  if (t.dtype == DType::STRING) {
    TFA_CHECK(n <= cap / 32, "string TensorProto with ", n, " elements exceeds the constant size limit");
    t.strings.resize(n);
    for (int64_t i = 0; i < n; ++i)
      t.strings[i] = svals.empty() ? std::string() : svals[std::min<int64_t>(i, svals.size() - 1)];
    return t;
  }
  int64_t es = dtype_size(t.dtype);
  TFA_CHECK(es > 0, "unsupported TensorProto dtype ", static_cast<int>(t.dtype));
  TFA_CHECK(n <= cap / es, "TensorProto of ", n, " elements exceeds the constant size limit (", cap, " bytes)");
  if (has_content) {
    TFA_CHECK(static_cast<int64_t>(content.size()) == n * es, "tensor_content has ", content.size(),
              " bytes, expected ", n * es, " for shape ", t.shape.str());
    t.bytes.assign(reinterpret_cast<const uint8_t*>(content.data()),
                   reinterpret_cast<const uint8_t*>(content.data()) + content.size());
    return t;
  }
  t.bytes.assign(n * es, 0);
  if (nvals == 0) return t;  // zero-filled
  // Repeat-last-value fill rule (reference: src/main/protobuf/tensorflow/core/framework/tensor.proto:25-27).
  for (int64_t i = 0; i < n; ++i) {
    int64_t j = std::min(i, nvals - 1);
    uint8_t* dst = t.bytes.data() + i * es;
    switch (t.dtype) {
      case DType::F32: {
        float f;
        std::memcpy(&f, vals.data() + j * 4, 4);
        std::memcpy(dst, &f, 4);
        break;
      }
      case DType::F64: {
        double d;
        std::memcpy(&d, vals.data() + j * 8, 8);
        std::memcpy(dst, &d, 8);
        break;
      }
      default: {
        int64_t v;
        std::memcpy(&v, vals.data() + j * 8, 8);
        switch (es) {
          case 1: { uint8_t x = static_cast<uint8_t>(v); std::memcpy(dst, &x, 1); break; }
          case 2: { uint16_t x = static_cast<uint16_t>(v); std::memcpy(dst, &x, 2); break; }
          case 4: { int32_t x = static_cast<int32_t>(v); std::memcpy(dst, &x, 4); break; }
          case 8: std::memcpy(dst, &v, 8); break;
        }
      }
    }
  }
  return t;
}

AttrValue decode_attr(std::string_view bytes);

AttrList decode_list(std::string_view bytes) {
  AttrList l;
  Reader r(bytes);
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
    switch (field) {
      case 2: l.s.emplace_back(r.bytes()); break;
      case 3:
        read_repeated(r, wt, [&](Reader& q, bool) { l.i.push_back(static_cast<int64_t>(q.varint())); });
        break;
      case 4:
        read_repeated(r, wt, [&](Reader& q, bool) {
          uint32_t u = q.fixed32();
          float f;
          std::memcpy(&f, &u, 4);
          l.f.push_back(f);
        });
        break;
      case 5:
        read_repeated(r, wt, [&](Reader& q, bool) { l.b.push_back(q.varint() != 0); });
        break;
      case 6:
        read_repeated(r, wt, [&](Reader& q, bool) { l.type.push_back(static_cast<DType>(q.varint())); });
        break;
      case 7: l.shape.push_back(decode_shape(r.bytes())); break;
      case 8: l.tensor.push_back(decode_tensor(r.bytes())); break;
      default: r.skip(wt);
    }
  }
  return l;
}

AttrValue decode_attr(std::string_view bytes) {
  AttrValue a;
  Reader r(bytes);
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
    switch (field) {
      case 1: a.kind = AttrValue::LIST; a.list = std::make_shared<AttrList>(decode_list(r.bytes())); break;
      case 2: a.kind = AttrValue::S; a.s = r.bytes(); break;
      case 3: a.kind = AttrValue::I; a.i = static_cast<int64_t>(r.varint()); break;
      case 4: {
        a.kind = AttrValue::F;
        uint32_t u = r.fixed32();
        std::memcpy(&a.f, &u, 4);
        break;
      }
      case 5: a.kind = AttrValue::B; a.b = r.varint() != 0; break;
      case 6: a.kind = AttrValue::TYPE; a.type = static_cast<DType>(r.varint()); break;
      case 7: a.kind = AttrValue::SHAPE; a.shape = decode_shape(r.bytes()); break;
      case 8: a.kind = AttrValue::TENSOR; a.tensor = std::make_shared<HostTensor>(decode_tensor(r.bytes())); break;
      case 9: a.kind = AttrValue::PLACEHOLDER; a.s = r.bytes(); break;
      case 10: {
        a.kind = AttrValue::FUNC;
        std::string_view fn = r.bytes();
        Reader q(fn);
        while (!q.done()) {
          uint64_t k = q.varint();
          if ((k >> 3) == 1 && (k & 7) == 2) a.s = q.bytes(); else q.skip(static_cast<int>(k & 7));
        }
        break;
      }
      default: r.skip(wt);
    }
  }
  return a;
}

NodeDef decode_node(std::string_view bytes) {
  NodeDef n;
  Reader r(bytes);
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
    switch (field) {
      case 1: n.name = r.bytes(); break;
      case 2: n.op = r.bytes(); break;
      case 3: n.inputs.emplace_back(r.bytes()); break;
      case 4: n.device = r.bytes(); break;
      case 5: {
        std::string_view entry = r.bytes();
        Reader e(entry);
        std::string k;
        AttrValue v;
        while (!e.done()) {
          uint64_t kk = e.varint();
          int f = static_cast<int>(kk >> 3), w = static_cast<int>(kk & 7);
          if (f == 1) k = e.bytes();
          else if (f == 2) v = decode_attr(e.bytes());
          else e.skip(w);
        }
        n.attr[k] = std::move(v);
        break;
      }
      default: r.skip(wt);
    }
  }
  return n;
}

// ---------------------------------------------------------------- writer
struct Writer {
  std::string out;
  void varint(uint64_t v) {
    while (v >= 0x80) {
      out.push_back(static_cast<char>((v & 0x7f) | 0x80));
      v >>= 7;
    }
    out.push_back(static_cast<char>(v));
  }
  void key(int field, int wt) { varint((static_cast<uint64_t>(field) << 3) | wt); }
  void bytes_field(int field, const std::string& s) {
    key(field, 2);
    varint(s.size());
    out += s;
  }
  void varint_field(int field, uint64_t v) {
    key(field, 0);
    varint(v);
  }
};

std::string encode_shape(const Shape& s) {
  Writer w;
  if (s.unknown_rank) {
    w.varint_field(3, 1);
    return w.out;
  }
  for (auto d : s.dims) {
    Writer dim;
    dim.varint_field(1, static_cast<uint64_t>(d));
    w.bytes_field(2, dim.out);
  }
  return w.out;
}

std::string encode_tensor(const HostTensor& t) {
  Writer w;
  w.varint_field(1, static_cast<uint64_t>(t.dtype));
  w.bytes_field(2, encode_shape(t.shape));
  if (t.dtype == DType::STRING) {
    for (auto& s : t.strings) w.bytes_field(8, s);
  } else {
    w.bytes_field(4, std::string(reinterpret_cast<const char*>(t.bytes.data()), t.bytes.size()));
  }
  return w.out;
}

std::string encode_attr(const AttrValue& a) {
  Writer w;
  switch (a.kind) {
    case AttrValue::LIST: {
      Writer l;
      const AttrList& L = *a.list;
      for (auto& s : L.s) l.bytes_field(2, s);
      if (!L.i.empty()) {
        Writer p;
        for (auto v : L.i) p.varint(static_cast<uint64_t>(v));
        l.bytes_field(3, p.out);
      }
      if (!L.f.empty()) {
        std::string p(L.f.size() * 4, '\0');
        std::memcpy(&p[0], L.f.data(), p.size());
        l.bytes_field(4, p);
      }
      if (!L.b.empty()) {
        Writer p;
        for (bool v : L.b) p.varint(v ? 1 : 0);
        l.bytes_field(5, p.out);
      }
      if (!L.type.empty()) {
        Writer p;
        for (auto v : L.type) p.varint(static_cast<uint64_t>(v));
        l.bytes_field(6, p.out);
      }
      for (auto& s : L.shape) l.bytes_field(7, encode_shape(s));
      for (auto& t : L.tensor) l.bytes_field(8, encode_tensor(t));
      w.bytes_field(1, l.out);
      break;
    }
    case AttrValue::S: w.bytes_field(2, a.s); break;
    case AttrValue::I: w.varint_field(3, static_cast<uint64_t>(a.i)); break;
    case AttrValue::F: {
      w.key(4, 5);
      char buf[4];
      std::memcpy(buf, &a.f, 4);
      w.out.append(buf, 4);
      break;
    }
    case AttrValue::B: w.varint_field(5, a.b ? 1 : 0); break;
    case AttrValue::TYPE: w.varint_field(6, static_cast<uint64_t>(a.type)); break;
    case AttrValue::SHAPE: w.bytes_field(7, encode_shape(a.shape)); break;
    case AttrValue::TENSOR: w.bytes_field(8, encode_tensor(*a.tensor)); break;
    case AttrValue::PLACEHOLDER: w.bytes_field(9, a.s); break;
    case AttrValue::FUNC: {
      Writer f;
      f.bytes_field(1, a.s);
      w.bytes_field(10, f.out);
      break;
    }
    default: break;
  }
  return w.out;
}

}  // namespace

GraphDef parse_graphdef(const std::string& bytes) {
  GraphDef g;
  Reader r(bytes);
  while (!r.done()) {
    uint64_t key = r.varint();
    int field = static_cast<int>(key >> 3), wt = static_cast<int>(key & 7);
    if (field == 1 && wt == 2) {
      g.nodes.push_back(decode_node(r.bytes()));
    } else if (field == 4 && wt == 2) {
      std::string_view v = r.bytes();
      Reader q(v);
      while (!q.done()) {
        uint64_t k = q.varint();
        if ((k >> 3) == 1 && (k & 7) == 0) g.producer = static_cast<int>(q.varint());
        else q.skip(static_cast<int>(k & 7));
      }
    } else {
      r.skip(wt);
    }
  }
  return g;
}

HostTensor parse_tensor_proto(const std::string& bytes) { return decode_tensor(bytes); }
Shape parse_shape_proto(const std::string& bytes) { return decode_shape(bytes); }

std::string serialize_tensor_proto(const HostTensor& t) { return encode_tensor(t); }

std::string serialize_graphdef(const GraphDef& g) {
  Writer w;
  for (auto& n : g.nodes) {
    Writer nw;
    nw.bytes_field(1, n.name);
    nw.bytes_field(2, n.op);
    for (auto& i : n.inputs) nw.bytes_field(3, i);
    if (!n.device.empty()) nw.bytes_field(4, n.device);
    for (auto& kv : n.attr) {
      Writer e;
      e.bytes_field(1, kv.first);
      e.bytes_field(2, encode_attr(kv.second));
      nw.bytes_field(5, e.out);
    }
    w.bytes_field(1, nw.out);
  }
  if (g.producer) {
    Writer v;
    v.varint_field(1, static_cast<uint64_t>(g.producer));
    w.bytes_field(4, v.out);
  }
  return w.out;
}

}  // namespace tfa

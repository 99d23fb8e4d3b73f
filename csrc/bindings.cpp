// pybind11 module `tensorframes_amd._C`: graph import/analysis, the executor,
// pinned host memory. Replaces the Py4J + JNI bridges of the reference
// (reference: src/main/scala/org/tensorframes/impl/PythonInterface.scala:21-180).
#include <torch/extension.h>

#include <unordered_map>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>

#include "comm/comm.h"
#include "ir/graph.h"
#include "kernels/kernels.h"
#include "runtime/device_pool.h"
#include "runtime/executor.h"
#include "runtime/jit.h"
#include "runtime/jpeg_decode.h"
#include <rocprofiler-sdk-roctx/roctx.h>

namespace py = pybind11;
using namespace tfa;

namespace tfa {
void register_packer(py::module& m);  // runtime/packer.cpp
void register_pyencode(py::module& m);  // proto/pyencode.cpp
}

namespace {

py::object shape_to_py(const Shape& s) {
  if (s.unknown_rank) return py::none();
  py::list l;
  for (auto d : s.dims) l.append(d);
  return l;
}

Shape shape_from_py(const py::object& o) {
  if (o.is_none()) return Shape::unknown();
  std::vector<int64_t> d;
  for (auto v : o) d.push_back(v.is_none() ? -1 : v.cast<int64_t>());
  return Shape(d);
}

const char* row_name(RowClass r) {
  switch (r) {
    case RowClass::CONST: return "const";
    case RowClass::ROW: return "row";
    default: return "mixed";
  }
}

// {name: (dtype_enum, dims|None)} -> TensorInfo map
std::map<std::string, TensorInfo> infos_from_py(const py::dict& d) {
  std::map<std::string, TensorInfo> m;
  for (auto kv : d) {
    auto t = kv.second.cast<py::tuple>();
    TensorInfo ti;
    ti.dtype = static_cast<DType>(t[0].cast<int>());
    ti.shape = shape_from_py(t[1]);
    m[kv.first.cast<std::string>()] = ti;
  }
  return m;
}

py::list infos_to_py(const std::vector<TensorInfo>& v) {
  py::list l;
  for (auto& ti : v) {
    py::dict d;
    d["dtype"] = static_cast<int>(ti.dtype);
    d["shape"] = shape_to_py(ti.shape);
    d["row"] = row_name(ti.row);
    d["const"] = ti.value.has_value();
    l.append(d);
  }
  return l;
}

// Static inference over every node of a graph (used by the DSL for
// get_shape()). Nodes that fail inference report an error string.
py::dict infer_all(const std::string& bytes) {
  auto g = Graph::from_bytes(bytes);
  std::vector<TensorRef> all;
  for (size_t i = 0; i < g->nodes().size(); ++i) all.push_back({static_cast<int>(i), 0});
  auto order = g->closure(all);
  Graph::Infos infos = g->infer(order, {}, false);
  py::dict out;
  for (size_t i = 0; i < g->nodes().size(); ++i) out[py::str(g->node(i).name)] = infos_to_py(infos[i]);
  return out;
}

// order-preserving integer image of float keys, the host twin of
// key_image in kernels/groupby.hip: NaNs -> one canonical NaN (sorted last),
// -0.0 -> +0.0, negative values' magnitude bits flipped
template <typename F, typename S>
at::Tensor key_image_typed(const at::Tensor& keys, at::ScalarType st) {
  at::Tensor out = pool_empty({keys.size(0)}, keys.options().dtype(st));
  const F* in = keys.data_ptr<F>();
  S* o = out.data_ptr<S>();
  const S flip = std::numeric_limits<S>::max();
  for (int64_t i = 0; i < keys.size(0); ++i) {
    F v = in[i];
    if (v != v) v = std::numeric_limits<F>::quiet_NaN();
    if (v == F(0)) v = F(0);
    S b;
    std::memcpy(&b, &v, sizeof(b));
    o[i] = b < 0 ? S(b ^ flip) : b;
  }
  return out;
}

template <typename F, typename S>
at::Tensor key_from_image_typed(const at::Tensor& img, at::ScalarType st) {
  at::Tensor out = pool_empty({img.size(0)}, img.options().dtype(st));
  const S* in = img.data_ptr<S>();
  F* o = out.data_ptr<F>();
  const S flip = std::numeric_limits<S>::max();
  for (int64_t i = 0; i < img.size(0); ++i) {
    S b = in[i] < 0 ? S(in[i] ^ flip) : in[i];
    std::memcpy(&o[i], &b, sizeof(b));
  }
  return out;
}

at::Tensor host_key_image(const at::Tensor& keys) {
  return keys.scalar_type() == at::kDouble ? key_image_typed<double, int64_t>(keys, at::kLong)
                                           : key_image_typed<float, int32_t>(keys, at::kInt);
}

at::Tensor host_key_from_image(const at::Tensor& img, at::ScalarType st) {
  return st == at::kDouble ? key_from_image_typed<double, int64_t>(img, st) : key_from_image_typed<float, int32_t>(img, st);
}

}  // namespace

namespace tfa {
namespace k {
void set_conv_smallc(int on);  // kernels/conv_smallc.hip
void set_conv_direct(int on);  // kernels/conv_direct.hip
}  // namespace k
void set_pool_conv_fusion(bool on);  // runtime/executor.cpp
}  // namespace tfa

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "tensorframes_amd native runtime (GraphDef executor + HIP/CDNA4 kernels)";

  py::register_exception<GraphError>(m, "GraphError", PyExc_ValueError);
  py::register_exception<comm::CollectiveError>(m, "CollectiveError", PyExc_RuntimeError);

  py::class_<Graph, std::shared_ptr<Graph>>(m, "Graph")
      .def(py::init([](py::bytes b) { return Graph::from_bytes(std::string(b)); }))
      .def("structure_key", [](const Graph& g) { return g.structure_key(); },
           "hash of the graph without its parameter constants' payloads (Graph::structure_key)")
      .def("parameter_consts",
           [](const Graph& g) {
             std::vector<std::string> v;
             const auto& p = g.parameter_consts();
             for (size_t i = 0; i < p.size(); ++i)
               if (p[i]) v.push_back(g.node(static_cast<int>(i)).name);
             return v;
           })
      .def("node_names",
           [](const Graph& g) {
             std::vector<std::string> v;
             for (auto& n : g.nodes()) v.push_back(n.name);
             return v;
           })
      .def("node_ops",
           [](const Graph& g) {
             std::vector<std::string> v;
             for (auto& n : g.nodes()) v.push_back(n.op);
             return v;
           })
      .def("node_inputs",
           [](const Graph& g, const std::string& name) {
             int i = g.find(name);
             TFA_CHECK(i >= 0, "no node named '", name, "'");
             return g.def().nodes[i].inputs;
           })
      .def("placeholders",
           [](const Graph& g) {
             std::vector<std::string> v;
             for (int i : g.placeholders()) v.push_back(g.node(i).name);
             return v;
           })
      .def("zero_input_nodes",
           [](const Graph& g) {
             std::vector<std::string> v;
             for (auto& n : g.nodes())
               if (n.inputs.empty() && n.control.empty()) v.push_back(n.name);
             return v;
           })
      .def("has_node", [](const Graph& g, const std::string& n) { return g.find(n) >= 0; })
      .def("node_attr_scalars",
           [](const Graph& g, const std::string& name) {
             // scalar attrs (i / f / b / type / s) of one node, no tensors
             int i = g.find(name);
             TFA_CHECK(i >= 0, "no node named '", name, "'");
             py::dict d;
             for (auto& kv : g.def().nodes[i].attr) {
               const AttrValue& a = kv.second;
               switch (a.kind) {
                 case AttrValue::I: d[py::str(kv.first)] = a.i; break;
                 case AttrValue::F: d[py::str(kv.first)] = a.f; break;
                 case AttrValue::B: d[py::str(kv.first)] = a.b; break;
                 case AttrValue::TYPE: d[py::str(kv.first)] = static_cast<int>(a.type); break;
                 case AttrValue::S: d[py::str(kv.first)] = py::bytes(a.s); break;
                 default: break;
               }
             }
             return d;
           })
      .def("const_strings",
           [](const Graph& g, const std::string& name) {
             int i = g.find(name);
             TFA_CHECK(i >= 0, "no node named '", name, "'");
             const NodeDef& nd = g.def().nodes[i];
             py::list l;
             const AttrValue* v = nd.find_attr("value");
             if (nd.op == "Const" && v && v->tensor && v->tensor->dtype == DType::STRING)
               for (auto& str : v->tensor->strings) l.append(py::bytes(str));
             return l;
           })
      .def("serialize", [](const Graph& g) { return py::bytes(serialize_graphdef(g.def())); })
      .def("__len__", [](const Graph& g) { return g.nodes().size(); });

  py::class_<Program, std::shared_ptr<Program>>(m, "Program")
      .def(py::init([](std::shared_ptr<Graph> g, std::vector<std::string> fetches,
                       std::vector<std::string> feeds) {
             return std::make_shared<Program>(g, fetches, feeds);
           }),
           py::arg("graph"), py::arg("fetches"), py::arg("feeds"))
      .def_property_readonly("fetch_names", &Program::fetch_names)
      .def_property_readonly("feed_names", &Program::feed_names)
      .def("row_separable",
           [](const Program& p, py::dict hints) { return p.row_separable(infos_from_py(hints)); })
      .def("rebind", &Program::rebind, py::arg("values"), py::call_guard<py::gil_scoped_release>(),
           "a program with new parameter-constant payloads that takes over this one's plans")
      .def("adopt", &Program::adopt, py::arg("old"), py::call_guard<py::gil_scoped_release>(),
           "take over the plans of a structurally equal program (see executor.h)")
      .def("monoids",
           [](const Program& p) {
             py::list l;
             for (auto& mi : p.monoids()) l.append(py::make_tuple(mi.fetch, mi.placeholder, mi.op));
             return l;
           })
      .def("run", &Program::run, py::call_guard<py::gil_scoped_release>())
      .def("run_concurrent", &Program::run_concurrent, py::arg("inputs_list"), py::arg("max_streams") = 4,
           py::call_guard<py::gil_scoped_release>(),
           "independent runs over several input sets on one GPU, forked onto engine side streams and joined "
           "back into the caller's stream")
      .def("run_chunked", &Program::run_chunked, py::arg("seg_inputs"), py::arg("seg_outputs"),
           py::arg("chunk_rows"), py::arg("device"), py::arg("depth") = 3, py::arg("wait") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("release_pipeline", &Program::release_pipeline, py::call_guard<py::gil_scoped_release>(),
           "drain and free the persistent chunk pipeline (after a deferred run_chunked sequence)")
      .def("run_chunked_reduce", &Program::run_chunked_reduce, py::arg("seg_inputs"), py::arg("chunk_rows"),
           py::arg("device"), py::arg("depth") = 3, py::call_guard<py::gil_scoped_release>())
      .def("describe", &Program::describe_plan, py::arg("inputs"), py::arg("as_gpu") = false)
      .def("fused_sources", &Program::fused_sources)
      .def("reset_stats", &Program::reset_stats)
      .def("stats", [](const Program& p) {
        ExecStats s = p.stats();
        py::dict d;
        d["runs"] = s.runs;
        d["kernels"] = s.kernels;
        d["plans_built"] = s.plans_built;
        d["plans_adopted"] = s.plans_adopted;
        d["h2d_bytes"] = s.h2d_bytes;
        d["d2h_bytes"] = s.d2h_bytes;
        d["chunks"] = s.chunks;
        d["wall_ms"] = s.wall_ms;
        d["plan_ms"] = s.plan_ms;
        d["exec_ms"] = s.exec_ms;
        d["h2d_ms"] = s.h2d_ms;        // device time of the host->device copies (hipEvents)
        d["compute_ms"] = s.compute_ms;
        d["d2h_ms"] = s.d2h_ms;
        d["graphs_captured"] = s.graphs_captured;
        d["graph_replays"] = s.graph_replays;
        d["graph_failures"] = s.graph_failures;
        d["graphs_declined"] = s.graphs_declined;
        d["graph_busy"] = s.graph_busy;
        return d;
      });

  m.def("analyze_fetches",
        [](std::shared_ptr<Graph> g, std::vector<std::string> fetches, std::vector<std::string> feeds,
           py::dict hints) {
          Program p(g, fetches, feeds);
          Graph::Infos infos = p.analyze(infos_from_py(hints));
          py::dict out;
          // per fetch and per feed: info of output 0 (or the indexed output)
          auto info_of = [&](const std::string& f) -> py::object {
            TensorRef r = g->resolve(f);
            TFA_CHECK(r.index < static_cast<int>(infos[r.node].size()), "tensor '", f,
                      "' does not exist (node has ", infos[r.node].size(), " outputs)");
            py::list l = infos_to_py({infos[r.node][r.index]});
            return py::object(l[0]);
          };
          for (auto& f : fetches) out[py::str(f)] = info_of(f);
          for (auto& f : feeds) out[py::str(f)] = info_of(f);
          return out;
        });
  m.def("infer_fed",
        [](std::shared_ptr<Graph> g, std::vector<std::string> fetches, std::vector<std::string> feeds,
           py::dict hints) {
          // per-node infos of a program's closure under concrete feed infos
          // (the map_rows vectorizer needs every tensor's rank)
          Program p(g, fetches, feeds);
          Graph::Infos infos = p.analyze(infos_from_py(hints));
          py::dict out;
          for (size_t i = 0; i < infos.size(); ++i)
            if (!infos[i].empty()) out[py::str(g->node(static_cast<int>(i)).name)] = infos_to_py(infos[i]);
          return out;
        });
  m.def("infer_all", &infer_all);
  // A GraphDef whose Const nodes above `max_elems` elements are replaced by
  // same-typed Placeholders: structure-only views of big models for
  // Python-side graph analysis (weights never cross into Python).
  m.def("light_graphdef", [](py::bytes b, int64_t max_elems) {
    GraphDef g = parse_graphdef(std::string(b));
    for (auto& nd : g.nodes) {
      if (nd.op != "Const") continue;
      const AttrValue* v = nd.find_attr("value");
      if (!v || !v->tensor || v->tensor->num_elements() <= max_elems) continue;
      AttrValue dt;
      dt.kind = AttrValue::TYPE;
      dt.type = v->tensor->dtype;
      AttrValue shp;
      shp.kind = AttrValue::SHAPE;
      shp.shape = v->tensor->shape;
      nd.op = "Placeholder";
      nd.attr.clear();
      nd.attr["dtype"] = dt;
      nd.attr["shape"] = shp;
    }
    return py::bytes(serialize_graphdef(g));
  });
  // `orig` with every node of `patch` replacing the same-named node (or
  // appended when new): applies a Python-side rewrite of a light view back
  // onto the full graph.
  m.def("patch_graphdef", [](py::bytes orig, py::bytes patch) {
    GraphDef g = parse_graphdef(std::string(orig));
    GraphDef p = parse_graphdef(std::string(patch));
    std::unordered_map<std::string, size_t> at;
    for (size_t i = 0; i < g.nodes.size(); ++i) at[g.nodes[i].name] = i;
    for (auto& nd : p.nodes) {
      auto it = at.find(nd.name);
      if (it != at.end()) g.nodes[it->second] = nd;
      else g.nodes.push_back(nd);
    }
    return py::bytes(serialize_graphdef(g));
  });
  m.def("registered_ops", [] { return OpRegistry::get().names(); });
  // float32 MatMul/Conv2D compute mode: 0 exact f32, 1 bf16, 2 bf16x3 (kernels/gemm_bf16.hip)
  m.def("set_f32_precision", [](int mode) { k::set_f32_precision(mode); });
  // device groupBy segmentation (kernels/groupby.hip); host tensors use the ATen oracle
  m.def("factorize", [](const at::Tensor& keys0) {
    TFA_CHECK(keys0.dim() == 1, "factorize: keys must be 1-D");
    at::Tensor keys = keys0.contiguous();
    const int64_t n = keys.size(0);
    if (!keys.is_cuda()) {
      // float keys through their order image (groupby.hip): every NaN is one
      // key sorted last, -0.0 and 0.0 are one key
      const bool fl = keys.scalar_type() == at::kFloat || keys.scalar_type() == at::kDouble;
      at::Tensor img = fl ? host_key_image(keys) : keys;
      auto r = at::_unique2(img, /*sorted=*/true, /*return_inverse=*/true, /*return_counts=*/false);
      at::Tensor uniq = fl ? host_key_from_image(std::get<0>(r), keys.scalar_type()) : std::get<0>(r);
      return py::make_tuple(std::get<1>(r).to(at::kLong), uniq);
    }
    c10::hip::HIPGuard guard(keys.device().index());
    auto opts = keys.options();
    if (n == 0) return py::make_tuple(pool_empty({0}, opts.dtype(at::kLong)), pool_empty({0}, opts));
    hipStream_t s = c10::hip::getCurrentHIPStream(keys.device().index()).stream();
    const DType dt = from_scalar_type(keys.scalar_type());
    const size_t wsb = k::factorize_workspace_bytes(dt, n);
    at::Tensor ws = pool_empty({static_cast<int64_t>(wsb)}, opts.dtype(at::kByte));
    at::Tensor ids = pool_empty({n}, opts.dtype(at::kLong));
    at::Tensor uniq = pool_empty({n}, opts);
    int64_t nseg = 0;
    {
      py::gil_scoped_release nogil;
      nseg = k::factorize(dt, keys.data_ptr(), n, ids.data_ptr<int64_t>(), uniq.data_ptr(), ws.data_ptr(), wsb, s);
    }
    return py::make_tuple(ids, uniq.narrow(0, 0, nseg));
  }, "keys [n] -> (group id per row int64, distinct keys ascending)");
  m.def("string_words", [](const at::Tensor& offsets, const at::Tensor& data, int64_t W) {
    TFA_CHECK(offsets.scalar_type() == at::kLong && offsets.dim() == 1 && offsets.size(0) >= 1,
              "string_words: offsets must be int64[n+1]");
    TFA_CHECK(data.scalar_type() == at::kByte && data.dim() == 1, "string_words: data must be uint8[bytes]");
    TFA_CHECK(W >= 1 && W <= 4096, "string_words: 1..4096 words");
    TFA_CHECK(offsets.device() == data.device(), "string_words: offsets and data on different devices");
    const int64_t n = offsets.size(0) - 1;
    at::Tensor oc = offsets.contiguous(), dc = data.contiguous();
    if (!oc.is_cuda()) {  // host: the same packing, a plain loop
      at::Tensor out = at::empty({W + 1, n}, oc.options());
      const int64_t* o = oc.data_ptr<int64_t>();
      const uint8_t* d = dc.data_ptr<uint8_t>();
      int64_t* y = out.data_ptr<int64_t>();
      for (int64_t i = 0; i < n; ++i) {
        const int64_t a = o[i], len = o[i + 1] - a;
        for (int64_t w = 0; w < W; ++w) {
          uint64_t v = 0;
          for (int b = 0; b < 8; ++b) {
            const int64_t j = w * 8 + b;
            v |= static_cast<uint64_t>(j < len ? d[a + j] : 0) << (56 - 8 * b);
          }
          y[w * n + i] = static_cast<int64_t>(v ^ 0x8000000000000000ull);
        }
        y[W * n + i] = len;
      }
      return out;
    }
    c10::hip::HIPGuard guard(oc.device().index());
    at::Tensor out = pool_empty({W + 1, n}, oc.options());
    k::string_words(oc.data_ptr<int64_t>(), dc.data_ptr<uint8_t>(), n, static_cast<int>(W), out.data_ptr<int64_t>(),
                    c10::hip::getCurrentHIPStream(oc.device().index()).stream());
    return out;
  }, py::arg("offsets"), py::arg("data"), py::arg("words"),
        "string keys -> [words + 1, n] int64: big-endian 8-byte words (sign-flipped) + byte length; signed order "
        "of the columns = lexicographic order of the strings");
  m.def("string_key_hash", [](const at::Tensor& offsets, const at::Tensor& data) {
    TFA_CHECK(offsets.scalar_type() == at::kLong && offsets.dim() == 1 && offsets.size(0) >= 1,
              "string_key_hash: offsets must be int64[n+1]");
    TFA_CHECK(data.scalar_type() == at::kByte && data.dim() == 1, "string_key_hash: data must be uint8[bytes]");
    TFA_CHECK(offsets.device() == data.device(), "string_key_hash: offsets and data on different devices");
    const int64_t n = offsets.size(0) - 1;
    at::Tensor oc = offsets.contiguous(), dc = data.contiguous();
    if (!oc.is_cuda()) {
      at::Tensor out = at::empty({2, n}, oc.options());
      const int64_t* o = oc.data_ptr<int64_t>();
      const uint8_t* d = dc.data_ptr<uint8_t>();
      int64_t* y = out.data_ptr<int64_t>();
      for (int64_t i = 0; i < n; ++i) {
        const int64_t a = o[i], len = o[i + 1] - a;
        uint64_t v = 0;
        for (int b = 0; b < 8; ++b) v |= static_cast<uint64_t>(b < len ? d[a + b] : 0) << (56 - 8 * b);
        y[i] = static_cast<int64_t>(v ^ 0x8000000000000000ull);
        y[n + i] = len > 8 ? static_cast<int64_t>(k::string_key_hash_host(d + a, len) + 9) : len;
      }
      return out;
    }
    c10::hip::HIPGuard guard(oc.device().index());
    at::Tensor out = pool_empty({2, n}, oc.options());
    k::string_key_hash(oc.data_ptr<int64_t>(), dc.data_ptr<uint8_t>(), n, out.data_ptr<int64_t>(),
                   c10::hip::getCurrentHIPStream(oc.device().index()).stream());
    return out;
  }, py::arg("offsets"), py::arg("data"),
        "bounded-width string keys -> [2, n] int64: sign-flipped big-endian word 0, tag = length for keys of "
        "<= 8 bytes, else 9 + a 62-bit hash of the whole key");
  m.def("string_verify", [](const at::Tensor& offsets, const at::Tensor& data, const at::Tensor& ids,
                            const at::Tensor& rep) {
    TFA_CHECK(offsets.scalar_type() == at::kLong && ids.scalar_type() == at::kLong && rep.scalar_type() == at::kLong,
              "string_verify: int64 offsets / ids / representatives");
    const int64_t n = offsets.size(0) - 1;
    TFA_CHECK(ids.dim() == 1 && ids.size(0) == n, "string_verify: one id per string");
    TFA_CHECK(offsets.device() == data.device() && ids.device() == data.device() && rep.device() == data.device(),
              "string_verify: tensors on different devices");
    at::Tensor oc = offsets.contiguous(), dc = data.contiguous(), ic = ids.contiguous(), rc = rep.contiguous();
    if (!oc.is_cuda()) {
      const int64_t* o = oc.data_ptr<int64_t>();
      const uint8_t* d = dc.data_ptr<uint8_t>();
      const int64_t* id = ic.data_ptr<int64_t>();
      const int64_t* r = rc.data_ptr<int64_t>();
      for (int64_t i = 0; i < n; ++i) {
        const int64_t a = o[i], len = o[i + 1] - a, q = r[id[i]];
        if (len <= 8 || q == i) continue;
        if (o[q + 1] - o[q] != len || std::memcmp(d + a, d + o[q], len) != 0) return false;
      }
      return true;
    }
    c10::hip::HIPGuard guard(oc.device().index());
    hipStream_t st = c10::hip::getCurrentHIPStream(oc.device().index()).stream();
    at::Tensor flag = pool_empty({1}, oc.options().dtype(at::kInt));
    TFA_CHECK(hipMemsetAsync(flag.data_ptr(), 0, sizeof(int), st) == hipSuccess, "string_verify: memset failed");
    k::string_verify(oc.data_ptr<int64_t>(), dc.data_ptr<uint8_t>(), ic.data_ptr<int64_t>(), rc.data_ptr<int64_t>(), n,
                     flag.data_ptr<int>(), st);
    return flag.item<int>() == 0;
  }, "True when every string equals its group representative's (no hash collision)");
  m.def("gather_strings", [](const at::Tensor& offsets, const at::Tensor& data, const at::Tensor& idx) {
    // rows idx of a device string column -> (host offsets [n+1], device bytes)
    TFA_CHECK(offsets.is_cuda() && data.is_cuda() && idx.is_cuda() && offsets.scalar_type() == at::kLong &&
                  idx.scalar_type() == at::kLong && data.scalar_type() == at::kByte,
              "gather_strings: device int64 offsets / idx and uint8 data expected");
    c10::hip::HIPGuard guard(data.device().index());
    hipStream_t st = c10::hip::getCurrentHIPStream(data.device().index()).stream();
    at::Tensor oc = offsets.contiguous(), ic = idx.contiguous(), dc = data.contiguous();
    const int64_t n = ic.numel();
    at::Tensor lens = pool_empty({std::max<int64_t>(n, 1)}, oc.options());
    k::string_lens(oc.data_ptr<int64_t>(), ic.data_ptr<int64_t>(), n, lens.data_ptr<int64_t>(), st);
    at::Tensor new_offs = at::empty({n + 1}, at::TensorOptions().dtype(at::kLong));
    int64_t* no = new_offs.data_ptr<int64_t>();
    no[0] = 0;
    if (n) {
      std::vector<int64_t> lh(n);
      TFA_CHECK(hipMemcpyAsync(lh.data(), lens.data_ptr(), n * sizeof(int64_t), hipMemcpyDeviceToHost, st) == hipSuccess &&
                    hipStreamSynchronize(st) == hipSuccess, "gather_strings: length copy failed");
      for (int64_t g = 0; g < n; ++g) no[g + 1] = no[g] + lh[g];
    }
    at::Tensor out = pool_empty({std::max<int64_t>(no[n], 1)}, dc.options());
    if (n) {
      at::Tensor dno = pool_empty({n + 1}, oc.options());
      TFA_CHECK(hipMemcpyAsync(dno.data_ptr(), no, (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st) == hipSuccess,
                "gather_strings: offset copy failed");
      k::gather_bytes(dc.data_ptr<uint8_t>(), oc.data_ptr<int64_t>(), ic.data_ptr<int64_t>(), dno.data_ptr<int64_t>(), n,
                      out.data_ptr<uint8_t>(), st);
      TFA_CHECK(hipStreamSynchronize(st) == hipSuccess, "gather_strings: gather failed");  // `no` is pageable
    }
    return py::make_tuple(new_offs, out.narrow(0, 0, no[n]));
  }, "rows idx of a device string column -> (host int64 offsets [n+1], device uint8 bytes)");
  m.def("key_dest", [](const std::vector<at::Tensor>& keys, int64_t world) {
    TFA_CHECK(!keys.empty() && keys[0].is_cuda(), "key_dest: device key columns expected");
    c10::hip::HIPGuard guard(keys[0].device().index());
    const int64_t n = keys[0].size(0);
    hipStream_t s = c10::hip::getCurrentHIPStream(keys[0].device().index()).stream();
    at::Tensor h = pool_empty({n}, keys[0].options().dtype(at::kLong));
    for (size_t i = 0; i < keys.size(); ++i) {
      at::Tensor kc = keys[i].contiguous();
      TFA_CHECK(kc.dim() == 1 && kc.size(0) == n, "key_dest: key columns must be 1-D of equal length");
      k::key_hash(from_scalar_type(kc.scalar_type()), kc.data_ptr(), n,
                  reinterpret_cast<uint64_t*>(h.data_ptr<int64_t>()), i > 0, s);
    }
    at::Tensor dest = pool_empty({n}, h.options());
    k::hash_mod(reinterpret_cast<const uint64_t*>(h.data_ptr<int64_t>()), n, world, dest.data_ptr<int64_t>(), s);
    return dest;
  }, "destination rank of every row: hash(keys) % world (same on every rank)");
  m.def("group_representatives", [](const at::Tensor& ids, int64_t nseg) {
    TFA_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.dim() == 1, "group_representatives: device int64 ids");
    c10::hip::HIPGuard guard(ids.device().index());
    at::Tensor rep = pool_empty({nseg}, ids.options());
    k::group_representatives(ids.contiguous().data_ptr<int64_t>(), ids.size(0), rep.data_ptr<int64_t>(),
                             c10::hip::getCurrentHIPStream(ids.device().index()).stream());
    return rep;
  }, "one row index per group (device)");
  m.def("partition_rows", [](const at::Tensor& dest0, int64_t world) {
    TFA_CHECK(dest0.is_cuda() && dest0.scalar_type() == at::kLong && dest0.dim() == 1, "partition_rows: device int64 dest");
    c10::hip::HIPGuard guard(dest0.device().index());
    at::Tensor dest = dest0.contiguous();
    const int64_t n = dest.size(0);
    hipStream_t s = c10::hip::getCurrentHIPStream(dest.device().index()).stream();
    const size_t wsb = k::partition_workspace_bytes(n);
    at::Tensor ws = pool_empty({static_cast<int64_t>(wsb)}, dest.options().dtype(at::kByte));
    at::Tensor perm = pool_empty({n}, dest.options());
    at::Tensor counts = pool_empty({world}, dest.options());
    k::partition_rows(dest.data_ptr<int64_t>(), n, world, perm.data_ptr<int64_t>(), counts.data_ptr<int64_t>(),
                      ws.data_ptr(), wsb, s);
    return py::make_tuple(perm, counts);
  }, "rows ordered by destination rank (stable) + rows per destination (device)");
  m.def("segment_csr", [](const at::Tensor& ids0, int64_t nseg) {
    TFA_CHECK(ids0.is_cuda() && ids0.dim() == 1 && (ids0.scalar_type() == at::kLong || ids0.scalar_type() == at::kInt),
              "segment_csr: device int ids");
    c10::hip::HIPGuard guard(ids0.device().index());
    at::Tensor ids = ids0.contiguous();
    const int64_t n = ids.size(0);
    hipStream_t s = c10::hip::getCurrentHIPStream(ids.device().index()).stream();
    at::Tensor perm = pool_empty({n}, ids.options().dtype(at::kLong));
    at::Tensor off = pool_empty({nseg + 1}, ids.options().dtype(at::kLong));
    const size_t wsb = k::segment_csr_workspace_bytes(n, nseg);
    at::Tensor ws = pool_empty({static_cast<int64_t>(wsb)}, ids.options().dtype(at::kByte));
    k::segment_csr(from_scalar_type(ids.scalar_type()), ids.data_ptr(), n, nseg, perm.data_ptr<int64_t>(),
                   off.data_ptr<int64_t>(), ws.data_ptr(), wsb, s);
    return py::make_tuple(perm, off);
  }, "ids [n] in [0, nseg) -> (rows ordered by segment, stable; CSR offsets [nseg + 1]) on the device");
  m.def("segment_rows", [](const at::Tensor& perm, const at::Tensor& offs, int64_t size) {
    TFA_CHECK(perm.is_cuda() && offs.is_cuda() && perm.scalar_type() == at::kLong && offs.scalar_type() == at::kLong,
              "segment_rows: device int64 tensors");
    c10::hip::HIPGuard guard(perm.device().index());
    const int64_t G = offs.size(0);
    at::Tensor idx = pool_empty({G * size}, perm.options());
    k::segment_rows(perm.contiguous().data_ptr<int64_t>(), offs.contiguous().data_ptr<int64_t>(), G, size,
                    idx.data_ptr<int64_t>(), c10::hip::getCurrentHIPStream(perm.device().index()).stream());
    return idx;
  }, "row ids of G equal-size segments: perm[offs[g] + j] for j < size -> [G * size]");
  m.def("scatter_rows", [](at::Tensor dst, const at::Tensor& idx, const at::Tensor& src0) {
    TFA_CHECK(dst.is_cuda() && idx.is_cuda() && src0.is_cuda() && idx.scalar_type() == at::kLong,
              "scatter_rows: device tensors");
    TFA_CHECK(dst.is_contiguous() && dst.dim() >= 1 && src0.scalar_type() == dst.scalar_type(),
              "scatter_rows: contiguous dst of the source dtype");
    c10::hip::HIPGuard guard(dst.device().index());
    at::Tensor src = src0.contiguous();
    TFA_CHECK(src.size(0) == idx.size(0), "scatter_rows: one index per source row");
    const int64_t row = dst.size(0) ? dst.numel() / dst.size(0) : 0;
    TFA_CHECK(src.numel() == idx.size(0) * row, "scatter_rows: source rows must match the destination row shape");
    k::scatter_rows(row * dst.element_size(), src.data_ptr(), idx.contiguous().data_ptr<int64_t>(), dst.data_ptr(),
                    idx.size(0), c10::hip::getCurrentHIPStream(dst.device().index()).stream());
    return dst;
  }, "dst[idx[j]] = src[j] along dim 0 (device scatter kernel), in place");
  // one record per row holding every column (the keyed shuffle's single
  // all-to-all payload): column c at byte offset offs[c] of R-byte records
  m.def("pack_rows", [](const std::vector<at::Tensor>& cols, std::optional<at::Tensor> perm) {
    TFA_CHECK(!cols.empty() && cols.size() <= static_cast<size_t>(k::kMaxPackCols), "pack_rows: 1..16 columns");
    const int64_t n = perm ? perm->size(0) : cols[0].size(0);
    k::PackCols pc;
    pc.n = static_cast<int>(cols.size());
    std::vector<at::Tensor> keep;
    int64_t R = 0;
    for (size_t c = 0; c < cols.size(); ++c) {
      at::Tensor t = cols[c].contiguous();
      TFA_CHECK(t.is_cuda() && t.dim() >= 1 && t.device() == cols[0].device(), "pack_rows: device columns");
      TFA_CHECK(perm || t.size(0) == n, "pack_rows: columns disagree on rows");
      const int64_t rb = t.size(0) ? t.numel() / t.size(0) * t.element_size() : 0;
      pc.row_bytes[c] = rb;
      pc.off[c] = R;
      pc.ptr[c] = t.data_ptr();
      R += (rb + 3) / 4 * 4;
      keep.push_back(t);
    }
    c10::hip::HIPGuard guard(cols[0].device().index());
    at::Tensor out = pool_empty({n, R}, cols[0].options().dtype(at::kByte));
    const int64_t* pp = nullptr;
    at::Tensor pc_t;
    if (perm) {
      pc_t = perm->contiguous();
      TFA_CHECK(pc_t.is_cuda() && pc_t.scalar_type() == at::kLong, "pack_rows: device int64 perm");
      pp = pc_t.data_ptr<int64_t>();
    }
    k::pack_rows(pc, pp, n, R, out.data_ptr(), c10::hip::getCurrentHIPStream(cols[0].device().index()).stream());
    std::vector<int64_t> offs(pc.off, pc.off + pc.n);
    return py::make_tuple(out, offs);
  }, py::arg("cols"), py::arg("perm") = py::none(),
     "device columns -> (uint8 records [n, R] in perm order, byte offset of each column)");
  m.def("unpack_rows", [](const at::Tensor& rec, const std::vector<at::Tensor>& outs) {
    TFA_CHECK(rec.is_cuda() && rec.dim() == 2 && rec.scalar_type() == at::kByte, "unpack_rows: device uint8 records");
    TFA_CHECK(!outs.empty() && outs.size() <= static_cast<size_t>(k::kMaxPackCols), "unpack_rows: 1..16 columns");
    const int64_t n = rec.size(0);
    k::PackCols pc;
    pc.n = static_cast<int>(outs.size());
    int64_t R = 0;
    for (size_t c = 0; c < outs.size(); ++c) {
      const at::Tensor& t = outs[c];
      TFA_CHECK(t.is_cuda() && t.is_contiguous() && t.size(0) == n, "unpack_rows: contiguous device outputs of n rows");
      const int64_t rb = n ? t.numel() / n * t.element_size() : 0;
      pc.row_bytes[c] = rb;
      pc.off[c] = R;
      pc.ptr[c] = t.data_ptr();
      R += (rb + 3) / 4 * 4;
    }
    TFA_CHECK(R == rec.size(1), "unpack_rows: record width ", rec.size(1), " does not match the columns (", R, ")");
    c10::hip::HIPGuard guard(rec.device().index());
    k::unpack_rows(pc, rec.contiguous().data_ptr(), n, R, c10::hip::getCurrentHIPStream(rec.device().index()).stream());
  }, "records [n, R] -> the preallocated device columns (same layout as pack_rows)");
  // native JPEG decode into one ragged (pinned) buffer (runtime/jpeg_decode.cpp)
  struct PyJpegBatch {
    std::vector<py::buffer_info> views;  // keep the cells' buffers exported while decoding
    std::unique_ptr<tfa::JpegBatch> job;
    ~PyJpegBatch() { job.reset(); }  // waits for the tasks before the views go
  };
  py::class_<PyJpegBatch>(m, "JpegBatch")
      .def(py::init([](const py::list& cells, int channels, int threads, bool pinned) {
             TFA_CHECK(channels == 1 || channels == 3, "JpegBatch: channels must be 1 or 3");
             auto b = std::make_unique<PyJpegBatch>();
             std::vector<std::pair<const uint8_t*, size_t>> ptrs;
             b->views.reserve(cells.size());
             for (auto c : cells) {
               b->views.push_back(py::reinterpret_borrow<py::buffer>(c).request());
               const auto& v = b->views.back();
               ptrs.emplace_back(static_cast<const uint8_t*>(v.ptr), static_cast<size_t>(v.size * v.itemsize));
             }
             b->job = std::make_unique<tfa::JpegBatch>(std::move(ptrs), channels, threads, pinned);
             return b;
           }),
           py::arg("cells"), py::arg("channels"), py::arg("threads"), py::arg("pinned") = true)
      .def_property_readonly("header_ok", [](const PyJpegBatch& b) { return b.job->header_ok(); })
      .def_property_readonly("bad_header", [](const PyJpegBatch& b) { return b.job->bad_header(); })
      .def("wait", [](PyJpegBatch& b) {
        py::gil_scoped_release nogil;
        return b.job->wait();
      }, "block until every image is decoded; returns the indices that failed")
      .def_property_readonly("buffer", [](const PyJpegBatch& b) { return b.job->buffer(); })
      .def_property_readonly("meta_bytes", [](const PyJpegBatch& b) { return b.job->meta_bytes(); })
      .def_property_readonly("offsets_bytes", [](const PyJpegBatch& b) { return b.job->offsets_bytes(); })
      .def("shape", [](const PyJpegBatch& b, int64_t i) { return b.job->shape(i); })
      .def("pixel_offset", [](const PyJpegBatch& b, int64_t i) { return b.job->pixel_offset(i); });
  m.def("jpeg_native_available", [] {
    std::string why;
    bool ok = tfa::jpeg_native_available(&why);
    return py::make_tuple(ok, why);
  });
  m.def("set_step_timing", &tfa::set_step_timing, py::arg("on"),
        "time every step of GPU plan runs (a hipEvent pair each) until turned off");
  m.def("read_step_timing", [] {
    py::list out;
    for (const auto& r : tfa::read_step_timing()) {
      py::dict d;
      d["node"] = r.node;
      d["op"] = r.op;
      d["label"] = r.label;
      d["flops"] = r.flops;
      d["bytes"] = r.bytes;
      d["ms"] = r.ms;
      out.append(d);
    }
    return out;
  }, "wait for and drain the step records: [{node, op, label, flops, ms}] in launch order");
  m.def("roctx_push", [](const std::string& name) { roctxRangePushA(name.c_str()); }, py::arg("name"),
        "open a roctx range (rocprofv3 --marker-trace)");
  m.def("roctx_pop", [] { roctxRangePop(); });
  m.def("jpeg_native_info", [] {
    tfa::JpegLibInfo i = tfa::jpeg_native_info();
    py::dict d;
    d["ok"] = i.ok;
    d["version"] = i.version;
    d["struct_size"] = i.struct_size;
    d["soname"] = i.soname;
    d["why"] = i.why;
    return d;
  }, "the loaded libjpeg: its own version and decompressor size, and whether that layout is a known one");
  m.def("jpeg_force_version", &tfa::jpeg_force_version, py::arg("version"),
        "tests: treat the loaded libjpeg as this version (0 = its real one); unknown layouts disable the native path");
  m.def("jpeg_decode", [](const py::buffer& data, int channels) {
    auto v = data.request();
    tfa::JpegHeader h;
    const auto* p = static_cast<const uint8_t*>(v.ptr);
    size_t n = static_cast<size_t>(v.size * v.itemsize);
    TFA_CHECK(tfa::jpeg_parse_header(p, n, &h), "jpeg_decode: not a supported JPEG");
    at::Tensor out = at::empty({h.height, h.width, channels}, at::kByte);
    std::string err;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = tfa::jpeg_decode_into(p, n, channels, out.data_ptr<uint8_t>(), out.numel(), &err);
    }
    TFA_CHECK(ok, "jpeg_decode: ", err);
    return out;
  }, py::arg("data"), py::arg("channels") = 3, "decode one JPEG on the calling thread (tests, tools)");
  m.def("decode_pool_threads", &tfa::decode_pool_threads);
  m.def("ragged_image_prep", [](const at::Tensor& data, const at::Tensor& offs, const at::Tensor& hw, int C, int OH,
                                 int OW, int mode, int oy, int ox, int h, int w,
                                 const std::vector<std::pair<int, std::vector<float>>>& ops,
                                 std::optional<at::Tensor> row_params) {
    // the batched map_rows image pre-stage (kernels/image.hip ragged_prep_kernel)
    TFA_CHECK(data.is_cuda() && data.scalar_type() == at::kByte && data.dim() == 1 && data.is_contiguous(),
              "ragged_image_prep: data must be a contiguous uint8 device buffer");
    const int64_t n = offs.numel();
    TFA_CHECK(offs.is_cuda() && offs.scalar_type() == at::kLong && offs.is_contiguous() && hw.is_cuda() &&
                  hw.scalar_type() == at::kInt && hw.is_contiguous() && hw.numel() == 2 * n,
              "ragged_image_prep: offsets int64 [n] and hw int32 [n, 2] device tensors expected");
    TFA_CHECK(ops.size() <= 4, "ragged_image_prep: at most 4 elementwise steps");
    k::RaggedPrepArgs a;
    a.n = n; a.C = C; a.OH = OH; a.OW = OW; a.mode = mode; a.oy = oy; a.ox = ox; a.h = h; a.w = w;
    a.nops = static_cast<int>(ops.size());
    for (size_t q = 0; q < ops.size(); ++q) {
      TFA_CHECK(ops[q].first >= 0 && ops[q].first <= 3,
                "ragged_image_prep: step kind must be 0 add, 1 sub, 2 mul, 3 div");
      const auto& v = ops[q].second;
      TFA_CHECK(v.size() == 1 || static_cast<int>(v.size()) == C, "ragged_image_prep: step constant of ", v.size(),
                " values for ", C, " channels");
      a.op_kind[q] = ops[q].first;
      a.op_chan[q] = v.size() > 1;
      for (size_t c = 0; c < v.size(); ++c) a.op_val[q][c] = v[c];
    }
    c10::hip::HIPGuard guard(data.device().index());
    at::Tensor rp;
    if (row_params) {
      // per-row (OH, OW, oy, ox): checked here on the host copy (the kernel
      // trusts them), then copied to the device on the stream
      const at::Tensor& hp = *row_params;
      TFA_CHECK(!hp.is_cuda() && hp.scalar_type() == at::kInt && hp.is_contiguous() && hp.numel() == 4 * n,
                "ragged_image_prep: row_params must be a host int32 [n, 4] tensor");
      const int32_t* p = hp.data_ptr<int32_t>();
      for (int64_t r = 0; r < n; ++r) {
        const int32_t RH = p[4 * r], RW = p[4 * r + 1], py = p[4 * r + 2], px = p[4 * r + 3];
        TFA_CHECK(RH > 0 && RW > 0 && py >= 0 && px >= 0 && py + h <= RH && px + w <= RW, "ragged_image_prep: row ",
                  r, ": crop ", h, "x", w, " at (", py, ", ", px, ") outside its ", RH, "x", RW, " resize");
      }
      rp = pool_empty({n, 4}, data.options().dtype(at::kInt));
      rp.copy_(hp, /*non_blocking=*/hp.is_pinned());
      a.rp = rp.data_ptr<int32_t>();
    }
    at::Tensor y = pool_empty({n, h, w, C}, data.options().dtype(at::kFloat));
    a.x = data.data_ptr<uint8_t>();
    a.offs = offs.data_ptr<int64_t>();
    a.hw = hw.data_ptr<int32_t>();
    a.y = y.data_ptr<float>();
    k::ragged_image_prep(a, c10::hip::getCurrentHIPStream(data.device().index()).stream());
    return y;
  }, py::arg("data"), py::arg("offsets"), py::arg("hw"), py::arg("channels"), py::arg("resize_h"),
        py::arg("resize_w"), py::arg("mode"), py::arg("crop_y"), py::arg("crop_x"), py::arg("crop_h"),
        py::arg("crop_w"), py::arg("ops"), py::arg("row_params") = py::none(),
        "n ragged uint8 HWC images -> f32 [n, crop_h, crop_w, C]: bilinear resize, crop, elementwise steps");
  m.def("gather_rows", [](const at::Tensor& x0, const at::Tensor& idx) {
    TFA_CHECK(x0.is_cuda() && idx.is_cuda() && idx.scalar_type() == at::kLong, "gather_rows: device tensors");
    c10::hip::HIPGuard guard(x0.device().index());
    at::Tensor x = x0.contiguous();
    auto sizes = x.sizes().vec();
    sizes[0] = idx.size(0);
    at::Tensor out = pool_empty(sizes, x.options());
    const int64_t inner = x.size(0) ? x.numel() / x.size(0) : 0;
    if (out.numel())
      k::gather(x.element_size(), DType::I64, x.data_ptr(), idx.contiguous().data_ptr(), out.data_ptr(), 1, x.size(0),
                idx.size(0), inner, c10::hip::getCurrentHIPStream(x.device().index()).stream());
    return out;
  }, "out[j] = x[idx[j]] along dim 0 (device gather kernel)");
  register_packer(m);
  register_pyencode(m);
  m.def("jit_compile", [](const std::string& src) { return jit::compile_only(src); },
        "compile a generated kernel with hiprtc for gfx950 (no device needed); returns the code-object size");
  m.def("jit_stats", []() {
    auto s = jit::stats();
    py::dict d;
    d["compiled"] = s.compiled;
    d["disk_hits"] = s.disk_hits;
    d["memory_hits"] = s.memory_hits;
    d["compile_ms"] = s.compile_ms;
    return d;
  });
  m.def("set_debug_sync", &set_debug_sync, "synchronise + check after every kernel (read per launch)");
  m.def("get_debug_sync", &get_debug_sync);
  m.def("f32_precision", [] { return k::f32_precision(); });
  m.def("set_gemm_tile", [](int cfg) { k::set_gemm_tile(cfg); });
  m.def("set_conv_smallc", [](bool on) { k::set_conv_smallc(on ? 1 : 0); },
        "route tiny-reduction convs (KH*KW*C <= 32) to the direct kernel (default on)");
  m.def("set_pool_conv_fusion", [](bool on) { tfa::set_pool_conv_fusion(on); }, py::arg("on"),
        "fuse a 3x3 VALID MaxPool into the 1x1 conv that alone reads it (GPU plans made after the call; default on)");
  m.def("set_conv_direct", [](bool on) { k::set_conv_direct(on ? 1 : 0); },
        "route narrow wide-image convs (C in {32, 64}, OC <= 64) to the direct LDS-filter kernel (default on)");
  m.def("set_conv_wino", [](bool on) { k::set_conv_wino(on ? 1 : 0); },
        "Winograd F(2x2,3x3) / F(2,7) for 3x3 / 1x7 / 7x1 stride-1 convs with constant filters (default on; TFA_CONV_ALGO=direct "
        "turns it off). Plans built while it is off carry no Winograd filters.");
  m.def("conv_wino_enabled", [] { return k::conv_wino_enabled(); });
  m.def("set_wino_5x5", [](bool on) { k::set_wino_5x5(on ? 1 : 0); }, py::arg("on"),
        "Winograd F(4,5) for 5x5 stride-1 convs in plans made after the call (opt-in)");
  m.def("set_wino_bn", &tfa::k::set_wino_bn, py::arg("bn"), "F(2x2,3x3) oc block: 0 auto (32 for OC <= 32), 32 or 64");
  m.def("set_wino_tile", [](int v) { k::set_wino_tile(v); },
        "force the Winograd kernel variant: -1 auto, 0 = 64 tiles x 64 oc, 1 = 128 tiles x 32 oc");
  m.def("conv_wino_filter", [](const at::Tensor& w) {
          TFA_CHECK(w.dim() == 4 && w.scalar_type() == at::kFloat, "conv_wino_filter: HWIO float32 filter");
          const int kind = k::conv_wino_kind(w.size(0), w.size(1), 1, 1, 1, 1, w.size(2), w.size(3));
          TFA_CHECK(kind != 0, "conv_wino_filter: 3x3, 1x7, 7x1 or 5x5 with C % 8 == 0 and OC % 4 == 0");
          at::Tensor wc = w.cpu().contiguous();
          at::Tensor u = at::empty({k::conv_wino_filter_elems(kind, wc.size(2), wc.size(3))}, wc.options());
          k::conv_wino_filter(kind, wc.data_ptr<float>(), wc.size(2), wc.size(3), u.data_ptr<float>());
          return u;
        }, "the planner's Winograd filter transform (fp64): 3x3 -> [C/8][16][2][OCP][4], 1x7 / 7x1 -> "
           "[C/8][8][2][OCP][4], flattened (tests)");
  m.def("gemm_tile_count", [] { return k::gemm_tile_count(); });
  m.def("gemm_tune_table", &k::gemm_tune_table, "the autotuner's tile picks: [(20-field shape key, tile)]");
  m.def("gemm_tune_seed", &k::gemm_tune_seed, py::arg("key"), py::arg("tile"),
        "a shipped default tile for a shape key (replaced only by a >= 2 % win confirmed twice)");
  m.def("gemm_tune_reset", &k::gemm_tune_reset, "forget the autotuner's picks (the defaults stay)");
  m.def("gemm_tile_dims", &k::gemm_tile_dims, py::arg("tile"), "{BM, BN, core}");
  m.def("roundtrip_graphdef",
        [](py::bytes b) { return py::bytes(serialize_graphdef(parse_graphdef(std::string(b)))); });
  m.def("decode_tensor_proto", [](py::bytes b) {
    HostTensor t = parse_tensor_proto(std::string(b));
    if (t.dtype == DType::STRING) {
      py::list l;
      for (auto& s : t.strings) l.append(py::bytes(s));
      return py::object(l);
    }
    return py::cast(host_tensor_to_at(t));
  });
  // Segmented reduction over rows sorted by segment (CSR offsets, int64):
  // the groupBy/aggregate monoid fast path. Device tensors run the HIP
  // kernel; host tensors the ATen reference.
  // Unsorted segmented reduction: out[ids[i]] op= x[i] (rows in any order),
  // the map-side combine of groupBy/aggregate. ids int32/int64 on x's device.
  m.def("unsorted_segment_reduce", [](const std::string& op, const at::Tensor& x, const at::Tensor& ids,
                                      int64_t nseg, std::optional<at::Tensor> out_opt) {
    TFA_CHECK(x.dim() >= 1 && ids.dim() == 1 && ids.size(0) == x.size(0), "unsorted_segment_reduce: ids must be [rows]");
    TFA_CHECK(ids.scalar_type() == at::kLong || ids.scalar_type() == at::kInt, "unsorted_segment_reduce: int ids");
    TFA_CHECK(ids.device() == x.device(), "unsorted_segment_reduce: ids and x on different devices");
    k::RedOp rop = op == "Sum" ? k::RedOp::SUM : op == "Min" ? k::RedOp::MIN : op == "Max" ? k::RedOp::MAX
                 : op == "Prod" ? k::RedOp::PROD : k::RedOp::ALL;
    TFA_CHECK(rop != k::RedOp::ALL, "unsorted_segment_reduce: unsupported op ", op);
    std::vector<int64_t> osz = x.sizes().vec();
    osz[0] = nseg;
    const int64_t nrows = x.size(0);
    if (!x.is_cuda()) {
      at::Tensor xs = x.reshape({nrows, -1});
      at::Tensor is = ids.to(at::kLong);
      at::Tensor out;
      if (rop == k::RedOp::SUM) {
        out = at::zeros({nseg, xs.size(1)}, x.options()).index_add_(0, is, xs);
      } else if (rop == k::RedOp::PROD) {
        out = at::ones({nseg, xs.size(1)}, x.options()).index_reduce_(0, is, xs, "prod", true);
      } else {
        const bool mx = rop == k::RedOp::MAX;
        out = at::empty({nseg, xs.size(1)}, x.options());
        out = out.index_reduce_(0, is, xs, mx ? "amax" : "amin", false);
      }
      out = out.reshape(osz).contiguous();
      if (out_opt) return out_opt->copy_(out);
      return out;
    }
    c10::hip::HIPGuard guard(x.device().index());
    at::Tensor xc = x.contiguous(), ic = ids.contiguous();
    at::Tensor out;
    if (out_opt) {  // write into a caller's slice (e.g. one partition's row of a stacked buffer)
      out = *out_opt;
      TFA_CHECK(out.is_cuda() && out.is_contiguous() && out.sizes().vec() == osz && out.scalar_type() == xc.scalar_type(),
                "unsorted_segment_reduce: out must be a contiguous device tensor of the result shape and dtype");
    } else {
      out = pool_empty(osz, xc.options());
    }
    if (!out.numel()) return out;
    const int64_t inner = out.numel() / nseg;
    const DType dt = from_scalar_type(xc.scalar_type());
    size_t ws = k::unsorted_segment_workspace_bytes(rop, dt, nrows, inner, nseg);
    at::Tensor work;
    if (ws) work = pool_empty({static_cast<int64_t>(ws)}, xc.options().dtype(at::kByte));
    k::unsorted_segment_reduce(rop, dt, from_scalar_type(ic.scalar_type()), xc.data_ptr(), ic.data_ptr(),
                               out.data_ptr(), nrows, inner, nseg, ws ? work.data_ptr() : nullptr,
                               c10::hip::getCurrentHIPStream(x.device().index()).stream());
    return out;
  }, py::arg("op"), py::arg("x"), py::arg("ids"), py::arg("nseg"), py::arg("out") = py::none());
  m.def("segment_reduce", [](const std::string& op, const at::Tensor& x, const at::Tensor& offsets) {
    TFA_CHECK(x.dim() >= 1, "segment_reduce needs rank >= 1");
    TFA_CHECK(offsets.scalar_type() == at::kLong && offsets.dim() == 1, "offsets must be int64[nseg+1]");
    int64_t nseg = offsets.size(0) - 1;
    std::vector<int64_t> osz = x.sizes().vec();
    osz[0] = nseg;
    k::RedOp rop = op == "Sum" ? k::RedOp::SUM : op == "Min" ? k::RedOp::MIN : op == "Max" ? k::RedOp::MAX
                 : op == "Prod" ? k::RedOp::PROD : op == "Mean" ? k::RedOp::MEAN : k::RedOp::ALL;
    TFA_CHECK(rop != k::RedOp::ALL, "segment_reduce: unsupported op ", op);
    if (!x.is_cuda()) {
      at::Tensor off = offsets.to(at::kCPU);
      const int64_t* o = off.data_ptr<int64_t>();
      std::vector<at::Tensor> parts;
      for (int64_t s = 0; s < nseg; ++s) {
        at::Tensor seg = x.narrow(0, o[s], o[s + 1] - o[s]);
        switch (rop) {
          case k::RedOp::SUM: parts.push_back(seg.sum(0, false, x.scalar_type())); break;
          case k::RedOp::MIN: parts.push_back(std::get<0>(seg.min(0))); break;
          case k::RedOp::MAX: parts.push_back(std::get<0>(seg.max(0))); break;
          case k::RedOp::PROD: parts.push_back(seg.prod(0, false, x.scalar_type())); break;
          default: parts.push_back(seg.to(at::kDouble).mean(0).to(x.scalar_type()));
        }
      }
      return nseg ? at::stack(parts, 0) : at::empty(osz, x.options());
    }
    c10::hip::HIPGuard guard(x.device().index());
    at::Tensor xc = x.contiguous();
    at::Tensor out = pool_empty(osz, xc.options());
    int64_t inner = nseg ? out.numel() / nseg : 0;
    if (out.numel())
      k::segment_reduce_csr(rop, from_scalar_type(xc.scalar_type()), xc.data_ptr(),
                            offsets.contiguous().data_ptr<int64_t>(), out.data_ptr(), nseg, inner,
                            c10::hip::getCurrentHIPStream(x.device().index()).stream());
    return out;
  });
  m.def("empty_pinned", &empty_pinned);
  m.def("trim_pinned_pool", &trim_pinned_pool);
  m.def("is_pinned", [](const at::Tensor& t) {
    // torch's is_pinned() only knows its own host allocator; ask HIP directly
    if (t.is_cuda() || !t.numel()) return false;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, t.data_ptr()) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return attr.type == hipMemoryTypeHost;
  });
  m.def("pinned_pool_cached_bytes", &pinned_pool_cached_bytes);
  m.def("device_pool_stats", [] {
    DevPoolStats v = dev_pool_stats();
    py::dict d;
    d["allocs"] = v.allocs;
    d["frees"] = v.frees;
    d["fallbacks"] = v.fallbacks;
    d["capture_allocs"] = v.capture_allocs;
    d["device_mallocs"] = v.device_mallocs;
    d["live"] = v.live_bytes;
    d["peak"] = v.peak_bytes;
    d["cached"] = v.cached_bytes;
    return d;
  }, "engine-owned device pool: allocations, frees, c10 fallbacks, HIP-graph capture allocations, hipMallocs, live / peak / cached bytes");
  m.def("trim_device_pool", &dev_pool_trim);
  // ---- engine-owned communicators (csrc/comm/comm.h)
  {
    using comm::Comm;
    using GR = py::call_guard<py::gil_scoped_release>;
    py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm",
        "engine communicator: all_reduce / all_gather / all_to_all_v / broadcast on the current stream")
        .def_property_readonly("rank", &Comm::rank)
        .def_property_readonly("size", &Comm::size)
        .def_property_readonly("kind", &Comm::kind)
        .def_property_readonly("calls", &Comm::calls)
        .def("all_reduce", [](Comm& c, at::Tensor t, const std::string& op) {
          c.all_reduce(t, comm::parse_op(op));
          return t;
        }, py::arg("tensor"), py::arg("op") = "Sum", GR())
        .def("all_gather", &Comm::all_gather, GR())
        .def("all_to_all_v", &Comm::all_to_all_v, py::arg("x"), py::arg("send_rows"), py::arg("recv_rows"), GR())
        .def("broadcast", [](Comm& c, at::Tensor t, int root) {
          c.broadcast(t, root);
          return t;
        }, py::arg("tensor"), py::arg("root") = 0, GR())
        .def("barrier", &Comm::barrier, GR());
    py::class_<comm::FakeWorld, std::shared_ptr<comm::FakeWorld>>(m, "FakeWorld",
        "N in-process ranks over host memory (CPU test double of the communicator)")
        .def(py::init<int>())
        .def_property_readonly("size", &comm::FakeWorld::size)
        .def("comm", [](std::shared_ptr<comm::FakeWorld> w, int r) {
          return std::shared_ptr<Comm>(std::make_shared<comm::FakeComm>(w, r));
        });
    py::class_<comm::RcclComm, Comm, std::shared_ptr<comm::RcclComm>>(m, "RcclComm",
        "an RCCL communicator of the engine's own (ncclCommInitRank)")
        .def(py::init([](py::bytes uid, int rank, int size, int device) {
          std::string u = uid;
          py::gil_scoped_release nogil;
          return std::make_shared<comm::RcclComm>(u, rank, size, device);
        }), py::arg("unique_id"), py::arg("rank"), py::arg("size"), py::arg("device"))
        .def("abort", &comm::RcclComm::abort, GR())
        .def("async_error", &comm::RcclComm::async_error)
        .def("set_timeout", &comm::RcclComm::set_timeout, py::arg("seconds"), py::arg("exit_on_timeout") = true,
             "seconds a collective may take (<= 0: unbounded); past it wait() raises CollectiveError, and past it "
             "plus a grace period the watchdog thread aborts the communicator and exits the process "
             "(exit_on_timeout) or marks it failed")
        .def_property_readonly("timeout", &comm::RcclComm::timeout)
        .def("wait", &comm::RcclComm::wait, GR(), "bounded wait for every collective issued so far")
        .def("check", &comm::RcclComm::check, "raises CollectiveError if the communicator failed")
        .def_property_readonly("failed", &comm::RcclComm::failed)
        .def_property_readonly("inflight", &comm::RcclComm::inflight)
        .def("set_test_stall", &comm::RcclComm::set_test_stall, py::arg("seconds"),
             "tests: a spin kernel inside each all_reduce, after its start event");
    py::class_<comm::ShmComm, Comm, std::shared_ptr<comm::ShmComm>>(m, "ShmComm",
        "host tensors of the ranks of one node through a POSIX shared-memory segment")
        .def(py::init<const std::string&, int, int, int64_t, bool>(), py::arg("name"), py::arg("rank"),
             py::arg("size"), py::arg("slot_bytes"), py::arg("create"), GR())
        .def("unlink", &comm::ShmComm::unlink)
        .def("set_timeout", &comm::ShmComm::set_timeout, py::arg("seconds"))
        .def("poison", &comm::ShmComm::poison, "make every rank's current / next collective raise")
        .def("reset_after_failure", &comm::ShmComm::reset_after_failure,
             "clear the barrier state (only once every rank has left the communicator)")
        .def_property_readonly("poisoned", &comm::ShmComm::poisoned)
        .def_property_readonly("slot_bytes", &comm::ShmComm::slot_bytes)
        .def_property_readonly("attached", &comm::ShmComm::attached);
    m.attr("EXIT_COLLECTIVE_TIMEOUT") = comm::kExitCollectiveTimeout;
    m.def("device_stall", [](double seconds) {
      k::device_stall(static_cast<uint64_t>(std::max(0.0, seconds) * 1e6),
                      c10::hip::getCurrentHIPStream().stream());
    }, py::arg("seconds"), "fault injection: a bounded (<= 60 s) spin kernel on the current stream");
    m.def("can_access_peer", [](int a, int b) {
      int ok = 0;
      if (hipDeviceCanAccessPeer(&ok, a, b) != hipSuccess) {
        (void)hipGetLastError();
        return false;
      }
      return ok != 0;
    }, py::arg("device"), py::arg("peer"));
    m.def("rccl_unique_id", [] { return py::bytes(comm::rccl_unique_id()); });
    py::class_<comm::OneShotComm, std::shared_ptr<comm::OneShotComm>>(m, "OneShotComm",
        "single-hop all-reduce of payloads <= 64 KB through IPC-mapped peer buffers")
        .def(py::init<int, int, int>(), py::arg("rank"), py::arg("size"), py::arg("device"))
        .def("ipc_handle", [](comm::OneShotComm& o) { return py::bytes(o.ipc_handle()); })
        .def("open", &comm::OneShotComm::open)
        .def_property_readonly("ready", &comm::OneShotComm::ready)
        .def_property_readonly("calls", &comm::OneShotComm::calls)
        .def_static("max_bytes", &comm::OneShotComm::max_bytes)
        .def("all_reduce", [](comm::OneShotComm& o, at::Tensor t, const std::string& op) {
          o.all_reduce(t, comm::parse_op(op));
          return t;
        }, py::arg("tensor"), py::arg("op") = "Sum", GR())
        .def("check", &comm::OneShotComm::check, GR())
        .def("set_timeout", &comm::OneShotComm::set_timeout, py::arg("seconds"))
        .def_property_readonly("alloc_kind", &comm::OneShotComm::alloc_kind)
        .def_property_readonly("failed", &comm::OneShotComm::failed);
  }
  m.def("cat_rows", [](const std::vector<at::Tensor>& ts) {
    TFA_CHECK(!ts.empty(), "cat_rows: no tensors");
    const at::Tensor& t0 = ts[0];
    TFA_CHECK(t0.is_cuda() && t0.dim() >= 1, "cat_rows: device tensors of rank >= 1 expected");
    std::vector<int64_t> sz = t0.sizes().vec();
    int64_t rows = 0;
    for (auto& t : ts) {
      TFA_CHECK(t.is_cuda() && t.device() == t0.device() && t.scalar_type() == t0.scalar_type() &&
                    t.dim() == t0.dim() && t.sizes().slice(1) == t0.sizes().slice(1),
                "cat_rows: tensors must share device, dtype and trailing shape");
      rows += t.size(0);
    }
    sz[0] = rows;
    c10::hip::HIPGuard guard(t0.device().index());
    at::Tensor out = pool_empty(sz, t0.options());
    hipStream_t st = c10::hip::getCurrentHIPStream(t0.device().index()).stream();
    std::vector<at::Tensor> keep;  // contiguous copies of strided inputs, alive until launched
    k::CopyPieces pc;
    int64_t off = 0;
    auto flush = [&]() {
      k::batched_copy(pc, out.data_ptr(), st);
      pc.n = 0;
    };
    for (auto& t0i : ts) {
      at::Tensor t = t0i.is_contiguous() ? t0i : t0i.contiguous();
      if (!t0i.is_contiguous()) keep.push_back(t);
      const int64_t nb = t.numel() * t.element_size();
      if (nb) {
        pc.src[pc.n] = t.data_ptr();
        pc.dst_off[pc.n] = off;
        pc.bytes[pc.n] = nb;
        if (++pc.n == k::kMaxCopyPieces) flush();
      }
      off += nb;
    }
    flush();
    for (auto& t : keep) dev_record_stream(t, st);
    return out;
  }, py::arg("tensors"), "row concatenation of device tensors into one pool buffer: one batched-copy kernel");
  m.def("cat_rows_many", [](const std::vector<std::vector<at::Tensor>>& cols) {
    // several row concatenations (the columns of merged partitions) into ONE
    // pool buffer with one batched-copy launch per 32 pieces; each result is
    // a view of that buffer at a 256-byte aligned offset
    TFA_CHECK(!cols.empty() && !cols[0].empty(), "cat_rows_many: no tensors");
    const at::Tensor& t00 = cols[0][0];
    TFA_CHECK(t00.is_cuda(), "cat_rows_many: device tensors expected");
    std::vector<std::vector<int64_t>> shapes;
    std::vector<int64_t> offs;
    int64_t total = 0;
    for (auto& ts : cols) {
      TFA_CHECK(!ts.empty(), "cat_rows_many: empty column");
      const at::Tensor& t0 = ts[0];
      TFA_CHECK(t0.dim() >= 1, "cat_rows_many: tensors of rank >= 1 expected");
      std::vector<int64_t> sz = t0.sizes().vec();
      int64_t rows = 0, nb = 0;
      for (auto& t : ts) {
        TFA_CHECK(t.is_cuda() && t.device() == t00.device() && t.scalar_type() == t0.scalar_type() &&
                      t.dim() == t0.dim() && t.sizes().slice(1) == t0.sizes().slice(1),
                  "cat_rows_many: the tensors of a column must share device, dtype and trailing shape");
        rows += t.size(0);
        nb += t.numel() * t.element_size();
      }
      sz[0] = rows;
      shapes.push_back(sz);
      offs.push_back(total);
      total += (nb + 255) / 256 * 256;
    }
    c10::hip::HIPGuard guard(t00.device().index());
    at::Tensor buf = pool_empty({std::max<int64_t>(total, 1)}, t00.options().dtype(at::kByte));
    hipStream_t st = c10::hip::getCurrentHIPStream(t00.device().index()).stream();
    std::vector<at::Tensor> keep;
    k::CopyPieces pc;
    auto flush = [&]() {
      k::batched_copy(pc, buf.data_ptr(), st);
      pc.n = 0;
    };
    for (size_t c = 0; c < cols.size(); ++c) {
      int64_t off = offs[c];
      for (auto& t0i : cols[c]) {
        at::Tensor t = t0i.is_contiguous() ? t0i : t0i.contiguous();
        if (!t0i.is_contiguous()) keep.push_back(t);
        const int64_t nb = t.numel() * t.element_size();
        if (nb) {
          pc.src[pc.n] = t.data_ptr();
          pc.dst_off[pc.n] = off;
          pc.bytes[pc.n] = nb;
          if (++pc.n == k::kMaxCopyPieces) flush();
        }
        off += nb;
      }
    }
    flush();
    for (auto& t : keep) dev_record_stream(t, st);
    std::vector<at::Tensor> out;
    for (size_t c = 0; c < cols.size(); ++c) {
      const auto dt = cols[c][0].scalar_type();
      int64_t n = 1;
      for (int64_t d : shapes[c]) n *= d;
      out.push_back(buf.narrow(0, offs[c], n * c10::elementSize(dt)).view(dt).view(shapes[c]));
    }
    return out;
  }, py::arg("columns"), "row concatenations of several columns into one pool buffer (views of it)");
  m.def("pipeline_wait", &pipeline_wait, py::arg("handle"), py::call_guard<py::gil_scoped_release>(),
        "wait for a run_chunked(wait=False) completion handle (and release it)");
  m.def("device_empty", [](const std::vector<int64_t>& sizes, at::ScalarType dt, int device) {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
    return pool_empty(sizes, at::TensorOptions().dtype(dt).device(at::kCUDA, static_cast<c10::DeviceIndex>(device)));
  }, py::arg("sizes"), py::arg("dtype"), py::arg("device"),
        "uninitialised device tensor from the engine pool, ordered on the device's current stream");
  m.def("device_zeros", [](const std::vector<int64_t>& sizes, at::ScalarType dt, int device) {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
    return pool_zeros(sizes, at::TensorOptions().dtype(dt).device(at::kCUDA, static_cast<c10::DeviceIndex>(device)));
  }, py::arg("sizes"), py::arg("dtype"), py::arg("device"), "zeroed (hipMemsetAsync) device tensor from the engine pool");
  m.def("fill_", [](at::Tensor& t, double value) {
    TFA_CHECK(t.is_cuda() && t.is_contiguous(), "fill_: contiguous device tensor expected");
    c10::hip::HIPGuard guard(t.device().index());
    k::fill(from_scalar_type(t.scalar_type()), t.data_ptr(), t.numel(), value,
            c10::hip::getCurrentHIPStream(t.device().index()).stream());
    return t;
  }, py::arg("tensor"), py::arg("value"), "fill a device tensor in place (kernels/elementwise fill)");
  m.def("record_stream", [](const at::Tensor& t, uint64_t stream) {
    TFA_CHECK(t.is_cuda(), "record_stream: device tensor expected");
    dev_record_stream(t, reinterpret_cast<hipStream_t>(stream));
  }, py::arg("tensor"), py::arg("stream"),
        "the tensor is also used on `stream` (a hipStream_t handle): its memory (engine pool or c10) is not "
        "reused before that stream's work queued so far has finished");
  m.def("pinned_pool_stats", [] {
    auto v = pinned_pool_stats();
    py::dict d;
    d["limit"] = v[0];
    d["cached"] = v[1];
    d["live"] = v[2];
    d["peak"] = v[3];
    return d;
  }, "page-locked pool: cap, cached free bytes, live bytes, peak live bytes");
  m.def("pin_host_tensor", &pin_host_tensor);
  m.def("unpin_host_tensor", &unpin_host_tensor);
}

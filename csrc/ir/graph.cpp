// Graph import, edge resolution, closure and static inference / constant folding.
#include <unordered_map>
#include "graph.h"

#include <chrono>
#include <cstring>
#include <string_view>
#include <cstdio>
#include <cstdlib>

#include <c10/hip/HIPFunctions.h>

#include "../runtime/device_pool.h"

#include <algorithm>
#include <set>

namespace tfa {

OpRegistry& OpRegistry::get() {
  static OpRegistry* r = [] {
    auto* reg = new OpRegistry();
    register_array_ops(*reg);
    register_math_ops(*reg);
    register_nn_ops(*reg);
    register_extra_ops(*reg);
    register_more_ops(*reg);
    return reg;
  }();
  return *r;
}

std::vector<std::string> OpRegistry::names() const {
  std::vector<std::string> v;
  for (auto& kv : ops_) v.push_back(kv.first);
  std::sort(v.begin(), v.end());
  return v;
}

// ------------------------------------------------------------------ attrs
static const AttrValue& need_attr(const Node& n, const std::string& k) {
  const AttrValue* a = n.def->find_attr(k);
  TFA_CHECK(a, "node '", n.name, "' (", n.op, ") is missing attribute '", k, "'");
  return *a;
}

int64_t Node::attr_i(const std::string& k, std::optional<int64_t> d) const {
  const AttrValue* a = def->find_attr(k);
  if (!a) {
    TFA_CHECK(d.has_value(), "node '", name, "' (", op, ") is missing attribute '", k, "'");
    return *d;
  }
  return a->i;
}
float Node::attr_f(const std::string& k, std::optional<float> d) const {
  const AttrValue* a = def->find_attr(k);
  if (!a) {
    TFA_CHECK(d.has_value(), "node '", name, "' (", op, ") is missing attribute '", k, "'");
    return *d;
  }
  return a->f;
}
bool Node::attr_b(const std::string& k, std::optional<bool> d) const {
  const AttrValue* a = def->find_attr(k);
  if (!a) {
    TFA_CHECK(d.has_value(), "node '", name, "' (", op, ") is missing attribute '", k, "'");
    return *d;
  }
  return a->b;
}
DType Node::attr_type(const std::string& k, std::optional<DType> d) const {
  const AttrValue* a = def->find_attr(k);
  if (!a) {
    TFA_CHECK(d.has_value(), "node '", name, "' (", op, ") is missing attribute '", k, "'");
    return *d;
  }
  return a->type;
}
std::string Node::attr_s(const std::string& k, std::optional<std::string> d) const {
  const AttrValue* a = def->find_attr(k);
  if (!a) {
    TFA_CHECK(d.has_value(), "node '", name, "' (", op, ") is missing attribute '", k, "'");
    return *d;
  }
  return a->s;
}
Shape Node::attr_shape(const std::string& k) const { return need_attr(*this, k).shape; }
std::vector<int64_t> Node::attr_ilist(const std::string& k, std::vector<int64_t> d) const {
  const AttrValue* a = def->find_attr(k);
  if (!a || !a->list) return d;
  return a->list->i;
}
const HostTensor& Node::attr_tensor(const std::string& k) const {
  const AttrValue& a = need_attr(*this, k);
  TFA_CHECK(a.tensor, "attribute '", k, "' of node '", name, "' is not a tensor");
  return *a.tensor;
}

// ------------------------------------------------------------------ dtype helpers
at::ScalarType to_scalar_type(DType d) {
  switch (d) {
    case DType::F32: return at::kFloat;
    case DType::F64: return at::kDouble;
    case DType::I32: return at::kInt;
    case DType::I64: return at::kLong;
    case DType::U8: return at::kByte;
    case DType::I8: return at::kChar;
    case DType::I16: return at::kShort;
    case DType::BOOL: return at::kBool;
    case DType::F16: return at::kHalf;
    case DType::BF16: return at::kBFloat16;
    default: TFA_CHECK(false, "dtype ", dtype_name(d), " has no tensor representation");
  }
  return at::kFloat;
}

DType from_scalar_type(at::ScalarType s) {
  switch (s) {
    case at::kFloat: return DType::F32;
    case at::kDouble: return DType::F64;
    case at::kInt: return DType::I32;
    case at::kLong: return DType::I64;
    case at::kByte: return DType::U8;
    case at::kChar: return DType::I8;
    case at::kShort: return DType::I16;
    case at::kBool: return DType::BOOL;
    case at::kHalf: return DType::F16;
    case at::kBFloat16: return DType::BF16;
    default: TFA_CHECK(false, "unsupported tensor scalar type ", c10::toString(s));
  }
  return DType::INVALID;
}

at::Tensor host_tensor_to_at(const HostTensor& t) {
  auto dims = dims_or_throw(t.shape, "constant");
  at::Tensor out = at::empty(dims, at::TensorOptions().dtype(to_scalar_type(t.dtype)));
  if (!t.bytes.empty()) std::memcpy(out.data_ptr(), t.bytes.data(), t.bytes.size());
  return out;
}

at::Tensor host_tensor_view(const HostTensor& t) {
  auto dims = dims_or_throw(t.shape, "constant");
  if (t.bytes.empty()) return at::empty(dims, at::TensorOptions().dtype(to_scalar_type(t.dtype)));
  TFA_CHECK(static_cast<int64_t>(t.bytes.size()) == t.num_elements() * dtype_size(t.dtype),
            "constant: ", t.bytes.size(), " bytes for ", t.num_elements(), " elements");
  return at::from_blob(const_cast<uint8_t*>(t.bytes.data()), dims,
                       at::TensorOptions().dtype(to_scalar_type(t.dtype)));
}

std::vector<int64_t> to_int_vector(const at::Tensor& t) {
  at::Tensor c = t.to(at::kCPU).to(at::kLong).contiguous().reshape({-1});
  const int64_t* p = c.data_ptr<int64_t>();
  return std::vector<int64_t>(p, p + c.numel());
}

Shape shape_of(const at::Tensor& t) { return Shape(t.sizes().vec()); }

std::vector<int64_t> dims_or_throw(const Shape& s, const char* what) {
  TFA_CHECK(s.fully_known(), "shape of ", what, " must be fully known, got ", s.str());
  return s.dims;
}

Shape broadcast_shapes(const Shape& a, const Shape& b) {
  if (a.unknown_rank || b.unknown_rank) return Shape::unknown();
  const Shape& hi = a.dims.size() >= b.dims.size() ? a : b;
  const Shape& lo = a.dims.size() >= b.dims.size() ? b : a;
  size_t off = hi.dims.size() - lo.dims.size();
  std::vector<int64_t> out(hi.dims.begin(), hi.dims.end());
  for (size_t i = 0; i < lo.dims.size(); ++i) {
    int64_t d1 = hi.dims[off + i], d2 = lo.dims[i];
    int64_t r;
    if (d1 == d2) r = d1;
    else if (d1 == 1) r = d2;
    else if (d2 == 1) r = d1;
    else if (d1 < 0) r = d2;   // unknown vs known (>1)
    else if (d2 < 0) r = d1;
    else {
      TFA_CHECK(false, "Incompatible shapes: ", a.str(), " ", b.str());
      r = -1;
    }
    out[off + i] = r;
  }
  return Shape(out);
}

// ------------------------------------------------------------------ ctx helpers
std::optional<std::vector<int64_t>> InferCtx::ivalue(int i) const {
  const TensorInfo& t = input(i);
  if (!t.value) return std::nullopt;
  return to_int_vector(*t.value);
}

std::optional<double> InferCtx::scalar_value(int i) const {
  const TensorInfo& t = input(i);
  if (!t.value || t.value->numel() != 1) return std::nullopt;
  return t.value->to(at::kDouble).item<double>();
}

bool InferCtx::all_const() const {
  for (auto* t : in)
    if (t->row != RowClass::CONST) return false;
  return true;
}

void InferCtx::rows_default() {
  RowClass r = all_const() ? RowClass::CONST : RowClass::MIXED;
  for (auto& o : out) o.row = r;
}

void InferCtx::rows_like(int i) {
  for (auto& o : out) o.row = input(i).row;
}

void InferCtx::rows_elementwise() {
  if (all_const()) {
    for (auto& o : out) o.row = RowClass::CONST;
    return;
  }
  int out_rank = out.at(0).shape.rank();
  RowClass r = RowClass::ROW;
  if (out_rank < 1) r = RowClass::MIXED;
  for (auto* t : in) {
    if (r == RowClass::MIXED) break;
    if (t->row == RowClass::MIXED) {
      r = RowClass::MIXED;
    } else if (t->row == RowClass::ROW) {
      if (t->shape.rank() != out_rank) r = RowClass::MIXED;
    } else {  // CONST operand: must not carry a row dim
      int rk = t->shape.rank();
      if (rk < 0) r = RowClass::MIXED;
      else if (rk == out_rank && t->shape.dims[0] != 1) r = RowClass::MIXED;
    }
  }
  for (auto& o : out) o.row = r;
}

at::TensorOptions ExecCtx::options(int i) const { return in.at(i).options(); }

std::vector<int64_t> ExecCtx::host_ivalue(int i) const {
  const TensorInfo* t = in_info->at(i);
  if (t->value) return to_int_vector(*t->value);
  return to_int_vector(in.at(i));  // data-dependent: device->host sync
}

at::Tensor ExecCtx::alloc_out(int i) {
  const TensorInfo& oi = out_info->at(i);
  auto dims = dims_or_throw(oi.shape, "output");
  at::TensorOptions opt = at::TensorOptions().dtype(to_scalar_type(oi.dtype));
  if (!in.empty() && in[0].defined()) opt = opt.device(in[0].device());
  else if (gpu) opt = opt.device(at::Device(at::kCUDA, c10::hip::current_device()));
  return alloc(dims, opt);
}

at::Tensor ExecCtx::alloc(at::IntArrayRef sizes, const at::TensorOptions& opts) const {
  if (gpu && opts.device().is_cuda())
    return dev_empty(sizes, opts.dtype().toScalarType(), opts.device(), static_cast<hipStream_t>(stream));
  return at::empty(sizes, opts);
}

// ------------------------------------------------------------------ Graph
static std::pair<std::string, int> split_tensor_name(const std::string& s) {
  auto pos = s.rfind(':');
  if (pos == std::string::npos) return {s, 0};
  std::string idx = s.substr(pos + 1);
  if (idx.empty() || !std::all_of(idx.begin(), idx.end(), ::isdigit)) return {s, 0};
  return {s.substr(0, pos), std::stoi(idx)};
}

Graph::Graph(GraphDef def) : def_(std::move(def)) {
  const OpRegistry& reg = OpRegistry::get();
  nodes_.resize(def_.nodes.size());
  for (size_t i = 0; i < def_.nodes.size(); ++i) {
    const NodeDef& nd = def_.nodes[i];
    TFA_CHECK(!nd.name.empty(), "GraphDef node ", i, " has no name");
    TFA_CHECK(!by_name_.count(nd.name), "duplicate node name '", nd.name, "' in GraphDef");
    by_name_[nd.name] = static_cast<int>(i);
    Node& n = nodes_[i];
    n.name = nd.name;
    n.op = nd.op;
    n.def = &nd;
  }
  for (size_t i = 0; i < def_.nodes.size(); ++i) {
    const NodeDef& nd = def_.nodes[i];
    Node& n = nodes_[i];
    for (const std::string& in : nd.inputs) {
      if (!in.empty() && in[0] == '^') {
        int j = find(in.substr(1));
        TFA_CHECK(j >= 0, "node '", n.name, "': unknown control input '", in, "'");
        n.control.push_back(j);
      } else {
        n.inputs.push_back(resolve(in));
      }
    }
    const OpDef* od = reg.find(n.op);
    n.num_outputs = od ? od->num_outputs(n) : 1;
  }
}

std::shared_ptr<Graph> Graph::from_bytes(const std::string& bytes) {
  return std::make_shared<Graph>(parse_graphdef(bytes));
}

TensorRef Graph::resolve(const std::string& name) const {
  auto [base, idx] = split_tensor_name(name);
  int n = find(base);
  if (n < 0) n = find(name);  // names that legitimately contain ':'
  TFA_CHECK(n >= 0, "Graph has no node named '", base, "'");
  return TensorRef{n, idx};
}

std::vector<int> Graph::closure(const std::vector<TensorRef>& fetches) const {
  std::vector<int> order;
  std::vector<int> state(nodes_.size(), 0);  // 0 new, 1 visiting, 2 done
  std::vector<std::pair<int, size_t>> stack;
  for (auto& f : fetches) {
    if (state[f.node]) continue;
    stack.push_back({f.node, 0});
    state[f.node] = 1;
    while (!stack.empty()) {
      auto& [n, k] = stack.back();
      const Node& nd = nodes_[n];
      size_t total = nd.inputs.size() + nd.control.size();
      if (k < total) {
        int dep = k < nd.inputs.size() ? nd.inputs[k].node : nd.control[k - nd.inputs.size()];
        ++k;
        if (state[dep] == 1) TFA_CHECK(false, "cycle in graph at node '", nodes_[dep].name, "'");
        if (state[dep] == 0) {
          state[dep] = 1;
          stack.push_back({dep, 0});
        }
      } else {
        state[n] = 2;
        order.push_back(n);
        stack.pop_back();
      }
    }
  }
  return order;
}

namespace {
struct KeyHash {
  uint64_t h = 1469598103934665603ull;
  void mix(uint64_t x) { h ^= x + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2); }
  void str(const std::string& s) {
    mix(std::hash<std::string_view>{}(s));
    mix(s.size());
  }
  void bytes(const void* p, size_t n) {
    mix(std::hash<std::string_view>{}(std::string_view(static_cast<const char*>(p), n)));
    mix(n);
  }
  void shape(const Shape& s) {
    mix(s.unknown_rank ? 1 : 0);
    mix(s.dims.size());
    for (auto d : s.dims) mix(static_cast<uint64_t>(d));
  }
  void tensor(const HostTensor& t, bool payload) {
    mix(static_cast<uint64_t>(t.dtype));
    shape(t.shape);
    if (!payload) return;
    bytes(t.bytes.data(), t.bytes.size());
    mix(t.strings.size());
    for (auto& x : t.strings) str(x);
  }
};
}  // namespace

const std::vector<char>& Graph::parameter_consts() const {
  (void)structure_key();
  return params_;
}

namespace {
// structure hash -> whether its candidate parameter constants are safe to
// treat as parameters (the taint walk below needs a whole-graph inference;
// a graph rebuilt every iteration with new parameter values has the same
// structure hash, so the walk runs once per structure, not per rebuild)
std::mutex& safe_mu() {
  static std::mutex m;
  return m;
}
std::unordered_map<uint64_t, bool>& safe_cache() {
  static std::unordered_map<uint64_t, bool> c;
  return c;
}
}  // namespace

uint64_t Graph::hash_nodes(const std::vector<char>& param) const {
  KeyHash k;
  for (size_t i = 0; i < nodes_.size(); ++i) {
    const NodeDef& d = *nodes_[i].def;
    k.str(d.name);
    k.str(d.op);
    k.mix(d.inputs.size());
    for (auto& in : d.inputs) k.str(in);
    k.str(d.device);
    k.mix(d.attr.size());
    for (auto& [name, a] : d.attr) {
      k.str(name);
      k.mix(static_cast<uint64_t>(a.kind));
      switch (a.kind) {
        case AttrValue::S:
        case AttrValue::PLACEHOLDER:
        case AttrValue::FUNC: k.str(a.s); break;
        case AttrValue::I: k.mix(static_cast<uint64_t>(a.i)); break;
        case AttrValue::F: {
          uint32_t b;
          std::memcpy(&b, &a.f, 4);
          k.mix(b);
          break;
        }
        case AttrValue::B: k.mix(a.b ? 1 : 0); break;
        case AttrValue::TYPE: k.mix(static_cast<uint64_t>(a.type)); break;
        case AttrValue::SHAPE: k.shape(a.shape); break;
        case AttrValue::TENSOR:
          if (a.tensor) k.tensor(*a.tensor, !(param[i] && name == "value"));
          break;
        case AttrValue::LIST:
          if (a.list) {
            const AttrList& l = *a.list;
            k.mix(l.s.size());
            for (auto& x : l.s) k.str(x);
            k.mix(l.i.size());
            for (auto x : l.i) k.mix(static_cast<uint64_t>(x));
            k.mix(l.f.size());
            for (auto x : l.f) {
              uint32_t b;
              std::memcpy(&b, &x, 4);
              k.mix(b);
            }
            k.mix(l.b.size());
            for (bool x : l.b) k.mix(x ? 1 : 0);
            k.mix(l.type.size());
            for (auto x : l.type) k.mix(static_cast<uint64_t>(x));
            k.mix(l.shape.size());
            for (auto& x : l.shape) k.shape(x);
            k.mix(l.tensor.size());
            for (auto& x : l.tensor) k.tensor(x, true);
          }
          break;
        default: break;
      }
    }
  }
  return k.h;
}

std::shared_ptr<Graph> Graph::with_values(const std::map<std::string, at::Tensor>& values) const {
  const std::vector<char>& params = parameter_consts();
  GraphDef d = def_;  // node copies; tensor payloads stay shared (shared_ptr<HostTensor>)
  for (const auto& [name, t] : values) {
    const int i = find(name);
    TFA_CHECK(i >= 0 && params[i], "with_values: '", name, "' is not a parameter constant of the graph");
    auto it = d.nodes[i].attr.find("value");
    TFA_CHECK(it != d.nodes[i].attr.end() && it->second.kind == AttrValue::TENSOR && it->second.tensor,
              "with_values: '", name, "' has no tensor value");
    const HostTensor& old = *it->second.tensor;
    at::Tensor c = t.contiguous();
    if (c.is_cuda()) c = c.cpu();
    TFA_CHECK(c.scalar_type() == to_scalar_type(old.dtype) && c.numel() == old.num_elements(),
              "with_values: '", name, "' needs ", old.num_elements(), " values of its dtype");
    auto ht = std::make_shared<HostTensor>();
    ht->dtype = old.dtype;
    ht->shape = old.shape;
    const auto* b = static_cast<const uint8_t*>(c.data_ptr());
    ht->bytes.assign(b, b + c.numel() * c.element_size());
    it->second.tensor = std::move(ht);
  }
  // same nodes, names and edges: copy the resolved structure instead of
  // re-resolving every input by name; only the def pointers move
  auto g = std::shared_ptr<Graph>(new Graph(*this, std::move(d)));
  std::lock_guard<std::mutex> lk(key_mu_);
  g->key_ = key_;
  g->params_ = params_;
  return g;
}

Graph::Graph(const Graph& base, GraphDef def) : def_(std::move(def)), nodes_(base.nodes_), by_name_(base.by_name_) {
  TFA_CHECK(def_.nodes.size() == nodes_.size(), "graph copy: node count changed");
  for (size_t i = 0; i < nodes_.size(); ++i) nodes_[i].def = &def_.nodes[i];
}

uint64_t Graph::structure_key() const {
  std::lock_guard<std::mutex> lk(key_mu_);
  if (key_) return *key_;
  std::vector<char> param(nodes_.size(), 0);
  bool any = false;
  for (size_t i = 0; i < nodes_.size(); ++i) {
    if (nodes_[i].op != "Const") continue;
    const AttrValue* v = nodes_[i].def->find_attr("value");
    if (v && v->kind == AttrValue::TENSOR && v->tensor && dtype_is_float(v->tensor->dtype) &&
        !v->tensor->shape.unknown_rank && v->tensor->num_elements() >= 2) {
      param[i] = 1;
      any = true;
    }
  }
  uint64_t h = hash_nodes(param);
  if (any) {
    bool safe;
    bool known = false;
    {
      std::lock_guard<std::mutex> g(safe_mu());
      auto it = safe_cache().find(h);
      if (it != safe_cache().end()) {
        safe = it->second;
        known = true;
      }
    }
    if (!known) {
      // taint: a folded value computed from a parameter must itself be a
      // floating tensor of >= 2 elements (never an integer shape/axis/multiple
      // or a scalar the planner bakes into a kernel)
      safe = true;
      try {
        std::vector<TensorRef> all;
        all.reserve(nodes_.size());
        for (size_t i = 0; i < nodes_.size(); ++i) all.push_back({static_cast<int>(i), 0});
        std::vector<int> order = closure(all);
        Infos inf = infer(order, {}, false);
        std::vector<char> taint(nodes_.size(), 0);
        for (int n : order) {
          bool t = param[n] != 0;
          for (auto& r : nodes_[n].inputs) t = t || taint[r.node];
          taint[n] = t;
          if (!t || param[n]) continue;
          for (auto& o : inf[n])
            if (o.value && !(dtype_is_float(o.dtype) && o.value->numel() >= 2)) safe = false;
        }
      } catch (const std::exception&) {
        safe = false;
      }
      std::lock_guard<std::mutex> g(safe_mu());
      if (safe_cache().size() > 4096) safe_cache().clear();
      safe_cache()[h] = safe;
    }
    if (!safe) {
      std::fill(param.begin(), param.end(), 0);
      h = hash_nodes(param);
    }
  }
  params_ = std::move(param);
  key_ = h;
  return h;
}

std::vector<int> Graph::placeholders() const {
  std::vector<int> v;
  for (size_t i = 0; i < nodes_.size(); ++i)
    if ((nodes_[i].op == "Placeholder" || nodes_[i].op == "PlaceholderV2") && nodes_[i].inputs.empty())
      v.push_back(static_cast<int>(i));
  return v;
}

// Largest result folded on the host (elements): shape arithmetic and small
// constant expressions. A big CONST-class tensor (a Tile of centroids to the
// block row count, K-Means) is cheaper to compute on the device each run than
// to build with ATen on the host at every analysis/plan and upload.
static constexpr int64_t kFoldLimit = int64_t(1) << 16;
// values that depend on the feeds' shapes (Shape -> StridedSlice -> Pack ->
// Tile/Fill multiples) fold only while small: shape arithmetic is a few
// elements, while a row-sized Tile/Fill folded on the host would be rebuilt
// and uploaded for every plan (every partition size, every rebuilt graph)
// instead of being written by one device kernel
static constexpr int64_t kDynFoldLimit = 1024;

Graph::Infos Graph::infer(const std::vector<int>& order, const std::map<int, TensorInfo>& feeds,
                          bool concrete) const {
  return infer_impl(order, feeds, concrete, nullptr, nullptr);
}

Graph::Infos Graph::infer_update(const std::vector<int>& order, const Infos& base, const std::vector<char>& redo,
                                 bool concrete) const {
  TFA_CHECK(base.size() == nodes_.size() && redo.size() == nodes_.size(), "infer_update: size mismatch");
  return infer_impl(order, {}, concrete, &base, &redo);
}

Graph::Infos Graph::infer_impl(const std::vector<int>& order, const std::map<int, TensorInfo>& feeds,
                               bool concrete, const Infos* base, const std::vector<char>* redo) const {
  const OpRegistry& reg = OpRegistry::get();
  Infos infos(nodes_.size());
  // dyn[n]: n depends on a placeholder or a stateful op (its info may change
  // with the feeds); every other node's info is memoised per graph
  std::vector<char> dyn(nodes_.size(), 0);
  const int ci = 0;  // (no op's inference of a placeholder-free node depends on `concrete`)
  {
    std::lock_guard<std::mutex> lk(static_mu_);
    if (static_known_[ci].size() != nodes_.size()) {
      static_known_[ci].assign(nodes_.size(), 0);
      static_infos_[ci].assign(nodes_.size(), {});
    }
  }
  for (int ni : order) {
    const Node& n = nodes_[ni];
    if (base && !(*redo)[ni]) {  // unchanged by the update: the base graph's infos
      infos[ni] = (*base)[ni];
      bool d = n.op == "Placeholder" || n.op == "PlaceholderV2";
      if (const OpDef* od0 = reg.find(n.op)) d = d || od0->stateful;
      for (auto& r : n.inputs) d = d || dyn[r.node];
      // a fed node (a cut point) carries no value: dynamic
      d = d || (!infos[ni].empty() && !infos[ni][0].value && infos[ni][0].row == RowClass::ROW);
      dyn[ni] = d;
      continue;
    }
    if (base && !n.inputs.empty()) {
      // redone, but every input that changed carries no value and kept its
      // dtype / shape / row class (inputs that did not change are the base's):
      // the node's infos are the base's (inference is a function of the input
      // infos and the unchanged attributes; a node with a valueless input is
      // never folded). A rebuilt K-Means graph re-infers only the few nodes
      // its new centres fold into, not everything downstream of them.
      bool same = base->at(ni).size() == static_cast<size_t>(n.num_outputs);
      for (auto& r : n.inputs) {
        if (!same) break;
        if (!(*redo)[r.node]) continue;
        if (r.index >= static_cast<int>(infos[r.node].size()) ||
            r.index >= static_cast<int>((*base)[r.node].size())) {
          same = false;
          break;
        }
        const TensorInfo& a = infos[r.node][r.index];
        const TensorInfo& b = (*base)[r.node][r.index];
        same = !a.value && !b.value && !a.strings && !b.strings && a.dtype == b.dtype && a.shape == b.shape &&
               a.row == b.row;
      }
      if (same) {
        infos[ni] = (*base)[ni];
        bool d = n.op == "Placeholder" || n.op == "PlaceholderV2";
        if (const OpDef* od0 = reg.find(n.op)) d = d || od0->stateful;
        for (auto& r : n.inputs) d = d || dyn[r.node];
        dyn[ni] = d;
        continue;
      }
    }
    auto fit = feeds.find(ni);
    if (fit != feeds.end()) {
      infos[ni] = {fit->second};
      infos[ni][0].row = fit->second.row;
      dyn[ni] = 1;
      continue;
    }
    const OpDef* od = reg.find(n.op);
    TFA_CHECK(od, "Op type not registered '", n.op, "' (node '", n.name,
              "'): tensorframes_amd has no kernel for it");
    bool d = od->stateful || n.op == "Placeholder" || n.op == "PlaceholderV2";
    for (auto& r : n.inputs) d = d || dyn[r.node];
    dyn[ni] = d;
    if (!d) {
      std::lock_guard<std::mutex> lk(static_mu_);
      if (static_known_[ci][ni]) {
        infos[ni] = static_infos_[ci][ni];
        continue;
      }
    }
    static const bool node_timing = [] {
      const char* e = std::getenv("TFA_PLAN_TIMING");
      return e && std::string(e) == "2";
    }();
    const auto tn0 = std::chrono::steady_clock::now();
    InferCtx ctx{n, {}, std::vector<TensorInfo>(n.num_outputs), concrete};
    for (auto& r : n.inputs) {
      TFA_CHECK(r.index < static_cast<int>(infos[r.node].size()), "node '", n.name,
                "' reads output ", r.index, " of '", nodes_[r.node].name, "' which has only ",
                infos[r.node].size(), " outputs");
      ctx.in.push_back(&infos[r.node][r.index]);
    }
    try {
      od->infer(ctx);
    } catch (const GraphError& e) {
      throw GraphError(str_cat("while inferring shapes of node '", n.name, "' (", n.op, "): ", e.what()));
    }
    if (od->rows) od->rows(ctx);
    else ctx.rows_default();
    // constant folding: every input statically known
    bool foldable = !od->stateful && n.op != "Placeholder" && n.op != "PlaceholderV2";
    for (auto* t : ctx.in)
      if (!t->value) foldable = false;
    for (auto& o : ctx.out)
      if (o.value || !o.shape.fully_known() || o.shape.num_elements() > (d ? kDynFoldLimit : kFoldLimit) ||
          o.dtype == DType::STRING)
        foldable = false;
    if (foldable && !ctx.in.empty() && od->compute) {
      ExecCtx ex{n, {}, {}, &ctx.out, &ctx.in, false, nullptr};
      for (auto* t : ctx.in) ex.in.push_back(*t->value);
      ex.out.resize(ctx.out.size());
      od->compute(ex);
      for (size_t k = 0; k < ctx.out.size(); ++k) ctx.out[k].value = ex.out[k].contiguous();
    }
    for (auto& o : ctx.out)
      if (o.value) o.row = RowClass::CONST;
    if (node_timing) {
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tn0).count();
      std::fprintf(stderr, "[tfa infer] %8.1fus %s %s%s\n", us, n.op.c_str(), n.name.c_str(),
                   ctx.out.size() && ctx.out[0].value ? " (folded)" : "");
    }
    if (!d) {
      std::lock_guard<std::mutex> lk(static_mu_);
      static_infos_[ci][ni] = ctx.out;
      static_known_[ci][ni] = 1;
    }
    infos[ni] = std::move(ctx.out);
  }
  return infos;
}

}  // namespace tfa

// Graph IR: an imported GraphDef with resolved edges, a per-op registry of
// shape/dtype inference + row-locality rules + compute functions.
//
// Replaces libtensorflow's Graph.importGraphDef + Operation.output(i).shape()
// (reference: src/main/scala/org/tensorframes/impl/TensorFlowOps.scala:87-150).
#pragma once

#include <ATen/ATen.h>

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "../proto/graphdef.h"

namespace tfa {

struct TensorRef {
  int node = -1;
  int index = 0;
  bool operator==(const TensorRef& o) const { return node == o.node && index == o.index; }
  bool operator<(const TensorRef& o) const {
    return node < o.node || (node == o.node && index < o.index);
  }
};

// How a tensor relates to the rows of the block that feeds the graph.
//  CONST : independent of every placeholder (foldable once shapes are known)
//  ROW   : leading dim is the block's row dim and row i depends only on input row i
//  MIXED : anything else (row-mixing, or depends on the number of rows)
enum class RowClass { CONST, ROW, MIXED };

struct TensorInfo {
  DType dtype = DType::INVALID;
  Shape shape = Shape::unknown();
  std::optional<at::Tensor> value;            // host (CPU) value when statically known
  std::shared_ptr<std::vector<std::string>> strings;  // string constants
  RowClass row = RowClass::CONST;
};

struct Node {
  std::string name;
  std::string op;
  const NodeDef* def = nullptr;
  std::vector<TensorRef> inputs;  // data inputs
  std::vector<int> control;       // control-dependency predecessors
  int num_outputs = 1;

  // attribute helpers (throw GraphError on missing/mistyped attrs)
  bool has_attr(const std::string& k) const { return def->find_attr(k) != nullptr; }
  int64_t attr_i(const std::string& k, std::optional<int64_t> dflt = std::nullopt) const;
  float attr_f(const std::string& k, std::optional<float> dflt = std::nullopt) const;
  bool attr_b(const std::string& k, std::optional<bool> dflt = std::nullopt) const;
  DType attr_type(const std::string& k, std::optional<DType> dflt = std::nullopt) const;
  std::string attr_s(const std::string& k, std::optional<std::string> dflt = std::nullopt) const;
  Shape attr_shape(const std::string& k) const;
  std::vector<int64_t> attr_ilist(const std::string& k, std::vector<int64_t> dflt = {}) const;
  const HostTensor& attr_tensor(const std::string& k) const;
};

struct InferCtx;
struct ExecCtx;

struct OpDef {
  // number of outputs (depends on attrs for a few ops, e.g. Unpack / IdentityN)
  std::function<int(const Node&)> num_outputs = [](const Node&) { return 1; };
  // shape & dtype inference; may read constant input values
  std::function<void(InferCtx&)> infer;
  // row-locality of outputs (given the input row classes)
  std::function<void(InferCtx&)> rows;
  // compute on concrete tensors (CPU via ATen, GPU via tensorframes_amd HIP kernels)
  std::function<void(ExecCtx&)> compute;
  // values of these input indices must be known at plan time (axes, shapes...)
  std::vector<int> host_inputs;
  bool stateful = false;
  bool host_only = false;  // runs in the Python host stage; a program must be cut at it
};

class OpRegistry {
 public:
  static OpRegistry& get();
  void add(const std::string& name, OpDef def) { ops_[name] = std::move(def); }
  const OpDef* find(const std::string& name) const {
    auto it = ops_.find(name);
    return it == ops_.end() ? nullptr : &it->second;
  }
  std::vector<std::string> names() const;

 private:
  std::unordered_map<std::string, OpDef> ops_;
};

// Registration helpers (defined in ops_*.cpp)
void register_array_ops(OpRegistry& r);
void register_math_ops(OpRegistry& r);
void register_nn_ops(OpRegistry& r);
void register_extra_ops(OpRegistry& r);
void register_more_ops(OpRegistry& r);

struct InferCtx {
  const Node& node;
  std::vector<const TensorInfo*> in;
  std::vector<TensorInfo> out;
  bool concrete;  // all placeholder shapes are fully known (plan time)

  const TensorInfo& input(int i) const { return *in.at(i); }
  TensorInfo& output(int i = 0) { return out.at(i); }
  // convenience: input value as int64 vector (requires known value)
  std::optional<std::vector<int64_t>> ivalue(int i) const;
  std::optional<double> scalar_value(int i) const;
  void set(int i, DType dt, Shape s) {
    out.at(i).dtype = dt;
    out.at(i).shape = std::move(s);
  }
  // default row rule: CONST if all inputs CONST, else MIXED
  void rows_default();
  // elementwise row rule (see RowClass)
  void rows_elementwise();
  // row-preserving op on input i (unary-like)
  void rows_like(int i);
  bool all_const() const;
};

struct ExecCtx {
  const Node& node;
  std::vector<at::Tensor> in;
  std::vector<at::Tensor> out;
  const std::vector<TensorInfo>* out_info;  // concrete output infos
  const std::vector<const TensorInfo*>* in_info;
  bool gpu;
  void* stream = nullptr;  // hipStream_t on GPU

  const at::Tensor& input(int i) const { return in.at(i); }
  at::TensorOptions options(int i = 0) const;
  const Shape& out_shape(int i = 0) const { return out_info->at(i).shape; }
  DType out_dtype(int i = 0) const { return out_info->at(i).dtype; }
  std::vector<int64_t> host_ivalue(int i) const;  // plan-time value of input i
  at::Tensor alloc_out(int i = 0);                  // allocate output i per out_info
  // scratch / intermediate tensor: on a GPU step from the engine's
  // stream-ordered device pool (runtime/device_pool.h), else at::empty
  at::Tensor alloc(at::IntArrayRef sizes, const at::TensorOptions& opts) const;
};

// Imported graph.
class Graph {
 public:
  explicit Graph(GraphDef def);
  static std::shared_ptr<Graph> from_bytes(const std::string& bytes);

  const GraphDef& def() const { return def_; }
  const std::vector<Node>& nodes() const { return nodes_; }
  const Node& node(int i) const { return nodes_.at(i); }
  int find(const std::string& name) const {
    auto it = by_name_.find(name);
    return it == by_name_.end() ? -1 : it->second;
  }
  // "x", "x:0", "x:1"
  TensorRef resolve(const std::string& name) const;
  // topological order of the closure of `fetches` (data + control edges)
  std::vector<int> closure(const std::vector<TensorRef>& fetches) const;
  // Placeholder nodes with no inputs (reference: TensorFlowOps.scala:106-108)
  std::vector<int> placeholders() const;

  // Static inference over the closure. `feeds` override placeholder infos
  // (dtype/shape). Returns infos indexed by node, then output.
  using Infos = std::vector<std::vector<TensorInfo>>;
  Infos infer(const std::vector<int>& order, const std::map<int, TensorInfo>& feeds,
              bool concrete) const;
  // The same inference, recomputing only the nodes marked in `redo` and taking
  // every other node's infos from `base` (the infos of a graph of the same
  // structure: a rebuilt graph whose parameter constants changed redoes only
  // the nodes those constants reach).
  Infos infer_update(const std::vector<int>& order, const Infos& base, const std::vector<char>& redo,
                     bool concrete) const;

  // Hash of the graph's structure: every node, input and attribute, except
  // the payloads of PARAMETER constants (floating-point Consts of >= 2
  // elements whose value reaches no plan-time decision: no folded integer or
  // scalar depends on them). Two graphs with equal keys have the same
  // inference results and plans up to those payloads (reference workload:
  // kmeans_demo.py:68-168 rebuilds its graphs with new centres every step).
  uint64_t structure_key() const;
  // hash of every node, parameter constants (param[i]) without their payloads
  uint64_t hash_nodes(const std::vector<char>& param) const;
  // node -> is a parameter constant (as used by structure_key)
  const std::vector<char>& parameter_consts() const;
  // The same graph with new payloads for some of its parameter constants
  // (same dtype and element count), built from the decoded GraphDef: no
  // serialisation or parse. The structure key carries over.
  std::shared_ptr<Graph> with_values(const std::map<std::string, at::Tensor>& values) const;

 private:
  // a copy of `base` (same structure) over `def`, a copy of base's GraphDef
  // with some constant payloads replaced (with_values)
  Graph(const Graph& base, GraphDef def);

  GraphDef def_;
  std::vector<Node> nodes_;
  std::unordered_map<std::string, int> by_name_;
  // infos of nodes that depend on no placeholder (constants and what folds
  // from them): the same in every inference of this graph, so analysis, the
  // row-separability check and planning fold each constant subgraph once
  // instead of once per call
  mutable std::mutex static_mu_;
  mutable std::vector<std::vector<TensorInfo>> static_infos_[1];
  mutable std::vector<char> static_known_[1];
  mutable std::mutex key_mu_;
  mutable std::optional<uint64_t> key_;
  mutable std::vector<char> params_;
  Infos infer_impl(const std::vector<int>& order, const std::map<int, TensorInfo>& feeds, bool concrete,
                   const Infos* base, const std::vector<char>* redo) const;
};

// dtype <-> ATen
at::ScalarType to_scalar_type(DType d);
DType from_scalar_type(at::ScalarType s);

// host value helpers
at::Tensor host_tensor_to_at(const HostTensor& t);
// zero-copy view of a HostTensor's bytes; valid while the owning Graph lives
at::Tensor host_tensor_view(const HostTensor& t);
std::vector<int64_t> to_int_vector(const at::Tensor& t);
Shape shape_of(const at::Tensor& t);
std::vector<int64_t> dims_or_throw(const Shape& s, const char* what);

// numpy-style broadcast of two (possibly partially unknown) shapes
Shape broadcast_shapes(const Shape& a, const Shape& b);

}  // namespace tfa

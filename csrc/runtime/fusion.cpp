// Elementwise-region fusion: region finding + HIP source generation (fusion.h).
#include "fusion.h"

#include <algorithm>
#include <cstdlib>
#include <functional>
#include <sstream>

namespace tfa {
namespace {

enum class Kind { UNARY, BINARY, VIEW, BCAST, CAST };

struct OpSpec {
  Kind kind;
  const char* fmt;   // {0} {1}: operand variables, {T}: the node's C type
  bool float_only;
};

const std::map<std::string, OpSpec>& op_table() {
  // Formulas mirror the unfused kernels (kernels/elementwise.hip un_apply /
  // bin_arith) so a fused region computes what the op-by-op plan computes.
  static const std::map<std::string, OpSpec> t = {
      {"Neg", {Kind::UNARY, "(-{0})", false}},
      {"Abs", {Kind::UNARY, "({0} < ({T})0 ? -{0} : {0})", false}},
      {"Square", {Kind::UNARY, "({0} * {0})", false}},
      {"Sqrt", {Kind::UNARY, "sqrt({0})", true}},
      {"Rsqrt", {Kind::UNARY, "(({T})1 / sqrt({0}))", true}},
      {"Exp", {Kind::UNARY, "exp({0})", true}},
      {"Log", {Kind::UNARY, "log({0})", true}},
      {"Log1p", {Kind::UNARY, "log1p({0})", true}},
      {"Expm1", {Kind::UNARY, "expm1({0})", true}},
      {"Reciprocal", {Kind::UNARY, "(({T})1 / {0})", true}},
      {"Inv", {Kind::UNARY, "(({T})1 / {0})", true}},
      {"Relu", {Kind::UNARY, "({0} > ({T})0 ? {0} : ({T})0)", false}},
      {"Relu6", {Kind::UNARY, "({0} > ({T})0 ? ({0} < ({T})6 ? {0} : ({T})6) : ({T})0)", false}},
      {"Elu", {Kind::UNARY, "({0} > ({T})0 ? {0} : expm1({0}))", true}},
      {"Selu", {Kind::UNARY,
                "({0} > ({T})0 ? ({T})1.0507009873554804934193349852946 * {0} : "
                "({T})1.0507009873554804934193349852946 * ({T})1.6732632423543772848170429916717 * expm1({0}))",
                true}},
      {"Sigmoid", {Kind::UNARY, "(({T})1 / (({T})1 + exp(-{0})))", true}},
      {"Tanh", {Kind::UNARY, "tanh({0})", true}},
      {"Softplus", {Kind::UNARY, "({0} > ({T})20 ? {0} : log1p(exp({0})))", true}},
      {"Softsign", {Kind::UNARY, "({0} / (({T})1 + fabs({0})))", true}},
      {"Floor", {Kind::UNARY, "floor({0})", true}},
      {"Ceil", {Kind::UNARY, "ceil({0})", true}},
      {"Rint", {Kind::UNARY, "rint({0})", true}},
      {"Round", {Kind::UNARY, "rint({0})", true}},
      {"Sign", {Kind::UNARY, "(({T})(({0} > ({T})0) - ({0} < ({T})0)))", false}},
      {"Sin", {Kind::UNARY, "sin({0})", true}},
      {"Cos", {Kind::UNARY, "cos({0})", true}},
      {"Erf", {Kind::UNARY, "erf({0})", true}},
      {"LeakyRelu", {Kind::UNARY, "", true}},  // formula built with the node's alpha
      {"Identity", {Kind::VIEW, "{0}", false}},
      {"Snapshot", {Kind::VIEW, "{0}", false}},
      {"StopGradient", {Kind::VIEW, "{0}", false}},
      {"PreventGradient", {Kind::VIEW, "{0}", false}},
      {"ExpandDims", {Kind::VIEW, "{0}", false}},
      {"Squeeze", {Kind::VIEW, "{0}", false}},
      {"Reshape", {Kind::VIEW, "{0}", false}},
      {"Tile", {Kind::BCAST, "{0}", false}},
      {"BroadcastTo", {Kind::BCAST, "{0}", false}},
      {"Cast", {Kind::CAST, "(({T}){0})", false}},
      {"Add", {Kind::BINARY, "({0} + {1})", false}},
      {"AddV2", {Kind::BINARY, "({0} + {1})", false}},
      {"BiasAdd", {Kind::BINARY, "({0} + {1})", false}},
      {"Sub", {Kind::BINARY, "({0} - {1})", false}},
      {"Mul", {Kind::BINARY, "({0} * {1})", false}},
      {"Div", {Kind::BINARY, "({0} / {1})", true}},
      {"RealDiv", {Kind::BINARY, "({0} / {1})", true}},
      {"Maximum", {Kind::BINARY, "tfa_max({0}, {1})", false}},
      {"Minimum", {Kind::BINARY, "tfa_min({0}, {1})", false}},
      {"SquaredDifference", {Kind::BINARY, "tfa_sqd({0}, {1})", false}},
      {"Pow", {Kind::BINARY, "pow({0}, {1})", true}},
      {"DivNoNan", {Kind::BINARY, "({1} == ({T})0 ? ({T})0 : {0} / {1})", true}},
  };
  return t;
}

const char* ctype(DType d) {
  switch (d) {
    case DType::F32: return "float";
    case DType::F64: return "double";
    case DType::I32: return "int";
    case DType::I64: return "long long";
    case DType::U8: return "unsigned char";
    default: return nullptr;
  }
}

bool value_dtype(DType d) { return d == DType::F32 || d == DType::F64 || d == DType::I32 || d == DType::I64; }

std::string fmt(const char* f, const std::vector<std::string>& args, const std::string& T) {
  std::string out;
  for (const char* p = f; *p; ++p) {
    if (*p == '{' && p[1] == 'T' && p[2] == '}') {
      out += T;
      p += 2;
    } else if (*p == '{' && p[1] >= '0' && p[1] <= '9' && p[2] == '}') {
      out += args.at(p[1] - '0');
      p += 2;
    } else {
      out += *p;
    }
  }
  return out;
}

std::vector<int64_t> nonunit(const std::vector<int64_t>& d) {
  std::vector<int64_t> r;
  for (auto x : d)
    if (x != 1) r.push_back(x);
  return r;
}

struct Finder {
  const FusionInput& in;
  const Graph& g;
  const Graph::Infos& infos;
  std::set<int> runtime_set;

  explicit Finder(const FusionInput& i) : in(i), g(*i.g), infos(*i.infos) {
    runtime_set.insert(i.runtime.begin(), i.runtime.end());
  }

  const TensorInfo& info(const TensorRef& r) const { return infos[r.node][r.index]; }

  // data operands of a fusible node (shape/axis/multiples operands are plan-time constants)
  std::vector<int> data_inputs(int n) const {
    const OpSpec& s = op_table().at(g.node(n).op);
    if (s.kind == Kind::BINARY) return {0, 1};
    return {0};
  }

  bool fusible(int n) const {
    const Node& nd = g.node(n);
    auto it = op_table().find(nd.op);
    if (it == op_table().end()) return false;
    const OpSpec& s = it->second;
    if (infos[n].size() != 1 || nd.num_outputs != 1) return false;
    const TensorInfo& o = infos[n][0];
    if (!value_dtype(o.dtype) || !o.shape.fully_known() || o.shape.rank() > 8 || o.value) return false;
    int64_t numel = 1;
    for (auto d : o.shape.dims) numel *= d;
    if (numel <= 0) return false;
    if (s.float_only && o.dtype != DType::F32 && o.dtype != DType::F64) return false;
    for (int k : data_inputs(n)) {
      if (k >= static_cast<int>(nd.inputs.size())) return false;
      const TensorInfo& ii = info(nd.inputs[k]);
      if (!ii.shape.fully_known() || ii.shape.rank() > o.shape.rank() + 8) return false;
      if (s.kind == Kind::CAST ? !(value_dtype(ii.dtype) || ii.dtype == DType::U8) : ii.dtype != o.dtype)
        return false;
    }
    const auto& od = o.shape.dims;
    if (nd.op == "BiasAdd" && nd.attr_s("data_format", std::string("NHWC")) == "NCHW") return false;
    if (s.kind == Kind::BINARY) {
      for (int k = 0; k < 2; ++k) {  // right-aligned broadcast into the output
        const auto& id = info(nd.inputs[k]).shape.dims;
        if (id.size() > od.size()) return false;
        for (size_t j = 0; j < id.size(); ++j)
          if (id[j] != 1 && id[j] != od[j + od.size() - id.size()]) return false;
      }
    }
    const auto& id0 = info(nd.inputs[0]).shape.dims;
    if (nd.op == "Reshape" && nonunit(id0) != nonunit(od)) return false;  // unit-dim reshapes only
    if (nd.op == "Tile") {
      if (id0.size() != od.size()) return false;
      for (size_t j = 0; j < od.size(); ++j)
        if (id0[j] != 1 && id0[j] != od[j]) return false;  // a pure broadcast, no repetition
    }
    if (nd.op == "BroadcastTo") {
      if (id0.size() > od.size()) return false;
      for (size_t j = 0; j < id0.size(); ++j)
        if (id0[j] != 1 && id0[j] != od[j + od.size() - id0.size()]) return false;
    }
    if ((nd.op == "Identity" || nd.op == "Snapshot" || nd.op == "StopGradient" || nd.op == "PreventGradient" ||
         nd.op == "Cast" || s.kind == Kind::UNARY) && id0 != od)
      return false;
    return true;
  }

  bool is_compute(int n) const {
    Kind k = op_table().at(g.node(n).op).kind;
    return k == Kind::UNARY || k == Kind::BINARY || k == Kind::CAST;
  }
  bool is_bcast(int n) const { return op_table().at(g.node(n).op).kind == Kind::BCAST; }
};

// ---------------------------------------------------------------- codegen
struct Gen {
  const Finder& f;
  const std::set<int>& members;
  std::vector<int64_t> root_dims;
  std::vector<std::string> stmts;  // element-loop body (leaf loads are "@Lk@" placeholders)
  std::map<std::pair<int, std::vector<int>>, std::string> memo;
  struct RawLeaf {
    TensorRef ref;
    DType dtype;
    std::vector<int64_t> coef;  // over root dims
  };
  std::vector<RawLeaf> leaves;
  std::map<std::pair<TensorRef, std::vector<int64_t>>, int> leaf_memo;
  int nvar = 0;
  std::ostringstream expr;

  Gen(const Finder& fi, const std::set<int>& m, std::vector<int64_t> rd)
      : f(fi), members(m), root_dims(std::move(rd)) {}

  std::string leaf(const TensorRef& r, const std::vector<int>& sel) {
    const TensorInfo& ti = f.info(r);
    const auto& d = ti.shape.dims;
    std::vector<int64_t> st(d.size(), 1);
    for (int j = static_cast<int>(d.size()) - 2; j >= 0; --j) st[j] = st[j + 1] * d[j + 1];
    std::vector<int64_t> coef(root_dims.size(), 0);
    for (size_t j = 0; j < d.size(); ++j)
      if (sel[j] >= 0 && d[j] != 1) coef[sel[j]] += st[j];
    auto key = std::make_pair(r, coef);
    auto it = leaf_memo.find(key);
    int idx;
    if (it != leaf_memo.end()) {
      idx = it->second;
    } else {
      idx = static_cast<int>(leaves.size());
      leaves.push_back({r, ti.dtype, coef});
      leaf_memo[key] = idx;
    }
    return "l" + std::to_string(idx);
  }

  std::string operand(const TensorRef& r, const std::vector<int>& sel) {
    if (r.index == 0 && members.count(r.node)) return value(r.node, sel);
    return leaf(r, sel);
  }

  // sel: for each dim of the node's output, the root dim it indexes (or -1 = index 0)
  std::string value(int n, const std::vector<int>& sel) {
    auto key = std::make_pair(n, sel);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    const Node& nd = f.g.node(n);
    const OpSpec& s = op_table().at(nd.op);
    const auto& od = f.infos[n][0].shape.dims;
    std::vector<std::string> args;
    auto operand_sel = [&](int k) {
      const auto& id = f.info(nd.inputs[k]).shape.dims;
      std::vector<int> si(id.size(), -1);
      if (nd.op == "ExpandDims") {
        int64_t a = f.infos[nd.inputs[1].node][nd.inputs[1].index].value
                        ? to_int_vector(*f.infos[nd.inputs[1].node][nd.inputs[1].index].value)[0]
                        : 0;
        if (a < 0) a += static_cast<int64_t>(od.size());
        for (size_t j = 0, o = 0; j < id.size(); ++j, ++o) {
          if (static_cast<int64_t>(o) == a) ++o;
          si[j] = sel[o];
        }
      } else if (nd.op == "Squeeze" || nd.op == "Reshape") {
        // the non-unit dims keep their order; unit input dims index 0
        std::vector<int> out_nonunit;
        for (size_t o = 0; o < od.size(); ++o)
          if (od[o] != 1) out_nonunit.push_back(sel[o]);
        size_t q = 0;
        for (size_t j = 0; j < id.size(); ++j) si[j] = id[j] == 1 ? -1 : out_nonunit.at(q++);
      } else {  // elementwise / broadcast: right-aligned
        for (size_t j = 0; j < id.size(); ++j) {
          size_t o = j + od.size() - id.size();
          si[j] = id[j] == 1 ? -1 : sel[o];
        }
      }
      return si;
    };
    for (int k : f.data_inputs(n)) args.push_back(operand(nd.inputs[k], operand_sel(k)));
    const std::string T = ctype(f.infos[n][0].dtype);
    std::string e;
    if (nd.op == "LeakyRelu") {
      std::ostringstream a;
      a.precision(17);
      a << nd.attr_f("alpha", 0.2f);
      e = "(" + args[0] + " >= (" + T + ")0 ? " + args[0] + " : " + args[0] + " * (" + T + ")" + a.str() + ")";
    } else {
      e = fmt(s.fmt, args, T);
    }
    std::string var = "v" + std::to_string(nvar++);
    stmts.push_back("const " + T + " " + var + " = " + e + ";");
    memo[key] = var;
    return var;
  }
};

// Drops unit dims, then merges neighbours that are contiguous for every
// array. With `barrier` > 0 dims [0, barrier) and [barrier, rank) collapse
// separately (rows and the reduced axis of a row reduction stay apart);
// returns the collapsed position of the barrier.
int collapse(std::vector<int64_t>& dims, std::vector<std::vector<int64_t>>& coefs, int barrier = 0) {
  auto one = [&](size_t a, size_t b, std::vector<int64_t>& md, std::vector<std::vector<int64_t>>& mc) {
    bool first = true;
    for (size_t p = a; p < b; ++p) {
      if (dims[p] == 1) continue;
      bool ok = !first;
      for (size_t k = 0; k < coefs.size() && ok; ++k) ok = mc[k].back() == coefs[k][p] * dims[p];
      if (ok) {
        md.back() *= dims[p];
        for (size_t k = 0; k < coefs.size(); ++k) mc[k].back() = coefs[k][p];
      } else {
        md.push_back(dims[p]);
        for (size_t k = 0; k < coefs.size(); ++k) mc[k].push_back(coefs[k][p]);
      }
      first = false;
    }
    if (first) {  // all unit dims: keep one
      md.push_back(1);
      for (size_t k = 0; k < coefs.size(); ++k) mc[k].push_back(0);
    }
  };
  std::vector<int64_t> md;
  std::vector<std::vector<int64_t>> mc(coefs.size());
  int pos = 0;
  if (barrier > 0) {
    one(0, barrier, md, mc);
    pos = static_cast<int>(md.size());
  }
  one(barrier, dims.size(), md, mc);
  dims = md;
  coefs = mc;
  return pos;
}

const char* I_T(bool idx64) { return idx64 ? "unsigned long long" : "unsigned int"; }

std::string preamble(const std::string& desc, bool idx64, int words) {
  std::ostringstream s;
  s << "// generated by tensorframes_amd (runtime/fusion.cpp): " << desc << "\n"
    << "typedef " << I_T(idx64) << " idx_t;\n"
    << "struct tfa_args { long long w[" << words << "]; };\n"
    << "template <typename T> __device__ __forceinline__ T tfa_max(T a, T b) {"
       " return (a != a || b != b) ? (a + b) : (a > b ? a : b); }\n"
    << "template <typename T> __device__ __forceinline__ T tfa_min(T a, T b) {"
       " return (a != a || b != b) ? (a + b) : (a < b ? a : b); }\n"
    << "template <typename T> __device__ __forceinline__ T tfa_sqd(T a, T b) { T d = a - b; return d * d; }\n";
  return s.str();
}

// word layout: [n][dims R][coef R per strided leaf][leaf ptrs][out ptrs]
struct Layout {
  int R, w_dims, w_coef, w_ptr, w_out, words;
  std::vector<int> strided;
};

Layout layout_of(const FusedRegion& r, int nout) {
  Layout L;
  L.R = static_cast<int>(r.dims.size());
  for (size_t k = 0; k < r.leaves.size(); ++k)
    if (r.leaves[k].kind == 2) L.strided.push_back(static_cast<int>(k));
  L.w_dims = 1;
  L.w_coef = 1 + L.R;
  L.w_ptr = L.w_coef + L.R * static_cast<int>(L.strided.size());
  L.w_out = L.w_ptr + static_cast<int>(r.leaves.size());
  L.words = L.w_out + nout;
  return L;
}

// declarations shared by both kernel kinds: dims, leaf pointers, strides
void emit_decls(std::ostringstream& s, const FusedRegion& r, const Layout& L, bool need_dims) {
  s << "  const idx_t n = (idx_t)a.w[0];\n";
  if (need_dims)
    for (int d = 0; d < L.R; ++d) s << "  const idx_t D" << d << " = (idx_t)a.w[" << (L.w_dims + d) << "];\n";
  for (size_t k = 0; k < r.leaves.size(); ++k) {
    const char* T = ctype(r.leaves[k].dtype);
    s << "  const " << T << "* __restrict__ p" << k << " = (const " << T << "*)a.w[" << (L.w_ptr + k) << "];\n";
  }
  for (size_t q = 0; q < L.strided.size(); ++q)
    for (int d = 0; d < L.R; ++d)
      s << "  const idx_t C" << L.strided[q] << "_" << d << " = (idx_t)a.w[" << (L.w_coef + q * L.R + d) << "];\n";
  for (size_t k = 0; k < r.leaves.size(); ++k)
    if (r.leaves[k].kind == 1) s << "  const " << ctype(r.leaves[k].dtype) << " s" << k << " = p" << k << "[0];\n";
}

// leaf loads + region statements for linear index `i`, with coordinates c0..c{R-1}
// already in scope when `have_coords`
void emit_body(std::ostringstream& s, const FusedRegion& r, const Layout& L, const Gen& gen, const char* ind,
               bool have_coords) {
  if (!L.strided.empty() && !have_coords) {
    s << ind << "idx_t rem = i;\n";
    for (int d = L.R - 1; d >= 1; --d)
      s << ind << "const idx_t q" << d << " = rem / D" << d << "; const idx_t c" << d << " = rem - q" << d
        << " * D" << d << "; rem = q" << d << ";\n";
    s << ind << "const idx_t c0 = rem;\n";
  }
  for (int k : L.strided) {
    s << ind << "const idx_t o" << k << " = ";
    for (int d = 0; d < L.R; ++d) s << (d ? " + " : "") << "c" << d << " * C" << k << "_" << d;
    s << ";\n";
  }
  for (size_t k = 0; k < r.leaves.size(); ++k) {
    s << ind << "const " << ctype(r.leaves[k].dtype) << " l" << k << " = ";
    if (r.leaves[k].kind == 0) s << "p" << k << "[i];\n";
    else if (r.leaves[k].kind == 1) s << "s" << k << ";\n";
    else s << "p" << k << "[o" << k << "];\n";
  }
  for (auto& st : gen.stmts) s << ind << st << "\n";
}

std::string generate_source(FusedRegion& r, const Gen& gen, const std::string& root_var, bool idx64) {
  Layout L = layout_of(r, 1);
  std::ostringstream s;
  s << preamble(r.expr, idx64, L.words)
    << "extern \"C\" __global__ void __launch_bounds__(" << kFusedBlock << ") " << r.entry << "(tfa_args a) {\n";
  emit_decls(s, r, L, !L.strided.empty());
  const char* TO = ctype(r.out_dtype);
  s << "  " << TO << "* __restrict__ po = (" << TO << "*)a.w[" << L.w_out << "];\n"
    << "  const idx_t base = (idx_t)blockIdx.x * " << (kFusedBlock * kFusedEPT) << " + threadIdx.x;\n"
    << "#pragma unroll\n"
    << "  for (int e = 0; e < " << kFusedEPT << "; ++e) {\n"
    << "    const idx_t i = base + (idx_t)e * " << kFusedBlock << ";\n"
    << "    if (i >= n) break;\n";
  emit_body(s, r, L, gen, "    ", false);
  s << "    po[i] = " << root_var << ";\n  }\n}\n";
  return s.str();
}

// Row reduction kernel: rows of the [outer, inner] view; one thread per row
// for short rows, one wave per row (shuffle tree) otherwise.
std::string generate_reduce_source(FusedRegion& r, const Gen* gen, const std::string& xvar, DType xdt,
                                   const std::vector<DType>& out_dt, bool idx64, bool wave) {
  Layout L = layout_of(r, static_cast<int>(r.outputs.size()));
  const bool fl = xdt == DType::F32 || xdt == DType::F64;
  const std::string T = ctype(xdt), A = fl ? "double" : "long long";
  std::ostringstream s;
  s << preamble(r.expr, idx64, L.words);
  s << "extern \"C\" __global__ void __launch_bounds__(256) " << r.entry << "(tfa_args a) {\n";
  emit_decls(s, r, L, !L.strided.empty());
  s << "  const idx_t outer = (idx_t)a.w[0];\n";  // w[0] carries the row count for reductions
  s << "  const idx_t inner = ";
  {
    // inner = product of the collapsed inner dims
    std::ostringstream e;
    for (int d = r.outer_rank; d < L.R; ++d) e << (d > r.outer_rank ? " * " : "") << "(idx_t)a.w[" << (L.w_dims + d) << "]";
    s << (e.str().empty() ? "1" : e.str()) << ";\n";
  }
  for (size_t k = 0; k < r.outputs.size(); ++k) {
    const char* TO = ctype(out_dt[k]);
    s << "  " << TO << "* __restrict__ y" << k << " = (" << TO << "*)a.w[" << (L.w_out + k) << "];\n";
  }
  if (wave) {
    s << "  const int lane = threadIdx.x & 63;\n"
      << "  const idx_t row = (idx_t)blockIdx.x * 4 + (threadIdx.x >> 6);\n"
      << "  if (row >= outer) return;\n";
  } else {
    s << "  const idx_t row = (idx_t)blockIdx.x * 256 + threadIdx.x;\n"
      << "  if (row >= outer) return;\n";
  }
  // accumulators
  for (size_t k = 0; k < r.red_ops.size(); ++k) {
    const std::string& op = r.red_ops[k];
    if (op == "Sum" || op == "Mean") s << "  " << A << " acc" << k << " = 0;\n";
    else if (op == "Prod") s << "  " << A << " acc" << k << " = 1;\n";
    else if (op == "Min") s << "  " << A << " acc" << k << " = " << (fl ? "__builtin_huge_val()" : "0x7fffffffffffffffLL") << ";\n";
    else if (op == "Max") s << "  " << A << " acc" << k << " = " << (fl ? "-__builtin_huge_val()" : "(-0x7fffffffffffffffLL - 1)") << ";\n";
    else s << "  " << T << " best" << k << " = 0; idx_t bi" << k << " = (idx_t)-1;\n";  // ArgMin / ArgMax
  }
  // coordinates of the row over the outer collapsed dims
  const bool coords = !L.strided.empty();
  if (coords) {
    s << "  idx_t rr = row;\n";
    for (int d = r.outer_rank - 1; d >= 1; --d)
      s << "  const idx_t c" << d << " = rr % D" << d << "; rr /= D" << d << ";\n";
    if (r.outer_rank >= 1) s << "  const idx_t c0 = rr;\n";
  }
  s << "  for (idx_t j = " << (wave ? "(idx_t)lane" : "0") << "; j < inner; j += " << (wave ? "64" : "1") << ") {\n"
    << "    const idx_t i = row * inner + j;\n";
  if (coords) {
    s << "    idx_t jj = j;\n";
    for (int d = L.R - 1; d > r.outer_rank; --d)
      s << "    const idx_t c" << d << " = jj % D" << d << "; jj /= D" << d << ";\n";
    if (L.R > r.outer_rank) s << "    const idx_t c" << r.outer_rank << " = jj;\n";
  }
  emit_body(s, r, L, *gen, "    ", true);
  s << "    const " << T << " x = " << xvar << ";\n";
  for (size_t k = 0; k < r.red_ops.size(); ++k) {
    const std::string& op = r.red_ops[k];
    if (op == "Sum" || op == "Mean") s << "    acc" << k << " += (" << A << ")x;\n";
    else if (op == "Prod") s << "    acc" << k << " *= (" << A << ")x;\n";
    else if (op == "Min") s << "    acc" << k << " = (" << A << ")x < acc" << k << " ? (" << A << ")x : acc" << k << ";\n";
    else if (op == "Max") s << "    acc" << k << " = (" << A << ")x > acc" << k << " ? (" << A << ")x : acc" << k << ";\n";
    else {
      const char* cmp = op == "ArgMin" ? "<" : ">";
      s << "    if (bi" << k << " == (idx_t)-1 || x " << cmp << " best" << k << ") { best" << k << " = x; bi" << k
        << " = j; }\n";
    }
  }
  s << "  }\n";
  if (wave) {
    s << "#pragma unroll\n  for (int off = 32; off > 0; off >>= 1) {\n";
    for (size_t k = 0; k < r.red_ops.size(); ++k) {
      const std::string& op = r.red_ops[k];
      if (op == "Sum" || op == "Mean") s << "    acc" << k << " += __shfl_xor(acc" << k << ", off, 64);\n";
      else if (op == "Prod") s << "    acc" << k << " *= __shfl_xor(acc" << k << ", off, 64);\n";
      else if (op == "Min" || op == "Max") {
        const char* cmp = op == "Min" ? "<" : ">";
        s << "    { const " << A << " o = __shfl_xor(acc" << k << ", off, 64); acc" << k << " = o " << cmp << " acc" << k
          << " ? o : acc" << k << "; }\n";
      } else {
        // first index among equal values; an empty lane (bi == -1) never wins
        const char* cmp = op == "ArgMin" ? "<" : ">";
        s << "    { const " << T << " ob = __shfl_xor(best" << k << ", off, 64); const idx_t oi = __shfl_xor(bi" << k
          << ", off, 64);\n"
          << "      if (oi != (idx_t)-1 && (bi" << k << " == (idx_t)-1 || ob " << cmp << " best" << k << " || (ob == best"
          << k << " && oi < bi" << k << "))) { best" << k << " = ob; bi" << k << " = oi; } }\n";
      }
    }
    s << "  }\n  if (lane != 0) return;\n";
  }
  for (size_t k = 0; k < r.red_ops.size(); ++k) {
    const std::string& op = r.red_ops[k];
    const char* TO = ctype(out_dt[k]);
    if (op == "Mean") s << "  y" << k << "[row] = (" << TO << ")(acc" << k << " / (" << A << ")inner);\n";
    else if (op == "ArgMin" || op == "ArgMax") s << "  y" << k << "[row] = (" << TO << ")bi" << k << ";\n";
    else s << "  y" << k << "[row] = (" << TO << ")acc" << k << ";\n";
  }
  s << "}\n";
  return s.str();
}

bool is_reduction_op(const std::string& op) {
  return op == "Sum" || op == "Mean" || op == "Min" || op == "Max" || op == "Prod" || op == "ArgMin" ||
         op == "ArgMax";
}

}  // namespace

bool fusible_op(const std::string& op) { return op_table().count(op) > 0; }

bool fusion_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TFA_FUSION");
    return !(e && e[0] == '0');
  }();
  return on;
}

namespace {

// Grows a region from `reg` through fusible producers whose every consumer is
// in the region or in `also` (the reductions a prologue feeds).
void grow(const Finder& f, const FusionInput& in, std::set<int>& reg, const std::set<int>& assigned,
          const std::set<int>& also) {
  for (bool grew = true; grew;) {
    grew = false;
    for (int m : std::vector<int>(reg.begin(), reg.end())) {
      for (int k : f.data_inputs(m)) {
        const TensorRef r = f.g.node(m).inputs[k];
        const int p = r.node;
        if (reg.count(p) || assigned.count(p) || in.excluded.count(p) || !f.runtime_set.count(p)) continue;
        if (r.index != 0 || in.fetched.count(TensorRef{p, 0}) || !f.fusible(p)) continue;
        auto cit = in.consumers.find(p);
        bool all_in = cit != in.consumers.end();
        if (all_in)
          for (int c : cit->second) all_in = all_in && (reg.count(c) || also.count(c));
        if (!all_in) continue;
        reg.insert(p);
        grew = true;
      }
    }
  }
}

// leaves of a Gen -> FusedLeaf, with the index space collapsed
void finish_leaves(const Finder& f, FusedRegion& r, const Gen& gen, const std::vector<int64_t>& xdims,
                   int barrier, int64_t* max_leaf) {
  std::vector<std::vector<int64_t>> coefs;
  std::vector<int64_t> st(xdims.size(), 1);
  for (int j = static_cast<int>(xdims.size()) - 2; j >= 0; --j) st[j] = st[j + 1] * xdims[j + 1];
  coefs.push_back(st);
  for (auto& l : gen.leaves) coefs.push_back(l.coef);
  std::vector<int64_t> dims = xdims;
  if (dims.empty()) {
    dims = {1};
    for (auto& c : coefs) c = {0};
  }
  r.outer_rank = collapse(dims, coefs, barrier);
  r.dims = dims;
  *max_leaf = 0;
  for (size_t k = 0; k < gen.leaves.size(); ++k) {
    FusedLeaf fl;
    fl.ref = gen.leaves[k].ref;
    fl.dtype = gen.leaves[k].dtype;
    fl.coef = coefs[k + 1];
    bool zero = std::all_of(fl.coef.begin(), fl.coef.end(), [](int64_t c) { return c == 0; });
    fl.kind = fl.coef == coefs[0] ? 0 : (zero ? 1 : 2);
    int64_t ln = 1;
    for (auto d : f.info(fl.ref).shape.dims) ln *= d;
    *max_leaf = std::max(*max_leaf, ln);
    r.leaves.push_back(fl);
  }
}

std::string ops_desc(const Graph& g, const std::vector<int>& nodes) {
  std::ostringstream e;
  for (size_t i = 0; i < nodes.size(); ++i) e << (i ? " " : "") << g.node(nodes[i]).op;
  return e.str();
}

}  // namespace

std::vector<FusedRegion> find_fused_regions(const FusionInput& in) {
  Finder f(in);
  std::vector<FusedRegion> out;
  std::set<int> assigned;
  std::map<int, int> pos;
  for (size_t i = 0; i < in.runtime.size(); ++i) pos[in.runtime[i]] = static_cast<int>(i);
  auto by_pos = [&](int a, int b) { return pos[a] < pos[b]; };

  // ---- pass 1: row reductions (sibling reductions of one tensor share a pass)
  std::map<std::pair<TensorRef, int>, std::vector<int>> groups;  // (X, first reduced axis) -> reductions
  for (int n : in.runtime) {
    const Node& nd = f.g.node(n);
    if (!is_reduction_op(nd.op) || in.excluded.count(n) || nd.inputs.size() != 2) continue;
    const TensorInfo& xi = f.info(nd.inputs[0]);
    const TensorInfo& ai = f.info(nd.inputs[1]);
    const TensorInfo& oi = f.infos[n][0];
    if (!value_dtype(xi.dtype) || !xi.shape.fully_known() || !ai.value || !oi.shape.fully_known()) continue;
    if (nd.op == "Mean" && !(xi.dtype == DType::F32 || xi.dtype == DType::F64) && false) continue;
    const int rank = xi.shape.rank();
    if (rank < 2) continue;
    std::vector<int64_t> axes = to_int_vector(*ai.value);
    if (axes.empty()) continue;
    for (auto& a : axes) a = a < 0 ? a + rank : a;
    std::sort(axes.begin(), axes.end());
    axes.erase(std::unique(axes.begin(), axes.end()), axes.end());
    // reduced axes must be the trailing ones [k, rank)
    const int k = static_cast<int>(axes.front());
    if (axes.back() != rank - 1 || static_cast<int>(axes.size()) != rank - k || k < 1) continue;
    if ((nd.op == "ArgMin" || nd.op == "ArgMax") && axes.size() != 1) continue;
    int64_t outer = 1, inner = 1;
    for (int d = 0; d < k; ++d) outer *= xi.shape.dims[d];
    for (int d = k; d < rank; ++d) inner *= xi.shape.dims[d];
    // long rows / few rows stay on the tuned block-reduction kernels
    if (outer < 256 || inner < 1 || inner > (1 << 16)) continue;
    groups[{nd.inputs[0], k}].push_back(n);
  }
  for (auto& [key, reds] : groups) {
    const TensorRef xref = key.first;
    const int k = key.second;
    std::sort(reds.begin(), reds.end(), by_pos);
    std::set<int> red_set(reds.begin(), reds.end());
    const TensorInfo& xi = f.info(xref);
    FusedRegion r;
    r.kind = 1;
    r.outputs = reds;
    for (int n : reds) r.red_ops.push_back(f.g.node(n).op);
    r.outer = 1;
    r.inner = 1;
    for (int d = 0; d < k; ++d) r.outer *= xi.shape.dims[d];
    for (int d = k; d < xi.shape.rank(); ++d) r.inner *= xi.shape.dims[d];
    r.numel = r.outer * r.inner;
    r.out_dtype = xi.dtype;
    // prologue: X's producer chain when all of X's consumers are these reductions
    const int p = xref.node;
    bool prologue = xref.index == 0 && f.runtime_set.count(p) && !assigned.count(p) && !in.excluded.count(p) &&
                    !in.fetched.count(TensorRef{p, 0}) && f.fusible(p);
    if (prologue) {
      auto cit = in.consumers.find(p);
      prologue = cit != in.consumers.end();
      if (prologue)
        for (int c : cit->second) prologue = prologue && red_set.count(c);
    }
    std::vector<int64_t> xdims = xi.shape.dims;
    std::string xvar;
    std::unique_ptr<Gen> gen;
    std::set<int> reg;
    if (prologue) {
      reg.insert(p);
      grow(f, in, reg, assigned, red_set);
      gen = std::make_unique<Gen>(f, reg, xdims);
      std::vector<int> sel(xdims.size());
      for (size_t d = 0; d < sel.size(); ++d) sel[d] = static_cast<int>(d);
      xvar = gen->value(p, sel);
      r.root = p;
      r.nodes.assign(reg.begin(), reg.end());
      std::sort(r.nodes.begin(), r.nodes.end(), by_pos);
      for (int m : reg) r.compute_ops += f.is_compute(m);
    } else {
      // a plain leaf: X read directly (still one pass for all siblings)
      gen = std::make_unique<Gen>(f, reg, xdims);
      std::vector<int> sel(xdims.size());
      for (size_t d = 0; d < sel.size(); ++d) sel[d] = static_cast<int>(d);
      xvar = gen->leaf(xref, sel);
    }
    // worth a generated kernel: a prologue, or several sibling reductions
    if (!prologue && reds.size() < 2) continue;
    int64_t max_leaf = 0;
    finish_leaves(f, r, *gen, xdims, k, &max_leaf);
    std::vector<DType> odt;
    for (int n : reds) odt.push_back(f.infos[n][0].dtype);
    bool ok = true;
    for (auto d : odt) ok = ok && value_dtype(d);
    if (!ok) continue;
    r.expr = (prologue ? ops_desc(f.g, r.nodes) + " -> " : std::string()) + ops_desc(f.g, reds);
    const bool idx64 = std::max(r.numel, max_leaf) >= (int64_t(1) << 31);
    const bool wave = r.inner > 16;
    r.entry = "tfa_fused_rowred";
    r.block = 256;
    r.grid = wave ? (r.outer + 3) / 4 : (r.outer + 255) / 256;
    r.source = generate_reduce_source(r, gen.get(), xvar, xi.dtype, odt, idx64, wave);
    assigned.insert(reg.begin(), reg.end());
    assigned.insert(reds.begin(), reds.end());
    out.push_back(std::move(r));
  }

  // ---- pass 2: elementwise regions
  for (auto it = in.runtime.rbegin(); it != in.runtime.rend(); ++it) {
    const int root = *it;
    if (in.excluded.count(root) || assigned.count(root) || !f.fusible(root)) continue;
    std::set<int> reg{root};
    grow(f, in, reg, assigned, {});
    int compute = 0, bcast = 0;
    for (int m : reg) {
      compute += f.is_compute(m);
      bcast += f.is_bcast(m);
    }
    if (!(compute >= 2 || (compute >= 1 && bcast >= 1))) continue;

    FusedRegion r;
    r.kind = 0;
    r.root = root;
    r.outputs = {root};
    r.nodes.assign(reg.begin(), reg.end());
    std::sort(r.nodes.begin(), r.nodes.end(), by_pos);
    r.compute_ops = compute;
    const TensorInfo& ro = f.infos[root][0];
    r.out_dtype = ro.dtype;
    std::vector<int64_t> root_dims = ro.shape.dims;
    r.numel = 1;
    for (auto d : root_dims) r.numel *= d;
    Gen gen(f, reg, root_dims);
    std::vector<int> sel(root_dims.size());
    for (size_t d = 0; d < sel.size(); ++d) sel[d] = static_cast<int>(d);
    std::string root_var = gen.value(root, sel);
    int64_t max_leaf = 0;
    finish_leaves(f, r, gen, root_dims, 0, &max_leaf);
    r.expr = ops_desc(f.g, r.nodes);
    const bool idx64 = std::max(r.numel, max_leaf) >= (int64_t(1) << 31);
    r.entry = "tfa_fused";
    r.block = kFusedBlock;
    r.grid = (r.numel + int64_t(kFusedBlock) * kFusedEPT - 1) / (int64_t(kFusedBlock) * kFusedEPT);
    r.source = generate_source(r, gen, root_var, idx64);
    assigned.insert(reg.begin(), reg.end());
    out.push_back(std::move(r));
  }
  // the executor places each region at its first output's step
  std::sort(out.begin(), out.end(),
            [&](const FusedRegion& a, const FusedRegion& b) { return pos[a.outputs.front()] < pos[b.outputs.front()]; });
  return out;
}

std::vector<int64_t> fused_args(const FusedRegion& r, const std::vector<const void*>& leaf_ptrs,
                                const std::vector<void*>& outs) {
  std::vector<int64_t> w;
  w.push_back(r.kind == 1 ? r.outer : r.numel);
  for (auto d : r.dims) w.push_back(d);
  for (auto& l : r.leaves)
    if (l.kind == 2)
      for (auto c : l.coef) w.push_back(c);
  TFA_CHECK(leaf_ptrs.size() == r.leaves.size(), "fused kernel: expected ", r.leaves.size(), " inputs, got ",
            leaf_ptrs.size());
  TFA_CHECK(outs.size() == r.outputs.size(), "fused kernel: expected ", r.outputs.size(), " outputs, got ",
            outs.size());
  for (auto p : leaf_ptrs) w.push_back(static_cast<int64_t>(reinterpret_cast<uintptr_t>(p)));
  for (auto p : outs) w.push_back(static_cast<int64_t>(reinterpret_cast<uintptr_t>(p)));
  return w;
}

}  // namespace tfa

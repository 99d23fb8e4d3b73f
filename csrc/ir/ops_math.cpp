// Math ops: elementwise unary/binary, reductions, arg-reductions, MatMul,
// segment reductions.
//
// Op set: every op the reference's DSL, tests and examples dispatch
// (reference: src/main/scala/org/tensorframes/dsl/DslImpl.scala:168-188,
// src/main/python/tensorframes_snippets/kmeans_demo.py:31-42,76-79,131-138,
// geom_mean.py:30-46) plus the natural extensions of each family.
#include <cmath>
#include <limits>

#include "ops_common.h"

namespace tfa {

namespace {

// ------------------------------------------------------------------ binary
struct BinInfo {
  k::BinOp op;
  bool is_cmp;
};

at::Tensor cpu_binary(k::BinOp op, const at::Tensor& a, const at::Tensor& b) {
  bool is_int = !at::isFloatingType(a.scalar_type());
  switch (op) {
    case k::BinOp::ADD: return at::add(a, b);
    case k::BinOp::SUB: return at::sub(a, b);
    case k::BinOp::MUL: return at::mul(a, b);
    case k::BinOp::DIV: return is_int ? at::div(a, b, "trunc") : at::div(a, b);
    case k::BinOp::FLOORDIV: return is_int ? at::div(a, b, "floor") : at::floor(at::div(a, b));
    case k::BinOp::FLOORMOD: return at::remainder(a, b);
    case k::BinOp::TRUNCMOD: return at::fmod(a, b);
    case k::BinOp::MAX: return at::maximum(a, b);
    case k::BinOp::MIN: return at::minimum(a, b);
    case k::BinOp::POW: return at::pow(a, b).to(a.scalar_type());
    case k::BinOp::SQDIFF: { at::Tensor d = at::sub(a, b); return at::mul(d, d); }
    case k::BinOp::EQ: return at::eq(a, b);
    case k::BinOp::NE: return at::ne(a, b);
    case k::BinOp::LT: return at::lt(a, b);
    case k::BinOp::LE: return at::le(a, b);
    case k::BinOp::GT: return at::gt(a, b);
    case k::BinOp::GE: return at::ge(a, b);
    case k::BinOp::LAND: return at::logical_and(a, b);
    case k::BinOp::LOR: return at::logical_or(a, b);
    case k::BinOp::ATAN2: return at::atan2(a, b);
    case k::BinOp::DIVNONAN: {
      at::Tensor q = at::div(a, b);
      return at::where(b == 0, at::zeros_like(q), q);
    }
  }
  return a;
}

bool is_cmp(k::BinOp op) {
  return op == k::BinOp::EQ || op == k::BinOp::NE || op == k::BinOp::LT || op == k::BinOp::LE ||
         op == k::BinOp::GT || op == k::BinOp::GE || op == k::BinOp::LAND || op == k::BinOp::LOR;
}

}  // namespace

// shared with ops_extra.cpp (ClipByValue)
void gpu_binary(ExecCtx& c, k::BinOp op, const at::Tensor& a0, const at::Tensor& b0) {
  at::Tensor a = materialize(c, a0), b = materialize(c, b0);
  const auto& od = c.out_shape().dims;
  at::Tensor out = c.alloc_out(0);
  int64_t n = out.numel();
  c.out[0] = out;
  if (n == 0) return;
  DType dt = dt_of(a);
  int mode = 4;
  int64_t inner = 1;
  k::Bcast bc;
  bool a_full = a.numel() == n && a.sizes().vec() == od;
  bool b_full = b.numel() == n && b.sizes().vec() == od;
  if (a_full && b_full) mode = 0;
  else if (a_full && b.numel() == 1) mode = 1;
  else if (b_full && a.numel() == 1) mode = 2;
  else if (a_full && !od.empty() && b.numel() == od.back() && b.size(-1) == od.back() &&
           b.numel() > 1) {
    mode = 3;
    inner = od.back();
  }
  if (mode == 4) bc = make_bcast(od, a, b);
  k::binary(op, dt, a.data_ptr(), b.data_ptr(), out.data_ptr(), n, mode, inner,
            mode == 4 ? &bc : nullptr, stream_of(c));
}

namespace {

OpDef make_binary(k::BinOp op) {
  OpDef d;
  d.infer = [op](InferCtx& c) {
    const TensorInfo& a = c.input(0);
    const TensorInfo& b = c.input(1);
    TFA_CHECK(a.dtype == b.dtype, "operands have different dtypes: ", dtype_name(a.dtype), " vs ",
              dtype_name(b.dtype), " (no implicit casting)");
    c.set(0, is_cmp(op) ? DType::BOOL : a.dtype, broadcast_shapes(a.shape, b.shape));
  };
  d.rows = [](InferCtx& c) { c.rows_elementwise(); };
  d.compute = [op](ExecCtx& c) {
    if (!c.gpu) {
      c.out[0] = cpu_binary(op, c.input(0), c.input(1)).expand(c.out_shape().dims).contiguous();
      return;
    }
    require_gpu_dtype(c.input(0), {at::kFloat, at::kDouble, at::kInt, at::kLong, at::kBool}, c.node.op.c_str());
    gpu_binary(c, op, c.input(0), c.input(1));
  };
  return d;
}

// ------------------------------------------------------------------ unary
at::Tensor cpu_unary(k::UnOp op, const at::Tensor& x) {
  switch (op) {
    case k::UnOp::NEG: return at::neg(x);
    case k::UnOp::ABS: return at::abs(x);
    case k::UnOp::SQUARE: return at::mul(x, x);
    case k::UnOp::SQRT: return at::sqrt(x);
    case k::UnOp::RSQRT: return at::rsqrt(x);
    case k::UnOp::EXP: return at::exp(x);
    case k::UnOp::LOG: return at::log(x);
    case k::UnOp::LOG1P: return at::log1p(x);
    case k::UnOp::EXPM1: return at::expm1(x);
    case k::UnOp::RECIP:
      return at::isFloatingType(x.scalar_type()) ? at::reciprocal(x) : at::div(at::ones_like(x), x, "trunc");
    case k::UnOp::RELU: return at::clamp_min(x, 0);
    case k::UnOp::RELU6: return at::clamp(x, 0, 6);
    case k::UnOp::ELU: return at::elu(x);
    case k::UnOp::SELU: return at::selu(x);
    case k::UnOp::SIGMOID: return at::sigmoid(x);
    case k::UnOp::TANH: return at::tanh(x);
    case k::UnOp::SOFTPLUS: return at::softplus(x);
    case k::UnOp::SOFTSIGN: return at::div(x, at::abs(x) + 1);
    case k::UnOp::FLOOR: return at::floor(x);
    case k::UnOp::CEIL: return at::ceil(x);
    case k::UnOp::ROUND: return at::round(x);
    case k::UnOp::SIGN: return at::sign(x);
    case k::UnOp::SIN: return at::sin(x);
    case k::UnOp::COS: return at::cos(x);
    case k::UnOp::TAN: return at::tan(x);
    case k::UnOp::NOT: return at::logical_not(x);
    case k::UnOp::IDENTITY: return x;
    case k::UnOp::ERF: return at::erf(x);
    case k::UnOp::ISNAN: return at::isnan(x);
    case k::UnOp::ISINF: return at::isinf(x);
    case k::UnOp::ISFINITE: return at::isfinite(x);
  }
  return x;
}

OpDef make_unary(k::UnOp op) {
  OpDef d;
  bool to_bool = op == k::UnOp::ISNAN || op == k::UnOp::ISINF || op == k::UnOp::ISFINITE;
  d.infer = [to_bool](InferCtx& c) { c.set(0, to_bool ? DType::BOOL : c.input(0).dtype, c.input(0).shape); };
  d.rows = [](InferCtx& c) { c.rows_like(0); };
  d.compute = [op](ExecCtx& c) {
    if (!c.gpu) { c.out[0] = cpu_unary(op, c.input(0)).contiguous(); return; }
    require_gpu_dtype(c.input(0), {at::kFloat, at::kDouble, at::kInt, at::kLong, at::kBool}, c.node.op.c_str());
    at::Tensor x = materialize(c, c.input(0));
    c.out[0] = c.alloc_out(0);
    if (x.numel()) k::unary(op, dt_of(x), x.data_ptr(), c.out[0].data_ptr(), x.numel(), stream_of(c));
  };
  return d;
}

// ------------------------------------------------------------------ reductions
std::vector<int64_t> norm_axes(std::vector<int64_t> axes, int64_t rank) {
  for (auto& a : axes) a = norm_axis(a, rank, "reduction axis");
  std::sort(axes.begin(), axes.end());
  axes.erase(std::unique(axes.begin(), axes.end()), axes.end());
  return axes;
}

bool keep_dims(const Node& n) {
  if (n.has_attr("keep_dims")) return n.attr_b("keep_dims");
  return n.attr_b("keepdims", false);
}

at::Tensor cpu_reduce(k::RedOp op, const at::Tensor& x, const std::vector<int64_t>& axes, bool keep) {
  if (axes.empty()) return x;
  at::ScalarType st = x.scalar_type();
  switch (op) {
    case k::RedOp::SUM: return at::sum(x, axes, keep, st);
    case k::RedOp::PROD: {
      at::Tensor r = x;
      for (auto it = axes.rbegin(); it != axes.rend(); ++it) r = at::prod(r, *it, true, st);
      if (!keep) r = r.squeeze(axes);
      return r;
    }
    case k::RedOp::MIN: return at::amin(x, axes, keep);
    case k::RedOp::MAX: return at::amax(x, axes, keep);
    case k::RedOp::MEAN: {
      if (at::isFloatingType(st)) return at::mean(x, axes, keep);
      int64_t cnt = 1;
      for (auto a : axes) cnt *= x.size(a);
      return at::div(at::sum(x, axes, keep, st), cnt, "trunc").to(st);
    }
    case k::RedOp::ALL: {
      at::Tensor r = x.to(at::kBool);
      for (auto it = axes.rbegin(); it != axes.rend(); ++it) r = at::all(r, *it, true);
      if (!keep) r = r.squeeze(axes);
      return r;
    }
    case k::RedOp::ANY: {
      at::Tensor r = x.to(at::kBool);
      for (auto it = axes.rbegin(); it != axes.rend(); ++it) r = at::any(r, *it, true);
      if (!keep) r = r.squeeze(axes);
      return r;
    }
  }
  return x;
}

// Reduce on device: make reduced axes contiguous (one transpose copy if needed),
// then run the [outer, r, inner] kernel.
at::Tensor gpu_reduce(ExecCtx& c, k::RedOp op, const at::Tensor& x0, const std::vector<int64_t>& axes) {
  at::Tensor x = materialize(c, x0);
  int64_t rank = x.dim();
  bool contiguous_axes = true;
  for (size_t i = 1; i < axes.size(); ++i)
    if (axes[i] != axes[i - 1] + 1) contiguous_axes = false;
  std::vector<int64_t> kept;
  for (int64_t i = 0; i < rank; ++i)
    if (!std::count(axes.begin(), axes.end(), i)) kept.push_back(i);
  int64_t outer = 1, r = 1, inner = 1;
  if (!contiguous_axes) {
    // permute to [kept..., axes...]
    std::vector<int64_t> perm = kept;
    perm.insert(perm.end(), axes.begin(), axes.end());
    x = materialize(c, x.permute(perm));
    for (auto k2 : kept) outer *= x0.size(k2);
    for (auto a : axes) r *= x0.size(a);
  } else {
    for (int64_t i = 0; i < axes.front(); ++i) outer *= x.size(i);
    for (auto a : axes) r *= x.size(a);
    for (int64_t i = axes.back() + 1; i < rank; ++i) inner *= x.size(i);
  }
  DType dt = dt_of(x);
  at::Tensor out = c.alloc_out(0);
  if (out.numel() == 0) return out;
  size_t ws = k::reduce_workspace_bytes(dt, outer, r, inner);
  at::Tensor work;
  if (ws) work = c.alloc({static_cast<int64_t>(ws)}, x.options().dtype(at::kByte));
  k::reduce(op, dt, x.data_ptr(), out.data_ptr(), outer, r, inner, ws ? work.data_ptr() : nullptr,
            stream_of(c));
  return out;
}

OpDef make_reduce(k::RedOp op) {
  OpDef d;
  d.host_inputs = {1};
  d.infer = [op](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    DType dt = (op == k::RedOp::ALL || op == k::RedOp::ANY) ? DType::BOOL : x.dtype;
    auto av = c.ivalue(1);
    bool keep = keep_dims(c.node);
    if (x.shape.unknown_rank) { c.set(0, dt, Shape::unknown()); return; }
    int rk = x.shape.rank();
    if (!av) {
      c.set(0, dt, keep ? Shape(std::vector<int64_t>(rk, -1)) : Shape::unknown());
      return;
    }
    std::vector<int64_t> axes = norm_axes(*av, std::max(rk, 1));
    if (rk == 0) axes.clear();
    std::vector<int64_t> d;
    for (int i = 0; i < rk; ++i) {
      bool red = std::count(axes.begin(), axes.end(), i) > 0;
      if (!red) d.push_back(x.shape.dims[i]);
      else if (keep) d.push_back(1);
    }
    c.set(0, dt, Shape(d));
  };
  d.rows = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    if (c.all_const()) { c.out[0].row = RowClass::CONST; return; }
    auto av = c.ivalue(1);
    if (x.row != RowClass::ROW || !av || x.shape.rank() < 1) { c.out[0].row = RowClass::MIXED; return; }
    for (auto a : norm_axes(*av, x.shape.rank()))
      if (a == 0) { c.out[0].row = RowClass::MIXED; return; }
    c.out[0].row = RowClass::ROW;
  };
  d.compute = [op](ExecCtx& c) {
    at::Tensor x = c.input(0);
    std::vector<int64_t> axes = norm_axes(c.host_ivalue(1), std::max<int64_t>(x.dim(), 1));
    if (x.dim() == 0) axes.clear();
    bool keep = keep_dims(c.node);
    if (!c.gpu) {
      at::Tensor r = cpu_reduce(op, x, axes, keep);
      if (op == k::RedOp::ALL || op == k::RedOp::ANY) r = r.to(at::kBool);
      c.out[0] = r.reshape(c.out_shape().dims).contiguous();
      return;
    }
    if (axes.empty() || x.numel() == 0) {
      if (x.numel() == 0 && !axes.empty()) {
        // reduction over an empty axis: identity element
        double ident = 0;
        if (op == k::RedOp::PROD || op == k::RedOp::ALL) ident = 1;
        if (op == k::RedOp::MIN) ident = std::numeric_limits<double>::infinity();
        if (op == k::RedOp::MAX) ident = -std::numeric_limits<double>::infinity();
        if (op == k::RedOp::MEAN) ident = std::nan("");
        c.out[0] = c.alloc_out(0);
        k::fill(c.out_dtype(), c.out[0].data_ptr(), c.out[0].numel(), ident, stream_of(c));
        return;
      }
      c.out[0] = materialize(c, x).reshape(c.out_shape().dims);
      return;
    }
    require_gpu_dtype(x, {at::kFloat, at::kDouble, at::kInt, at::kLong, at::kBool}, c.node.op.c_str());
    at::Tensor xin = x;
    if (op == k::RedOp::ALL || op == k::RedOp::ANY) TFA_CHECK(x.scalar_type() == at::kBool, c.node.op, " needs bool input");
    c.out[0] = gpu_reduce(c, op, xin, axes).reshape(c.out_shape().dims);
  };
  return d;
}

// ------------------------------------------------------------------ argmin / argmax
OpDef make_argreduce(bool is_min) {
  OpDef d;
  d.host_inputs = {1};
  d.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    DType ot = c.node.attr_type("output_type", DType::I64);
    auto av = c.ivalue(1);
    if (x.shape.unknown_rank || !av) { c.set(0, ot, Shape::unknown()); return; }
    int64_t ax = norm_axis((*av)[0], x.shape.rank());
    std::vector<int64_t> dd = x.shape.dims;
    dd.erase(dd.begin() + ax);
    c.set(0, ot, Shape(dd));
  };
  d.rows = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    if (c.all_const()) { c.out[0].row = RowClass::CONST; return; }
    auto av = c.ivalue(1);
    bool ok = x.row == RowClass::ROW && av && x.shape.rank() >= 2 && norm_axis((*av)[0], x.shape.rank()) != 0;
    c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  d.compute = [is_min](ExecCtx& c) {
    at::Tensor x = c.input(0);
    int64_t ax = norm_axis(c.host_ivalue(1)[0], x.dim());
    if (!c.gpu) {
      at::Tensor r = is_min ? at::argmin(x, ax) : at::argmax(x, ax);
      c.out[0] = r.to(to_scalar_type(c.out_dtype()));
      return;
    }
    require_gpu_dtype(x, {at::kFloat, at::kDouble, at::kInt, at::kLong}, c.node.op.c_str());
    at::Tensor xc = materialize(c, x);
    int64_t outer = 1, inner = 1;
    for (int64_t i = 0; i < ax; ++i) outer *= xc.size(i);
    for (int64_t i = ax + 1; i < xc.dim(); ++i) inner *= xc.size(i);
    c.out[0] = c.alloc_out(0);
    if (c.out[0].numel())
      k::argreduce(is_min, dt_of(xc), c.out_dtype(), xc.data_ptr(), c.out[0].data_ptr(), outer,
                   xc.size(ax), inner, stream_of(c));
  };
  return d;
}

// ------------------------------------------------------------------ MatMul
void infer_matmul(InferCtx& c, bool batch) {
  const TensorInfo& a = c.input(0);
  const TensorInfo& b = c.input(1);
  TFA_CHECK(a.dtype == b.dtype, "MatMul operands have different dtypes: ", dtype_name(a.dtype),
            " vs ", dtype_name(b.dtype));
  bool ta = batch ? c.node.attr_b("adj_x", false) : c.node.attr_b("transpose_a", false);
  bool tb = batch ? c.node.attr_b("adj_y", false) : c.node.attr_b("transpose_b", false);
  if (a.shape.unknown_rank || b.shape.unknown_rank) {
    c.set(0, a.dtype, batch ? Shape::unknown() : Shape({-1, -1}));
    return;
  }
  int ra = a.shape.rank(), rb = b.shape.rank();
  TFA_CHECK(ra >= 2 && rb >= 2, "MatMul operands must have rank >= 2, got ", a.shape.str(), " and ", b.shape.str());
  if (!batch) TFA_CHECK(ra == 2 && rb == 2, "MatMul operands must be rank 2, got ", a.shape.str(), " and ", b.shape.str());
  int64_t m = a.shape.dims[ta ? ra - 1 : ra - 2], ka = a.shape.dims[ta ? ra - 2 : ra - 1];
  int64_t kb = b.shape.dims[tb ? rb - 1 : rb - 2], n = b.shape.dims[tb ? rb - 2 : rb - 1];
  TFA_CHECK(ka < 0 || kb < 0 || ka == kb, "MatMul inner dimensions differ: ", a.shape.str(),
            (ta ? "^T" : ""), " x ", b.shape.str(), (tb ? "^T" : ""));
  std::vector<int64_t> d;
  if (batch) {
    Shape ba(std::vector<int64_t>(a.shape.dims.begin(), a.shape.dims.end() - 2));
    Shape bb(std::vector<int64_t>(b.shape.dims.begin(), b.shape.dims.end() - 2));
    d = broadcast_shapes(ba, bb).dims;
  }
  d.push_back(m);
  d.push_back(n);
  c.set(0, a.dtype, Shape(d));
}

}  // namespace

// shared with the planner's fused GEMM epilogue
void run_gemm(ExecCtx& c, const at::Tensor& a0, const at::Tensor& b0, bool ta, bool tb,
              const at::Tensor* bias, int act, at::Tensor& out, const std::vector<EpiStep>* epi) {
  if (!c.gpu) {
    at::Tensor a = ta ? a0.transpose(-1, -2) : a0;
    at::Tensor b = tb ? b0.transpose(-1, -2) : b0;
    at::Tensor r = at::matmul(a, b);
    if (bias) r = r + *bias;
    r = apply_act_host(r, act);
    if (epi) r = apply_epi_host(r.reshape({-1, r.size(-1)}), epi).reshape(r.sizes());
    out = r.contiguous();
    return;
  }
  require_gpu_dtype(a0, {at::kFloat, at::kDouble, at::kInt, at::kLong}, "MatMul");
  at::Tensor a = materialize(c, a0), b = materialize(c, b0);
  const auto& od = out.sizes();
  int64_t M = od[od.size() - 2], N = od[od.size() - 1];
  int64_t K = ta ? a.size(-2) : a.size(-1);
  int64_t batch = 1;
  for (size_t i = 0; i + 2 < od.size(); ++i) batch *= od[i];
  // batch broadcast: operands with batch 1 get stride 0
  auto bstride = [&](const at::Tensor& t) -> int64_t {
    int64_t tb2 = 1;
    for (int64_t i = 0; i + 2 < t.dim(); ++i) tb2 *= t.size(i);
    TFA_CHECK(tb2 == batch || tb2 == 1, "BatchMatMul: unsupported batch broadcast");
    return tb2 == 1 ? 0 : t.size(-1) * t.size(-2);
  };
  k::GemmArgs g;
  g.M = M; g.N = N; g.K = K;
  g.A = a.data_ptr(); g.lda = a.size(-1); g.strideA = bstride(a);
  g.B = b.data_ptr(); g.ldb = b.size(-1); g.strideB = bstride(b);
  // `out` may be a column slice of a wider [M, *] tensor (concat write-into-slice)
  const int64_t ldc = (out.dim() >= 2 && batch == 1) ? out.stride(-2) : N;
  TFA_CHECK(out.stride(-1) == 1 && (batch == 1 || out.is_contiguous()), "MatMul: unsupported output layout");
  g.C = out.data_ptr(); g.ldc = ldc; g.strideC = M * N;
  g.ta = ta; g.tb = tb;
  g.bias = bias ? bias->data_ptr() : nullptr;
  g.act = act;
  g.epi = epi_prog(epi);
  g.batch = batch;
  if (M == 0 || N == 0) return;
  if (K == 0) {
    k::fill(dt_of(out), out.data_ptr(), out.numel(), 0.0, stream_of(c));
    return;
  }
  at::Tensor work;
  if (size_t ws = k::gemm_workspace_bytes(dt_of(a), g)) {
    work = c.alloc({static_cast<int64_t>(ws)}, a.options().dtype(at::kByte));
    g.workspace = work.data_ptr();
  }
  k::gemm(dt_of(a), g, stream_of(c));
}

void register_math_ops(OpRegistry& r) {
  using B = k::BinOp;
  r.add("Add", make_binary(B::ADD));
  r.add("AddV2", make_binary(B::ADD));
  r.add("Sub", make_binary(B::SUB));
  r.add("Mul", make_binary(B::MUL));
  r.add("Div", make_binary(B::DIV));
  r.add("RealDiv", make_binary(B::DIV));
  r.add("TruncateDiv", make_binary(B::DIV));
  r.add("FloorDiv", make_binary(B::FLOORDIV));
  r.add("FloorMod", make_binary(B::FLOORMOD));
  r.add("Mod", make_binary(B::TRUNCMOD));
  r.add("TruncateMod", make_binary(B::TRUNCMOD));
  r.add("Maximum", make_binary(B::MAX));
  r.add("Minimum", make_binary(B::MIN));
  r.add("Pow", make_binary(B::POW));
  r.add("SquaredDifference", make_binary(B::SQDIFF));
  r.add("Equal", make_binary(B::EQ));
  r.add("NotEqual", make_binary(B::NE));
  r.add("Less", make_binary(B::LT));
  r.add("LessEqual", make_binary(B::LE));
  r.add("Greater", make_binary(B::GT));
  r.add("GreaterEqual", make_binary(B::GE));
  r.add("LogicalAnd", make_binary(B::LAND));
  r.add("LogicalOr", make_binary(B::LOR));
  r.add("Atan2", make_binary(B::ATAN2));
  r.add("DivNoNan", make_binary(B::DIVNONAN));

  using U = k::UnOp;
  r.add("Neg", make_unary(U::NEG));
  r.add("Abs", make_unary(U::ABS));
  r.add("Square", make_unary(U::SQUARE));
  r.add("Sqrt", make_unary(U::SQRT));
  r.add("Rsqrt", make_unary(U::RSQRT));
  r.add("Exp", make_unary(U::EXP));
  r.add("Log", make_unary(U::LOG));
  r.add("Log1p", make_unary(U::LOG1P));
  r.add("Expm1", make_unary(U::EXPM1));
  r.add("Reciprocal", make_unary(U::RECIP));
  r.add("Inv", make_unary(U::RECIP));
  r.add("Relu", make_unary(U::RELU));
  r.add("Relu6", make_unary(U::RELU6));
  r.add("Elu", make_unary(U::ELU));
  r.add("Selu", make_unary(U::SELU));
  r.add("Sigmoid", make_unary(U::SIGMOID));
  r.add("Tanh", make_unary(U::TANH));
  r.add("Softplus", make_unary(U::SOFTPLUS));
  r.add("Softsign", make_unary(U::SOFTSIGN));
  r.add("Floor", make_unary(U::FLOOR));
  r.add("Ceil", make_unary(U::CEIL));
  r.add("Round", make_unary(U::ROUND));
  r.add("Rint", make_unary(U::ROUND));
  r.add("Sign", make_unary(U::SIGN));
  r.add("Sin", make_unary(U::SIN));
  r.add("Cos", make_unary(U::COS));
  r.add("Tan", make_unary(U::TAN));
  r.add("LogicalNot", make_unary(U::NOT));
  r.add("Erf", make_unary(U::ERF));
  r.add("IsNan", make_unary(U::ISNAN));
  r.add("IsInf", make_unary(U::ISINF));
  r.add("IsFinite", make_unary(U::ISFINITE));

  // AddN: sum of N same-shape tensors
  OpDef addn;
  addn.infer = [](InferCtx& c) {
    Shape s = c.input(0).shape;
    for (size_t i = 1; i < c.in.size(); ++i) s = broadcast_shapes(s, c.input(static_cast<int>(i)).shape);
    c.set(0, c.input(0).dtype, s);
  };
  addn.rows = [](InferCtx& c) { c.rows_elementwise(); };
  addn.compute = [](ExecCtx& c) {
    if (!c.gpu) {
      at::Tensor s = c.input(0);
      for (size_t i = 1; i < c.in.size(); ++i) s = s + c.in[i];
      c.out[0] = s.contiguous();
      return;
    }
    at::Tensor acc = materialize(c, c.input(0));
    for (size_t i = 1; i < c.in.size(); ++i) {
      gpu_binary(c, k::BinOp::ADD, acc, c.in[i]);
      acc = c.out[0];
    }
    c.out[0] = acc;
  };
  r.add("AddN", addn);

  using R = k::RedOp;
  r.add("Sum", make_reduce(R::SUM));
  r.add("Prod", make_reduce(R::PROD));
  r.add("Min", make_reduce(R::MIN));
  r.add("Max", make_reduce(R::MAX));
  r.add("Mean", make_reduce(R::MEAN));
  r.add("All", make_reduce(R::ALL));
  r.add("Any", make_reduce(R::ANY));
  r.add("ArgMin", make_argreduce(true));
  r.add("ArgMax", make_argreduce(false));

  OpDef mm;
  mm.infer = [](InferCtx& c) { infer_matmul(c, false); };
  mm.rows = [](InferCtx& c) {
    if (c.all_const()) { c.out[0].row = RowClass::CONST; return; }
    bool ok = c.input(0).row == RowClass::ROW && !c.node.attr_b("transpose_a", false) &&
              c.input(1).row == RowClass::CONST;
    c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  mm.compute = [](ExecCtx& c) {
    at::Tensor out = c.gpu ? c.alloc_out(0) : at::Tensor();
    run_gemm(c, c.input(0), c.input(1), c.node.attr_b("transpose_a", false),
             c.node.attr_b("transpose_b", false), nullptr, 0, out);
    c.out[0] = out;
  };
  r.add("MatMul", mm);

  OpDef bmm;
  bmm.infer = [](InferCtx& c) { infer_matmul(c, true); };
  bmm.rows = [](InferCtx& c) {
    if (c.all_const()) { c.out[0].row = RowClass::CONST; return; }
    bool ok = c.input(0).row == RowClass::ROW && c.input(0).shape.rank() >= 3 &&
              c.input(1).row == RowClass::CONST && c.input(1).shape.rank() == 2;
    c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  bmm.compute = [](ExecCtx& c) {
    at::Tensor out = c.gpu ? c.alloc_out(0) : at::Tensor();
    run_gemm(c, c.input(0), c.input(1), c.node.attr_b("adj_x", false), c.node.attr_b("adj_y", false),
             nullptr, 0, out);
    c.out[0] = out.reshape(c.out_shape().dims);
  };
  r.add("BatchMatMul", bmm);
  r.add("BatchMatMulV2", bmm);
  r.add("BatchMatMulV3", bmm);

  // Unsorted segment reductions: data [ids.shape..., tail], ids, num_segments
  auto make_useg = [](R op) {
    OpDef d;
    d.host_inputs = {2};
    d.infer = [](InferCtx& c) {
      const TensorInfo& x = c.input(0);
      const TensorInfo& ids = c.input(1);
      auto nv = c.ivalue(2);
      if (x.shape.unknown_rank || ids.shape.unknown_rank) { c.set(0, x.dtype, Shape::unknown()); return; }
      std::vector<int64_t> d{nv ? (*nv)[0] : -1};
      for (int i = ids.shape.rank(); i < x.shape.rank(); ++i) d.push_back(x.shape.dims[i]);
      c.set(0, x.dtype, Shape(d));
    };
    d.compute = [op](ExecCtx& c) {
      at::Tensor x = c.input(0), ids = c.input(1);
      int64_t nseg = c.host_ivalue(2)[0];
      int64_t nrows = ids.numel();
      int64_t inner = nrows ? x.numel() / nrows : 0;
      if (!c.gpu) {
        at::Tensor xf = x.reshape({nrows, inner});
        at::Tensor idl = ids.reshape({-1}).to(at::kLong);
        at::Tensor valid = (idl >= 0) & (idl < nseg);
        at::Tensor xs = xf.index({valid});
        at::Tensor is = idl.index({valid});
        at::Tensor out;
        if (op == R::SUM) {
          out = at::zeros({nseg, inner}, x.options()).index_add_(0, is, xs);
        } else if (op == R::PROD) {
          out = at::ones({nseg, inner}, x.options());
          out = out.index_reduce_(0, is, xs, "prod", true);
        } else {
          bool mx = op == R::MAX;
          at::Scalar init;
          switch (x.scalar_type()) {
            case at::kInt:
              init = mx ? std::numeric_limits<int32_t>::lowest() : std::numeric_limits<int32_t>::max();
              break;
            case at::kLong:
              init = mx ? std::numeric_limits<int64_t>::lowest() : std::numeric_limits<int64_t>::max();
              break;
            case at::kFloat:
              init = mx ? std::numeric_limits<float>::lowest() : std::numeric_limits<float>::max();
              break;
            default:
              init = mx ? std::numeric_limits<double>::lowest() : std::numeric_limits<double>::max();
          }
          out = at::full({nseg, inner}, init, x.options());
          out = out.index_reduce_(0, is, xs, mx ? "amax" : "amin", true);
        }
        c.out[0] = out.reshape(c.out_shape().dims).contiguous();
        return;
      }
      require_gpu_dtype(x, {at::kFloat, at::kDouble, at::kInt, at::kLong}, c.node.op.c_str());
      at::Tensor xc = materialize(c, x), ic = materialize(c, ids);
      c.out[0] = c.alloc_out(0);
      if (!c.out[0].numel()) return;
      size_t ws = k::unsorted_segment_workspace_bytes(op, dt_of(xc), nrows, inner, nseg);
      at::Tensor work;
      if (ws) work = c.alloc({static_cast<int64_t>(ws)}, xc.options().dtype(at::kByte));
      k::unsorted_segment_reduce(op, dt_of(xc), dt_of(ic), xc.data_ptr(), ic.data_ptr(),
                                 c.out[0].data_ptr(), nrows, inner, nseg,
                                 ws ? work.data_ptr() : nullptr, stream_of(c));
    };
    return d;
  };
  r.add("UnsortedSegmentSum", make_useg(R::SUM));
  r.add("UnsortedSegmentProd", make_useg(R::PROD));
  r.add("UnsortedSegmentMax", make_useg(R::MAX));
  r.add("UnsortedSegmentMin", make_useg(R::MIN));
}

}  // namespace tfa

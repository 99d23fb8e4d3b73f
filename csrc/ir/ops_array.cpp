// Array / shape / data-movement ops.
//
// Semantics follow TF-1.x GraphDef ops as emitted by the reference's DSL
// (reference: src/main/scala/org/tensorframes/dsl/DslImpl.scala:77-107,
// package.scala:66-113) and by the example graphs
// (reference: src/main/python/tensorframes_snippets/kmeans_demo.py:26-41,133-144).
#include <numeric>

#include "ops_common.h"

namespace tfa {

// ------------------------------------------------------------------ helpers
void gpu_copy(const at::Tensor& src, const at::Tensor& dst, hipStream_t s) {
  TFA_CHECK(src.sizes() == dst.sizes(), "internal: gpu_copy size mismatch");
  TFA_CHECK(src.element_size() == dst.element_size(), "internal: gpu_copy dtype mismatch");
  if (src.numel() == 0) return;
  if (src.is_contiguous() && dst.is_contiguous()) {
    hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), src.numel() * src.element_size(),
                   hipMemcpyDeviceToDevice, s);
    return;
  }
  // merge dims that are contiguous in both operands
  std::vector<int64_t> dims, ss, ds;
  for (int64_t i = 0; i < src.dim(); ++i) {
    if (src.size(i) == 1) continue;
    if (!dims.empty() && ss.back() == src.stride(i) * src.size(i) &&
        ds.back() == dst.stride(i) * src.size(i)) {
      dims.back() *= src.size(i);
      ss.back() = src.stride(i);
      ds.back() = dst.stride(i);
    } else {
      dims.push_back(src.size(i));
      ss.push_back(src.stride(i));
      ds.push_back(dst.stride(i));
    }
  }
  if (dims.empty()) {
    dims = {1};
    ss = {1};
    ds = {1};
  }
  TFA_CHECK(static_cast<int>(dims.size()) <= k::kMaxRank, "copy of rank > ", k::kMaxRank);
  k::strided_copy(src.element_size(), static_cast<int>(dims.size()), dims.data(), src.data_ptr(),
                  ss.data(), dst.data_ptr(), ds.data(), s);
}

at::Tensor materialize(const ExecCtx& c, const at::Tensor& view) {
  if (!c.gpu) return view.contiguous();
  if (view.is_contiguous()) return view;
  at::Tensor out = pool_empty(view.sizes(), view.options());
  gpu_copy(view, out, stream_of(c));
  return out;
}

k::Bcast make_bcast(const std::vector<int64_t>& out, const at::Tensor& a, const at::Tensor& b,
                    const at::Tensor* c) {
  k::Bcast bc;
  TFA_CHECK(static_cast<int>(out.size()) <= k::kMaxRank, "broadcast of rank > ", k::kMaxRank);
  bc.rank = static_cast<int>(out.size());
  at::Tensor ea = a.expand(out), eb = b.expand(out);
  at::Tensor ec = c ? c->expand(out) : ea;
  for (int i = 0; i < bc.rank; ++i) {
    bc.dims[i] = out[i];
    bc.sa[i] = ea.stride(i);
    bc.sb[i] = eb.stride(i);
    bc.sc[i] = ec.stride(i);
  }
  return bc;
}

static at::Tensor scalar_host(const ExecCtx& c, int i) {
  const TensorInfo* t = c.in_info->at(i);
  if (t->value) return *t->value;
  return c.input(i).to(at::kCPU);
}

static void rows_identity(InferCtx& c) {
  for (size_t i = 0; i < c.out.size(); ++i) c.out[i].row = c.input(std::min(i, c.in.size() - 1)).row;
}

// StridedSlice (TF semantics) resolved against a known input shape.
struct SliceSpec {
  std::vector<int64_t> out_dims;     // final output dims
  int64_t offset = 0;                // element offset into input
  std::vector<int64_t> view_dims;    // dims of the strided view (before reshape)
  std::vector<int64_t> view_strides; // element strides into input
  std::vector<int> kept_input_dim;   // for each output dim: input dim it came from (-1 new axis)
};

static SliceSpec resolve_strided_slice(const Node& n, const std::vector<int64_t>& in_dims,
                                       std::vector<int64_t> begin, std::vector<int64_t> end,
                                       std::vector<int64_t> strides) {
  int64_t bm = n.attr_i("begin_mask", 0), em = n.attr_i("end_mask", 0);
  int64_t elm = n.attr_i("ellipsis_mask", 0), nam = n.attr_i("new_axis_mask", 0);
  int64_t sam = n.attr_i("shrink_axis_mask", 0);
  int nspec = static_cast<int>(begin.size());
  TFA_CHECK(end.size() == begin.size() && strides.size() == begin.size(),
            "StridedSlice begin/end/strides length mismatch");
  int rank = static_cast<int>(in_dims.size());
  std::vector<int64_t> in_strides(rank, 1);
  for (int i = rank - 2; i >= 0; --i) in_strides[i] = in_strides[i + 1] * in_dims[i + 1];
  // count dims consumed by specs (excluding ellipsis and new axes)
  int consumed = 0;
  for (int i = 0; i < nspec; ++i)
    if (!((elm >> i) & 1) && !((nam >> i) & 1)) ++consumed;
  SliceSpec sp;
  int d = 0;  // input dim cursor
  for (int i = 0; i < nspec; ++i) {
    if ((elm >> i) & 1) {
      int span = rank - consumed - d;
      // ellipsis covers dims not otherwise named; ellipsis expands to rank - (consumed)
      span = rank - consumed;
      int covered = 0;
      for (int j = 0; j < i; ++j)
        if (!((elm >> j) & 1) && !((nam >> j) & 1)) ++covered;
      (void)covered;
      int upto = d + (rank - consumed);
      for (; d < upto; ++d) {
        sp.view_dims.push_back(in_dims[d]);
        sp.view_strides.push_back(in_strides[d]);
        sp.out_dims.push_back(in_dims[d]);
        sp.kept_input_dim.push_back(d);
      }
      (void)span;
      continue;
    }
    if ((nam >> i) & 1) {
      sp.out_dims.push_back(1);
      sp.kept_input_dim.push_back(-1);
      continue;
    }
    TFA_CHECK(d < rank, "StridedSlice: too many slice dims for rank ", rank);
    int64_t dim = in_dims[d], st = strides[i];
    TFA_CHECK(st != 0, "StridedSlice: stride 0");
    if ((sam >> i) & 1) {
      int64_t b = begin[i] < 0 ? begin[i] + dim : begin[i];
      TFA_CHECK(b >= 0 && b < dim, "StridedSlice: index ", begin[i], " out of bounds for dim ", dim);
      sp.offset += b * in_strides[d];
      ++d;
      continue;
    }
    auto clampi = [&](int64_t v, bool is_begin) -> int64_t {
      if (v < 0) v += dim;
      if (st > 0) return std::min(std::max<int64_t>(v, 0), dim);
      return std::min(std::max<int64_t>(v, -1), dim - 1);
      (void)is_begin;
    };
    int64_t b = ((bm >> i) & 1) ? (st > 0 ? 0 : dim - 1) : clampi(begin[i], true);
    int64_t e = ((em >> i) & 1) ? (st > 0 ? dim : -1) : clampi(end[i], false);
    int64_t len = st > 0 ? std::max<int64_t>(0, (e - b + st - 1) / st)
                         : std::max<int64_t>(0, (b - e + (-st) - 1) / (-st));
    sp.offset += (len > 0 ? b : 0) * in_strides[d];
    sp.view_dims.push_back(len);
    sp.view_strides.push_back(st * in_strides[d]);
    sp.out_dims.push_back(len);
    sp.kept_input_dim.push_back(d);
    ++d;
  }
  for (; d < rank; ++d) {
    sp.view_dims.push_back(in_dims[d]);
    sp.view_strides.push_back(in_strides[d]);
    sp.out_dims.push_back(in_dims[d]);
    sp.kept_input_dim.push_back(d);
  }
  return sp;
}

static at::Tensor strided_view_copy(const ExecCtx& c, const at::Tensor& x, const SliceSpec& sp) {
  at::Tensor xc = x.contiguous();
  std::vector<int64_t> vd = sp.view_dims, vs = sp.view_strides;
  if (vd.empty()) {
    vd = {1};
    vs = {1};
  }
  int64_t total = 1;
  for (auto v : vd) total *= v;
  at::Tensor out = pool_empty(vd, xc.options());
  if (total > 0) {
    if (!c.gpu) {
      // negative strides are not expressible as an ATen view: gather via index math
      at::Tensor flat = xc.reshape({-1});
      at::Tensor idx = at::full({1}, sp.offset, at::kLong);
      for (size_t i = 0; i < vd.size(); ++i) {
        at::Tensor r = at::arange(vd[i], at::kLong) * vs[i];
        idx = (idx.unsqueeze(-1) + r).reshape({-1});
      }
      out = flat.index_select(0, idx).reshape(vd);
    } else {
      const char* base = static_cast<const char*>(xc.data_ptr()) + sp.offset * xc.element_size();
      std::vector<int64_t> dstr(vd.size(), 1);
      for (int i = static_cast<int>(vd.size()) - 2; i >= 0; --i) dstr[i] = dstr[i + 1] * vd[i + 1];
      TFA_CHECK(static_cast<int>(vd.size()) <= k::kMaxRank, "slice of rank > ", k::kMaxRank);
      k::strided_copy(xc.element_size(), static_cast<int>(vd.size()), vd.data(), base, vs.data(),
                      out.data_ptr(), dstr.data(), stream_of(c));
    }
  }
  return out.reshape(sp.out_dims);
}

// ------------------------------------------------------------------ registration
void register_array_ops(OpRegistry& r) {
  // ---- Placeholder
  OpDef ph;
  ph.infer = [](InferCtx& c) {
    DType dt = c.node.attr_type("dtype");
    Shape s = Shape::unknown();
    if (const AttrValue* a = c.node.def->find_attr("shape")) {
      if (a->kind == AttrValue::SHAPE) s = a->shape;
    }
    c.set(0, dt, s);
    c.out[0].row = RowClass::ROW;
  };
  ph.rows = [](InferCtx& c) { c.out[0].row = RowClass::ROW; };
  ph.compute = [](ExecCtx& c) {
    TFA_CHECK(false, "placeholder '", c.node.name, "' was not fed");
  };
  r.add("Placeholder", ph);
  r.add("PlaceholderV2", ph);

  OpDef phd;  // PlaceholderWithDefault: input is the default
  phd.infer = [](InferCtx& c) { infer_like(c); c.out[0].value = c.input(0).value; };
  phd.rows = rows_identity;
  phd.compute = [](ExecCtx& c) { c.out[0] = c.input(0); };
  r.add("PlaceholderWithDefault", phd);

  // ---- Const
  OpDef cst;
  cst.infer = [](InferCtx& c) {
    const HostTensor& t = c.node.attr_tensor("value");
    DType dt = c.node.attr_type("dtype", t.dtype);
    c.set(0, dt, t.shape);
    if (t.dtype == DType::STRING) {
      c.out[0].strings = std::make_shared<std::vector<std::string>>(t.strings);
    } else {
      // borrowed view of the GraphDef's bytes: no copy per plan (weights can be
      // GBs); anything handed to a caller is copied by Program::device_const
      at::Tensor v = host_tensor_view(t);
      if (dt != t.dtype) v = v.to(to_scalar_type(dt));
      c.out[0].value = v;
    }
    c.out[0].row = RowClass::CONST;
  };
  cst.rows = [](InferCtx& c) { c.out[0].row = RowClass::CONST; };
  cst.compute = [](ExecCtx&) {};
  r.add("Const", cst);

  // ---- Identity-like
  OpDef ident;
  ident.infer = [](InferCtx& c) {
    infer_like(c);
    c.out[0].value = c.input(0).value;
    c.out[0].strings = c.input(0).strings;
  };
  ident.rows = rows_identity;
  ident.compute = [](ExecCtx& c) { c.out[0] = c.input(0); };
  for (auto nm : {"Identity", "StopGradient", "Snapshot", "PreventGradient", "CheckNumerics",
                  "EnsureShape"})
    r.add(nm, ident);

  OpDef identn;
  identn.num_outputs = [](const Node& n) { return static_cast<int>(n.inputs.size()); };
  identn.infer = [](InferCtx& c) {
    for (size_t i = 0; i < c.in.size(); ++i) {
      c.set(static_cast<int>(i), c.input(static_cast<int>(i)).dtype, c.input(static_cast<int>(i)).shape);
      c.out[i].value = c.input(static_cast<int>(i)).value;
    }
  };
  identn.rows = [](InferCtx& c) {
    for (size_t i = 0; i < c.in.size(); ++i) c.out[i].row = c.in[i]->row;
  };
  identn.compute = [](ExecCtx& c) { c.out = c.in; };
  r.add("IdentityN", identn);

  OpDef noop;
  noop.num_outputs = [](const Node&) { return 0; };
  noop.infer = [](InferCtx&) {};
  noop.compute = [](ExecCtx&) {};
  r.add("NoOp", noop);

  // ---- Shape / Size / Rank: values come from (concrete) shapes
  OpDef shape;
  shape.infer = [](InferCtx& c) {
    DType ot = c.node.attr_type("out_type", DType::I32);
    const Shape& s = c.input(0).shape;
    c.set(0, ot, s.unknown_rank ? Shape({-1}) : Shape({static_cast<int64_t>(s.dims.size())}));
    if (s.fully_known()) {
      at::Tensor v = at::tensor(s.dims, at::kLong).to(to_scalar_type(ot));
      c.out[0].value = v;
    }
  };
  shape.rows = [](InferCtx& c) {
    c.out[0].row = c.input(0).row == RowClass::CONST ? RowClass::CONST : RowClass::MIXED;
  };
  shape.compute = [](ExecCtx& c) {
    c.out[0] = at::tensor(c.input(0).sizes().vec(), at::kLong).to(to_scalar_type(c.out_dtype()));
    if (c.gpu) c.out[0] = c.out[0].to(c.input(0).device());
  };
  r.add("Shape", shape);

  OpDef size;
  size.infer = [](InferCtx& c) {
    DType ot = c.node.attr_type("out_type", DType::I32);
    c.set(0, ot, Shape(std::vector<int64_t>{}));
    int64_t n = c.input(0).shape.num_elements();
    if (n >= 0) c.out[0].value = at::scalar_tensor(n, at::kLong).to(to_scalar_type(ot));
  };
  size.rows = shape.rows;
  size.compute = [](ExecCtx& c) {
    c.out[0] = at::scalar_tensor(c.input(0).numel(), at::kLong).to(to_scalar_type(c.out_dtype()));
    if (c.gpu) c.out[0] = c.out[0].to(c.input(0).device());
  };
  r.add("Size", size);

  OpDef rank;
  rank.infer = [](InferCtx& c) {
    c.set(0, DType::I32, Shape(std::vector<int64_t>{}));
    int rk = c.input(0).shape.rank();
    if (rk >= 0) c.out[0].value = at::scalar_tensor(rk, at::kInt);
  };
  rank.rows = [](InferCtx& c) { c.out[0].row = RowClass::CONST; };
  rank.compute = [](ExecCtx& c) {
    c.out[0] = at::scalar_tensor(c.input(0).dim(), at::kInt);
    if (c.gpu) c.out[0] = c.out[0].to(c.input(0).device());
  };
  r.add("Rank", rank);

  // ---- Reshape
  OpDef reshape;
  reshape.host_inputs = {1};
  reshape.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto sv = c.ivalue(1);
    if (!sv) {
      const Shape& ss = c.input(1).shape;
      if (ss.rank() == 1 && ss.dims[0] >= 0) c.set(0, x.dtype, Shape(std::vector<int64_t>(ss.dims[0], -1)));
      else c.set(0, x.dtype, Shape::unknown());
      return;
    }
    std::vector<int64_t> dims = *sv;
    int neg = -1;
    int64_t known = 1;
    for (size_t i = 0; i < dims.size(); ++i) {
      if (dims[i] == -1) {
        TFA_CHECK(neg < 0, "Reshape: only one dimension can be -1");
        neg = static_cast<int>(i);
      } else {
        known *= dims[i];
      }
    }
    int64_t total = x.shape.num_elements();
    if (neg >= 0 && total >= 0) {
      TFA_CHECK(known > 0 ? total % known == 0 : total == 0, "Reshape: cannot reshape ",
                x.shape.str(), " into ", Shape(*sv).str());
      dims[neg] = known > 0 ? total / known : 0;
    } else if (total >= 0) {
      TFA_CHECK(known == total, "Reshape: cannot reshape tensor with ", total,
                " elements into shape ", Shape(dims).str());
    }
    c.set(0, x.dtype, Shape(dims));
  };
  reshape.rows = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    if (x.row == RowClass::CONST) { c.out[0].row = RowClass::CONST; return; }
    c.out[0].row = RowClass::MIXED;
    if (x.row != RowClass::ROW || c.input(1).row != RowClass::CONST) return;
    auto sv = c.ivalue(1);
    if (!sv || sv->empty() || x.shape.rank() < 1) return;
    // row-preserving iff target is [-1, ...] and tail sizes match the input's per-row size
    if ((*sv)[0] != -1) return;
    int64_t tail_out = 1, tail_in = 1;
    for (size_t i = 1; i < sv->size(); ++i) {
      if ((*sv)[i] < 0) return;
      tail_out *= (*sv)[i];
    }
    for (int i = 1; i < x.shape.rank(); ++i) {
      if (x.shape.dims[i] < 0) return;
      tail_in *= x.shape.dims[i];
    }
    if (tail_in == tail_out) c.out[0].row = RowClass::ROW;
  };
  reshape.compute = [](ExecCtx& c) {
    c.out[0] = materialize(c, c.input(0)).reshape(c.out_shape().dims);
  };
  r.add("Reshape", reshape);

  // ---- Squeeze
  OpDef squeeze;
  squeeze.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    std::vector<int64_t> axes = c.node.attr_ilist("squeeze_dims");
    if (axes.empty()) axes = c.node.attr_ilist("axis");
    if (x.shape.unknown_rank) { c.set(0, x.dtype, Shape::unknown()); return; }
    int rk = x.shape.rank();
    std::vector<bool> drop(rk, false);
    if (axes.empty()) {
      for (int i = 0; i < rk; ++i) {
        // an unknown dim may or may not be 1: the rank is unknown until run time (as in TF)
        if (x.shape.dims[i] < 0) { c.set(0, x.dtype, Shape::unknown()); return; }
        drop[i] = x.shape.dims[i] == 1;
      }
    } else {
      for (auto a : axes) {
        int64_t ax = norm_axis(a, rk);
        TFA_CHECK(x.shape.dims[ax] == 1 || x.shape.dims[ax] < 0, "Squeeze: dim ", ax,
                  " of ", x.shape.str(), " is not 1");
        drop[ax] = true;
      }
    }
    std::vector<int64_t> d;
    for (int i = 0; i < rk; ++i)
      if (!drop[i]) d.push_back(x.shape.dims[i]);
    c.set(0, x.dtype, Shape(d));
  };
  squeeze.rows = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    c.out[0].row = x.row;
    if (x.row == RowClass::ROW) {
      std::vector<int64_t> axes = c.node.attr_ilist("squeeze_dims");
      if (axes.empty()) axes = c.node.attr_ilist("axis");
      if (axes.empty()) { c.out[0].row = RowClass::MIXED; return; }
      for (auto a : axes)
        if (norm_axis(a, x.shape.rank()) == 0) c.out[0].row = RowClass::MIXED;
    }
  };
  squeeze.compute = [](ExecCtx& c) { c.out[0] = materialize(c, c.input(0)).reshape(c.out_shape().dims); };
  r.add("Squeeze", squeeze);

  // ---- ExpandDims
  OpDef expand;
  expand.host_inputs = {1};
  expand.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto av = c.ivalue(1);
    if (x.shape.unknown_rank || !av) {
      c.set(0, x.dtype, Shape::unknown());
      return;
    }
    int rk = x.shape.rank();
    int64_t a = (*av)[0];
    if (a < 0) a += rk + 1;
    TFA_CHECK(a >= 0 && a <= rk, "ExpandDims: axis out of range");
    std::vector<int64_t> d = x.shape.dims;
    d.insert(d.begin() + a, 1);
    c.set(0, x.dtype, Shape(d));
  };
  expand.rows = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    c.out[0].row = x.row;
    if (x.row == RowClass::ROW) {
      auto av = c.ivalue(1);
      int64_t a = av ? (*av)[0] : 0;
      if (a < 0) a += x.shape.rank() + 1;
      if (a == 0) c.out[0].row = RowClass::MIXED;
    }
  };
  expand.compute = [](ExecCtx& c) { c.out[0] = materialize(c, c.input(0)).reshape(c.out_shape().dims); };
  r.add("ExpandDims", expand);

  // ---- Fill / ZerosLike / OnesLike
  OpDef fill;
  fill.host_inputs = {0};
  fill.infer = [](InferCtx& c) {
    auto dv = c.ivalue(0);
    DType dt = c.input(1).dtype;
    if (dv) c.set(0, dt, Shape(*dv));
    else if (c.input(0).shape.rank() == 1 && c.input(0).shape.dims[0] >= 0)
      c.set(0, dt, Shape(std::vector<int64_t>(c.input(0).shape.dims[0], -1)));
    else c.set(0, dt, Shape::unknown());
  };
  fill.compute = [](ExecCtx& c) {
    at::Tensor v = scalar_host(c, 1);
    if (!c.gpu) {
      c.out[0] = at::full(c.out_shape().dims, v.item(), v.options());
      return;
    }
    c.out[0] = c.alloc_out(0);
    k::fill(c.out_dtype(), c.out[0].data_ptr(), c.out[0].numel(), v.to(at::kDouble).item<double>(),
            stream_of(c));
  };
  r.add("Fill", fill);

  auto like = [](double val) {
    OpDef d;
    d.infer = [](InferCtx& c) { infer_like(c); };
    d.rows = [](InferCtx& c) { c.rows_like(0); };
    d.compute = [val](ExecCtx& c) {
      if (!c.gpu) {
        c.out[0] = at::full(c.input(0).sizes(), val, c.input(0).options());
        return;
      }
      c.out[0] = c.alloc_out(0);
      k::fill(c.out_dtype(), c.out[0].data_ptr(), c.out[0].numel(), val, stream_of(c));
    };
    return d;
  };
  r.add("ZerosLike", like(0.0));
  r.add("OnesLike", like(1.0));

  // ---- Range
  OpDef range;
  range.host_inputs = {0, 1, 2};
  range.infer = [](InferCtx& c) {
    DType dt = c.node.attr_type("Tidx", c.input(0).dtype);
    auto s = c.scalar_value(0), l = c.scalar_value(1), d = c.scalar_value(2);
    if (s && l && d) {
      TFA_CHECK(*d != 0, "Range: delta must not be 0");
      double n = std::ceil((*l - *s) / *d);
      if (dtype_is_int(dt)) n = std::ceil(std::fabs((*l - *s) / *d));
      c.set(0, dt, Shape({std::max<int64_t>(0, static_cast<int64_t>(n))}));
    } else {
      c.set(0, dt, Shape({-1}));
    }
  };
  range.compute = [](ExecCtx& c) {
    double s = scalar_host(c, 0).to(at::kDouble).item<double>();
    double d = scalar_host(c, 2).to(at::kDouble).item<double>();
    int64_t n = c.out_shape().dims[0];
    if (!c.gpu) {
      c.out[0] = (at::arange(n, at::kDouble) * d + s).to(to_scalar_type(c.out_dtype()));
      return;
    }
    c.out[0] = c.alloc_out(0);
    k::range(c.out_dtype(), c.out[0].data_ptr(), n, s, d, stream_of(c));
  };
  r.add("Range", range);

  // ---- Tile
  OpDef tile;
  tile.host_inputs = {1};
  tile.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto mv = c.ivalue(1);
    if (x.shape.unknown_rank) { c.set(0, x.dtype, Shape::unknown()); return; }
    std::vector<int64_t> d = x.shape.dims;
    if (!mv) {
      for (auto& v : d) v = -1;
    } else {
      TFA_CHECK(mv->size() == d.size(), "Tile: multiples length ", mv->size(), " != rank ", d.size());
      for (size_t i = 0; i < d.size(); ++i) d[i] = d[i] < 0 ? -1 : d[i] * (*mv)[i];
    }
    c.set(0, x.dtype, Shape(d));
  };
  tile.rows = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    if (x.row == RowClass::CONST && c.input(1).row == RowClass::CONST) { c.out[0].row = RowClass::CONST; return; }
    auto mv = c.ivalue(1);
    c.out[0].row = (x.row == RowClass::ROW && mv && !mv->empty() && (*mv)[0] == 1) ? RowClass::ROW
                                                                                  : RowClass::MIXED;
  };
  tile.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    std::vector<int64_t> m = c.host_ivalue(1);
    if (!c.gpu) { c.out[0] = x.repeat(m); return; }
    // view x[d0..] as [1,d0,1,d1,...] expanded to [m0,d0,m1,d1,...]
    std::vector<int64_t> vs, es;
    for (int64_t i = 0; i < x.dim(); ++i) {
      vs.push_back(1); vs.push_back(x.size(i));
      es.push_back(m[i]); es.push_back(x.size(i));
    }
    at::Tensor v = x.contiguous().reshape(vs).expand(es);
    at::Tensor out = pool_empty(es, x.options());
    gpu_copy(v, out, stream_of(c));
    c.out[0] = out.reshape(c.out_shape().dims);
  };
  r.add("Tile", tile);

  // ---- Pack / Unpack
  OpDef pack;
  pack.infer = [](InferCtx& c) {
    int64_t n = static_cast<int64_t>(c.in.size());
    const TensorInfo& x = c.input(0);
    if (x.shape.unknown_rank) { c.set(0, x.dtype, Shape::unknown()); return; }
    int rk = x.shape.rank();
    int64_t ax = c.node.attr_i("axis", 0);
    if (ax < 0) ax += rk + 1;
    TFA_CHECK(ax >= 0 && ax <= rk, "Pack: axis out of range");
    Shape s = x.shape;
    for (size_t i = 1; i < c.in.size(); ++i) {
      TFA_CHECK(c.input(static_cast<int>(i)).dtype == x.dtype, "Pack: inputs must share a dtype");
      s = broadcast_shapes(s, c.input(static_cast<int>(i)).shape);
    }
    std::vector<int64_t> d = s.dims;
    d.insert(d.begin() + ax, n);
    c.set(0, x.dtype, Shape(d));
  };
  pack.rows = [](InferCtx& c) {
    if (c.all_const()) { c.out[0].row = RowClass::CONST; return; }
    int64_t ax = c.node.attr_i("axis", 0);
    bool ok = ax >= 1 || (ax < 0 && ax + c.input(0).shape.rank() + 1 >= 1);
    for (auto* t : c.in) ok = ok && t->row == RowClass::ROW;
    c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  pack.compute = [](ExecCtx& c) {
    int rk = static_cast<int>(c.input(0).dim());
    int64_t ax = c.node.attr_i("axis", 0);
    if (ax < 0) ax += rk + 1;
    if (!c.gpu) { c.out[0] = at::stack(c.in, ax); return; }
    at::Tensor out = c.alloc_out(0);
    for (size_t i = 0; i < c.in.size(); ++i) gpu_copy(c.in[i], out.select(ax, static_cast<int64_t>(i)), stream_of(c));
    c.out[0] = out;
  };
  r.add("Pack", pack);

  OpDef unpack;
  unpack.num_outputs = [](const Node& n) { return static_cast<int>(n.attr_i("num")); };
  unpack.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    TFA_CHECK(!x.shape.unknown_rank, "Unpack needs a known rank");
    int64_t ax = norm_axis(c.node.attr_i("axis", 0), x.shape.rank());
    std::vector<int64_t> d = x.shape.dims;
    d.erase(d.begin() + ax);
    for (size_t i = 0; i < c.out.size(); ++i) c.set(static_cast<int>(i), x.dtype, Shape(d));
  };
  unpack.compute = [](ExecCtx& c) {
    int64_t ax = norm_axis(c.node.attr_i("axis", 0), c.input(0).dim());
    for (size_t i = 0; i < c.out.size(); ++i)
      c.out[i] = materialize(c, c.input(0).select(ax, static_cast<int64_t>(i)));
  };
  r.add("Unpack", unpack);

  // ---- ConcatV2 (values..., axis) / Concat (axis, values...)
  auto make_concat = [](bool v2) {
    OpDef d;
    d.host_inputs = {v2 ? -1 : 0};
    d.infer = [v2](InferCtx& c) {
      int nv = static_cast<int>(c.in.size()) - 1;
      int first = v2 ? 0 : 1, axis_i = v2 ? nv : 0;
      const TensorInfo& x = c.input(first);
      auto av = c.ivalue(axis_i);
      if (x.shape.unknown_rank || !av) { c.set(0, x.dtype, Shape::unknown()); return; }
      int rk = x.shape.rank();
      int64_t ax = norm_axis((*av)[0], rk);
      std::vector<int64_t> d = x.shape.dims;
      int64_t tot = 0;
      for (int i = 0; i < nv; ++i) {
        const TensorInfo& t = c.input(first + i);
        TFA_CHECK(t.dtype == x.dtype, "Concat: inputs must share a dtype");
        TFA_CHECK(t.shape.rank() == rk, "Concat: inputs must share a rank");
        int64_t v = t.shape.dims[ax];
        tot = (tot < 0 || v < 0) ? -1 : tot + v;
        for (int j = 0; j < rk; ++j)
          if (j != ax && d[j] < 0) d[j] = t.shape.dims[j];
      }
      d[ax] = tot;
      c.set(0, x.dtype, Shape(d));
    };
    d.rows = [v2](InferCtx& c) {
      int nv = static_cast<int>(c.in.size()) - 1;
      int first = v2 ? 0 : 1, axis_i = v2 ? nv : 0;
      bool allc = true, allrow = true;
      for (int i = 0; i < nv; ++i) {
        allc = allc && c.input(first + i).row == RowClass::CONST;
        allrow = allrow && c.input(first + i).row == RowClass::ROW;
      }
      if (allc) { c.out[0].row = RowClass::CONST; return; }
      auto av = c.ivalue(axis_i);
      int rk = c.input(first).shape.rank();
      bool ax_ok = av && rk > 0 && norm_axis((*av)[0], rk) != 0;
      c.out[0].row = (allrow && ax_ok) ? RowClass::ROW : RowClass::MIXED;
    };
    d.compute = [v2](ExecCtx& c) {
      int nv = static_cast<int>(c.in.size()) - 1;
      int first = v2 ? 0 : 1, axis_i = v2 ? nv : 0;
      int64_t ax = norm_axis(c.host_ivalue(axis_i)[0], c.input(first).dim());
      std::vector<at::Tensor> parts(c.in.begin() + first, c.in.begin() + first + nv);
      if (!c.gpu) { c.out[0] = at::cat(parts, ax); return; }
      at::Tensor out = c.alloc_out(0);
      int64_t off = 0;
      for (auto& p : parts) {
        int64_t len = p.size(ax);
        if (len > 0) gpu_copy(p, out.narrow(ax, off, len), stream_of(c));
        off += len;
      }
      c.out[0] = out;
    };
    return d;
  };
  r.add("ConcatV2", make_concat(true));
  r.add("Concat", make_concat(false));

  // ---- Transpose
  OpDef transpose;
  transpose.host_inputs = {1};
  transpose.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto pv = c.ivalue(1);
    if (x.shape.unknown_rank || !pv) { c.set(0, x.dtype, Shape::unknown()); return; }
    TFA_CHECK(static_cast<int>(pv->size()) == x.shape.rank(), "Transpose: perm size mismatch");
    std::vector<int64_t> d;
    for (auto p : *pv) d.push_back(x.shape.dims[norm_axis(p, x.shape.rank())]);
    c.set(0, x.dtype, Shape(d));
  };
  transpose.rows = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    if (x.row != RowClass::ROW) { c.out[0].row = x.row; return; }
    auto pv = c.ivalue(1);
    c.out[0].row = (pv && !pv->empty() && (*pv)[0] == 0) ? RowClass::ROW : RowClass::MIXED;
  };
  transpose.compute = [](ExecCtx& c) {
    std::vector<int64_t> p = c.host_ivalue(1);
    for (auto& v : p) v = norm_axis(v, c.input(0).dim());
    c.out[0] = materialize(c, c.input(0).permute(p));
  };
  r.add("Transpose", transpose);

  // ---- Slice
  OpDef slice;
  slice.host_inputs = {1, 2};
  slice.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto bv = c.ivalue(1), sv = c.ivalue(2);
    if (sv && (x.shape.unknown_rank || !bv)) {
      // begin computed per row (a central crop's offsets) or an input of
      // unknown rank: the sizes given as numbers are still static
      if (!x.shape.unknown_rank)
        TFA_CHECK(static_cast<int>(sv->size()) == x.shape.rank(), "Slice: size has ", sv->size(),
                  " entries for a rank-", x.shape.rank(), " input");
      std::vector<int64_t> d;
      for (int64_t s : *sv) d.push_back(s >= 0 ? s : -1);
      c.set(0, x.dtype, Shape(d));
      return;
    }
    if (x.shape.unknown_rank || !bv || !sv) {
      c.set(0, x.dtype, x.shape.unknown_rank ? Shape::unknown()
                                             : Shape(std::vector<int64_t>(x.shape.rank(), -1)));
      return;
    }
    std::vector<int64_t> d;
    for (int i = 0; i < x.shape.rank(); ++i) {
      int64_t s = (*sv)[i];
      if (s == -1) s = x.shape.dims[i] < 0 ? -1 : x.shape.dims[i] - (*bv)[i];
      d.push_back(s);
    }
    c.set(0, x.dtype, Shape(d));
  };
  slice.compute = [](ExecCtx& c) {
    auto b = c.host_ivalue(1);
    at::Tensor v = c.input(0);
    const auto& od = c.out_shape().dims;
    for (size_t i = 0; i < od.size(); ++i) v = v.narrow(static_cast<int64_t>(i), b[i], od[i]);
    c.out[0] = materialize(c, v);
  };
  r.add("Slice", slice);

  // ---- StridedSlice
  OpDef ss;
  ss.host_inputs = {1, 2, 3};
  ss.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto bv = c.ivalue(1), ev = c.ivalue(2), sv = c.ivalue(3);
    if (!x.shape.fully_known() || !bv || !ev || !sv) {
      // rank can still be determined when shapes are partially known
      if (!x.shape.unknown_rank && bv && ev && sv) {
        std::vector<int64_t> dims = x.shape.dims;
        for (auto& v : dims) if (v < 0) v = 1 << 30;
        SliceSpec sp = resolve_strided_slice(c.node, dims, *bv, *ev, *sv);
        std::vector<int64_t> od = sp.out_dims;
        for (size_t i = 0; i < od.size(); ++i) {
          int kd = sp.kept_input_dim[i];
          if (kd >= 0 && x.shape.dims[kd] < 0) od[i] = -1;
        }
        c.set(0, x.dtype, Shape(od));
      } else {
        c.set(0, x.dtype, Shape::unknown());
      }
      return;
    }
    SliceSpec sp = resolve_strided_slice(c.node, x.shape.dims, *bv, *ev, *sv);
    c.set(0, x.dtype, Shape(sp.out_dims));
  };
  ss.rows = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    if (x.row != RowClass::ROW) { c.out[0].row = x.row == RowClass::CONST && c.all_const() ? RowClass::CONST : (x.row == RowClass::CONST ? RowClass::MIXED : x.row); return; }
    // row-preserving iff the first spec keeps dim 0 whole with stride 1
    auto bv = c.ivalue(1), sv = c.ivalue(3);
    int64_t bm = c.node.attr_i("begin_mask", 0), em = c.node.attr_i("end_mask", 0);
    int64_t elm = c.node.attr_i("ellipsis_mask", 0), nam = c.node.attr_i("new_axis_mask", 0);
    int64_t sam = c.node.attr_i("shrink_axis_mask", 0);
    bool ok = bv && sv && !bv->empty() && (elm & 1) == 0 && (nam & 1) == 0 && (sam & 1) == 0 &&
              (bm & 1) && (em & 1) && (*sv)[0] == 1;
    if (bv && !bv->empty() && (elm & 1)) ok = true;  // leading ellipsis keeps dim 0
    c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  ss.compute = [](ExecCtx& c) {
    SliceSpec sp = resolve_strided_slice(c.node, c.input(0).sizes().vec(), c.host_ivalue(1),
                                         c.host_ivalue(2), c.host_ivalue(3));
    c.out[0] = strided_view_copy(c, c.input(0), sp);
  };
  r.add("StridedSlice", ss);

  // ---- Gather / GatherV2
  auto make_gather = [](bool v2) {
    OpDef d;
    if (v2) d.host_inputs = {2};
    d.infer = [v2](InferCtx& c) {
      const TensorInfo& p = c.input(0);
      const TensorInfo& ix = c.input(1);
      int64_t ax = 0;
      if (v2) {
        auto av = c.ivalue(2);
        if (!av || p.shape.unknown_rank) { c.set(0, p.dtype, Shape::unknown()); return; }
        ax = norm_axis((*av)[0], p.shape.rank());
      }
      if (p.shape.unknown_rank || ix.shape.unknown_rank) { c.set(0, p.dtype, Shape::unknown()); return; }
      std::vector<int64_t> d(p.shape.dims.begin(), p.shape.dims.begin() + ax);
      d.insert(d.end(), ix.shape.dims.begin(), ix.shape.dims.end());
      d.insert(d.end(), p.shape.dims.begin() + ax + 1, p.shape.dims.end());
      c.set(0, p.dtype, Shape(d));
    };
    d.rows = [v2](InferCtx& c) {
      if (c.all_const()) { c.out[0].row = RowClass::CONST; return; }
      int64_t ax = 0;
      if (v2) { auto av = c.ivalue(2); if (!av) { c.out[0].row = RowClass::MIXED; return; } ax = (*av)[0]; if (ax < 0) ax += c.input(0).shape.rank(); }
      const TensorInfo& p = c.input(0);
      const TensorInfo& ix = c.input(1);
      bool ok = false;
      if (ax == 0) ok = p.row == RowClass::CONST && ix.row == RowClass::ROW && ix.shape.rank() >= 1;
      else ok = p.row == RowClass::ROW && ix.row == RowClass::CONST;
      c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
    };
    d.compute = [v2](ExecCtx& c) {
      at::Tensor p = c.input(0), ix = c.input(1);
      int64_t ax = v2 ? norm_axis(c.host_ivalue(2)[0], p.dim()) : 0;
      if (!c.gpu) {
        at::Tensor flat = ix.reshape({-1}).to(at::kLong);
        c.out[0] = p.index_select(ax, flat).reshape(c.out_shape().dims);
        return;
      }
      at::Tensor pc = materialize(c, p);
      int64_t outer = 1, inner = 1;
      for (int64_t i = 0; i < ax; ++i) outer *= pc.size(i);
      for (int64_t i = ax + 1; i < pc.dim(); ++i) inner *= pc.size(i);
      at::Tensor out = c.alloc_out(0);
      if (out.numel() > 0)
        k::gather(pc.element_size(), dt_of(ix), pc.data_ptr(), materialize(c, ix).data_ptr(),
                  out.data_ptr(), outer, pc.size(ax), ix.numel(), inner, stream_of(c));
      c.out[0] = out;
    };
    return d;
  };
  r.add("Gather", make_gather(false));
  r.add("GatherV2", make_gather(true));

  // ---- OneHot (indices, depth, on_value, off_value)
  OpDef onehot;
  onehot.host_inputs = {1, 2, 3};
  onehot.infer = [](InferCtx& c) {
    const TensorInfo& ix = c.input(0);
    auto dv = c.ivalue(1);
    DType dt = c.input(2).dtype;
    int64_t ax = c.node.attr_i("axis", -1);
    if (ix.shape.unknown_rank) { c.set(0, dt, Shape::unknown()); return; }
    TFA_CHECK(ax == -1 || ax == ix.shape.rank(), "OneHot: only axis=-1 is supported");
    std::vector<int64_t> d = ix.shape.dims;
    d.push_back(dv ? (*dv)[0] : -1);
    c.set(0, dt, Shape(d));
  };
  onehot.rows = [](InferCtx& c) { c.rows_like(0); if (c.input(0).shape.rank() < 1 && c.out[0].row == RowClass::ROW) c.out[0].row = RowClass::MIXED; };
  onehot.compute = [](ExecCtx& c) {
    int64_t depth = c.host_ivalue(1)[0];
    double on = scalar_host(c, 2).to(at::kDouble).item<double>();
    double off = scalar_host(c, 3).to(at::kDouble).item<double>();
    at::Tensor ix = c.input(0);
    if (!c.gpu) {
      at::Tensor l = ix.to(at::kLong);
      at::Tensor valid = (l >= 0) & (l < depth);
      at::Tensor oh = at::one_hot(at::where(valid, l, at::zeros_like(l)), depth) *
                      valid.unsqueeze(-1).to(at::kLong);
      c.out[0] = (oh.to(at::kDouble) * (on - off) + off).to(to_scalar_type(c.out_dtype()));
      return;
    }
    c.out[0] = c.alloc_out(0);
    k::one_hot(c.out_dtype(), dt_of(ix), materialize(c, ix).data_ptr(), c.out[0].data_ptr(),
               ix.numel(), depth, on, off, stream_of(c));
  };
  r.add("OneHot", onehot);

  // ---- Cast
  OpDef cast;
  cast.infer = [](InferCtx& c) { c.set(0, c.node.attr_type("DstT"), c.input(0).shape); };
  cast.rows = [](InferCtx& c) { c.rows_like(0); };
  cast.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    DType to = c.out_dtype();
    if (!c.gpu) { c.out[0] = x.to(to_scalar_type(to)); return; }
    if (dt_of(x) == to) { c.out[0] = x; return; }
    at::Tensor xc = materialize(c, x);
    c.out[0] = c.alloc_out(0);
    k::cast(dt_of(xc), to, xc.data_ptr(), c.out[0].data_ptr(), xc.numel(), stream_of(c));
  };
  r.add("Cast", cast);

  // ---- Select (v1: cond may be a vector over dim 0) / SelectV2 (broadcasting)
  auto make_select = [](bool v2) {
    OpDef d;
    d.infer = [v2](InferCtx& c) {
      const TensorInfo& t = c.input(1);
      const TensorInfo& e = c.input(2);
      TFA_CHECK(t.dtype == e.dtype, "Select: branches must share a dtype");
      Shape s = broadcast_shapes(t.shape, e.shape);
      if (v2) s = broadcast_shapes(s, c.input(0).shape);
      c.set(0, t.dtype, s);
    };
    d.rows = [](InferCtx& c) { c.rows_elementwise(); };
    d.compute = [v2](ExecCtx& c) {
      at::Tensor cond = c.input(0), t = c.input(1), e = c.input(2);
      const auto& od = c.out_shape().dims;
      if (!v2 && cond.dim() == 1 && static_cast<int64_t>(od.size()) > 1) {
        std::vector<int64_t> cs(od.size(), 1);
        cs[0] = cond.size(0);
        cond = cond.reshape(cs);
      }
      if (!c.gpu) { c.out[0] = at::where(cond.to(at::kBool), t, e).expand(od).contiguous(); return; }
      at::Tensor cc = materialize(c, cond), tc = materialize(c, t), ec = materialize(c, e);
      c.out[0] = c.alloc_out(0);
      k::Bcast bc = make_bcast(od, tc, ec, &cc);
      k::select(c.out_dtype(), cc.data_ptr(), tc.data_ptr(), ec.data_ptr(), c.out[0].data_ptr(),
                c.out[0].numel(), bc, stream_of(c));
    };
    return d;
  };
  r.add("Select", make_select(false));
  r.add("SelectV2", make_select(true));
}

}  // namespace tfa

// The wider TF-1.x op set found in frozen model graphs beyond the reference's
// own examples: Pad / PadV2 / MirrorPad, Split / SplitV, Cumsum / Cumprod,
// LeakyRelu, ClipByValue, ReverseV2, DepthwiseConv2dNative, LRN, GatherNd.
// (The reference delegated every op to libtensorflow, so any op of a user's
// GraphDef was available there; reference:
// src/main/scala/org/tensorframes/impl/TensorFlowOps.scala:76-95.)
//
// Same contract as the other op files: CPU compute through ATen (the oracle),
// GPU compute through the HIP kernels of kernels/extra.hip (no ATen fallback
// on device tensors).
#include <cmath>

#include "ops_common.h"

namespace tfa {

void gpu_binary(ExecCtx& c, k::BinOp op, const at::Tensor& a0, const at::Tensor& b0);

namespace {

// row class: a ROW input stays ROW when dim 0 is untouched, CONST inputs fold
void rows_unless_axis0(InferCtx& c, bool touches_axis0) {
  if (c.all_const()) {
    for (auto& o : c.out) o.row = RowClass::CONST;
    return;
  }
  const bool ok = c.input(0).row == RowClass::ROW && !touches_axis0;
  for (size_t i = 1; i < c.in.size(); ++i)
    if (c.in[i]->row != RowClass::CONST) {
      for (auto& o : c.out) o.row = RowClass::MIXED;
      return;
    }
  for (auto& o : c.out) o.row = ok ? RowClass::ROW : RowClass::MIXED;
}

// ---------------------------------------------------------------- padding
std::vector<std::pair<int64_t, int64_t>> paddings_of(const std::vector<int64_t>& flat, int64_t rank,
                                                     const char* op) {
  TFA_CHECK(static_cast<int64_t>(flat.size()) == 2 * rank, op, ": paddings must be [", rank, ", 2], got ",
            flat.size(), " values");
  std::vector<std::pair<int64_t, int64_t>> p;
  for (int64_t d = 0; d < rank; ++d) {
    TFA_CHECK(flat[2 * d] >= 0 && flat[2 * d + 1] >= 0, op, ": paddings must be non-negative");
    p.push_back({flat[2 * d], flat[2 * d + 1]});
  }
  return p;
}

int mirror_mode(const Node& n) {
  if (n.op != "MirrorPad") return 0;
  std::string m = n.attr_s("mode", std::string("REFLECT"));
  TFA_CHECK(m == "REFLECT" || m == "SYMMETRIC", "MirrorPad: unknown mode '", m, "'");
  return m == "REFLECT" ? 1 : 2;
}

at::Tensor mirror_index(int64_t len, int64_t before, int64_t after, int mode) {
  std::vector<int64_t> idx;
  for (int64_t o = 0; o < len + before + after; ++o) {
    int64_t s = o - before;
    if (s < 0) s = mode == 1 ? -s : -s - 1;
    else if (s >= len) s = mode == 1 ? 2 * (len - 1) - s : 2 * len - 1 - s;
    idx.push_back(s);
  }
  return at::tensor(idx, at::kLong);
}

OpDef make_pad() {
  OpDef d;
  d.host_inputs = {1, 2};
  d.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto pv = c.ivalue(1);
    if (x.shape.unknown_rank) { c.set(0, x.dtype, Shape::unknown()); return; }
    std::vector<int64_t> dims = x.shape.dims;
    if (!pv) {
      for (auto& v : dims) v = -1;
    } else {
      auto p = paddings_of(*pv, x.shape.rank(), c.node.op.c_str());
      for (size_t i = 0; i < dims.size(); ++i)
        if (dims[i] >= 0) dims[i] += p[i].first + p[i].second;
    }
    c.set(0, x.dtype, Shape(dims));
  };
  d.rows = [](InferCtx& c) {
    auto pv = c.ivalue(1);
    bool axis0 = !pv || pv->size() < 2 || (*pv)[0] != 0 || (*pv)[1] != 0;
    rows_unless_axis0(c, axis0);
  };
  d.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    auto p = paddings_of(c.host_ivalue(1), x.dim(), c.node.op.c_str());
    const int mode = mirror_mode(c.node);
    double cval = 0.0;
    if (c.node.op == "PadV2") {
      const TensorInfo* t = c.in_info->at(2);
      at::Tensor v = t->value ? *t->value : c.input(2).to(at::kCPU);
      cval = v.to(at::kDouble).item<double>();
    }
    if (!c.gpu) {
      if (mode == 0) {
        std::vector<int64_t> pad;
        for (int64_t d = x.dim() - 1; d >= 0; --d) {
          pad.push_back(p[d].first);
          pad.push_back(p[d].second);
        }
        c.out[0] = at::constant_pad_nd(x, pad, cval).contiguous();
      } else {
        at::Tensor y = x;
        for (int64_t d = 0; d < x.dim(); ++d)
          if (p[d].first || p[d].second) {
            TFA_CHECK(p[d].first <= x.size(d) - (mode == 1) && p[d].second <= x.size(d) - (mode == 1),
                      "MirrorPad: paddings must not exceed the dimension size");
            y = y.index_select(d, mirror_index(x.size(d), p[d].first, p[d].second, mode));
          }
        c.out[0] = y.contiguous();
      }
      return;
    }
    at::Tensor xc = materialize(c, x);
    c.out[0] = c.alloc_out(0);
    if (!c.out[0].numel()) return;
    TFA_CHECK(xc.dim() >= 1 && xc.dim() <= k::kMaxRank, c.node.op, ": rank ", xc.dim(), " not supported");
    k::PadArgs a;
    a.rank = static_cast<int>(xc.dim());
    a.mode = mode;
    for (int d = 0; d < a.rank; ++d) {
      a.out_dims[d] = c.out[0].size(d);
      a.in_dims[d] = xc.size(d);
      a.in_strides[d] = xc.stride(d);
      a.before[d] = p[d].first;
    }
    // constant value as the element's bit pattern
    uint64_t bits = 0;
    at::Tensor cv = at::scalar_tensor(cval, at::kDouble).to(xc.scalar_type());
    std::memcpy(&bits, cv.data_ptr(), cv.element_size());
    k::pad_nd(xc.element_size(), a, xc.data_ptr(), c.out[0].data_ptr(), bits, stream_of(c));
  };
  return d;
}

// ---------------------------------------------------------------- split
OpDef make_split(bool v) {
  OpDef d;
  d.num_outputs = [](const Node& n) { return static_cast<int>(n.attr_i("num_split")); };
  d.host_inputs = v ? std::vector<int>{1, 2} : std::vector<int>{0};
  d.infer = [v](InferCtx& c) {
    const TensorInfo& x = c.input(v ? 0 : 1);
    const int ns = static_cast<int>(c.node.attr_i("num_split"));
    auto av = c.ivalue(v ? 2 : 0);
    if (x.shape.unknown_rank || !av) {
      for (int i = 0; i < ns; ++i) c.set(i, x.dtype, Shape::unknown());
      return;
    }
    const int64_t ax = norm_axis((*av)[0], x.shape.rank());
    const int64_t len = x.shape.dims[ax];
    std::vector<int64_t> sizes(ns, -1);
    if (!v) {
      if (len >= 0) {
        TFA_CHECK(len % ns == 0, "Split: dimension ", len, " not divisible by num_split ", ns);
        for (auto& s : sizes) s = len / ns;
      }
    } else {
      auto sv = c.ivalue(1);
      TFA_CHECK(sv && static_cast<int>(sv->size()) == ns, "SplitV: size_splits must have num_split values");
      int64_t known = 0, unk = -1;
      for (int i = 0; i < ns; ++i) {
        if ((*sv)[i] == -1) {
          TFA_CHECK(unk < 0, "SplitV: at most one -1 in size_splits");
          unk = i;
        } else {
          sizes[i] = (*sv)[i];
          known += (*sv)[i];
        }
      }
      if (unk >= 0) sizes[unk] = len >= 0 ? len - known : -1;
      else if (len >= 0) TFA_CHECK(known == len, "SplitV: sizes sum to ", known, ", dimension is ", len);
    }
    for (int i = 0; i < ns; ++i) {
      std::vector<int64_t> dims = x.shape.dims;
      dims[ax] = sizes[i];
      c.set(i, x.dtype, Shape(dims));
    }
  };
  d.rows = [v](InferCtx& c) {
    auto av = c.ivalue(v ? 2 : 0);
    const TensorInfo& x = c.input(v ? 0 : 1);
    if (c.all_const()) {
      for (auto& o : c.out) o.row = RowClass::CONST;
      return;
    }
    const bool ok = x.row == RowClass::ROW && av && x.shape.rank() > 0 &&
                    norm_axis((*av)[0], x.shape.rank()) != 0;
    for (auto& o : c.out) o.row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  d.compute = [v](ExecCtx& c) {
    at::Tensor x = c.input(v ? 0 : 1);
    const int64_t ax = norm_axis(c.host_ivalue(v ? 2 : 0)[0], x.dim());
    int64_t off = 0;
    for (size_t i = 0; i < c.out.size(); ++i) {
      const int64_t sz = c.out_info->at(i).shape.dims[ax];
      c.out[i] = materialize(c, x.narrow(ax, off, sz));
      off += sz;
    }
  };
  return d;
}

// ---------------------------------------------------------------- scans
OpDef make_scan(bool prod) {
  OpDef d;
  d.host_inputs = {1};
  d.infer = [](InferCtx& c) { infer_like(c); };
  d.rows = [](InferCtx& c) {
    auto av = c.ivalue(1);
    const int rk = c.input(0).shape.rank();
    rows_unless_axis0(c, !av || rk < 1 || norm_axis((*av)[0], rk) == 0);
  };
  d.compute = [prod](ExecCtx& c) {
    at::Tensor x = c.input(0);
    const int64_t ax = norm_axis(c.host_ivalue(1)[0], x.dim());
    const bool excl = c.node.attr_b("exclusive", false), rev = c.node.attr_b("reverse", false);
    if (!c.gpu) {
      at::Tensor t = rev ? x.flip({ax}) : x;
      at::Tensor r = prod ? at::cumprod(t, ax) : at::cumsum(t, ax);
      if (excl) {
        at::Tensor ident = prod ? at::ones_like(t.narrow(ax, 0, 1)) : at::zeros_like(t.narrow(ax, 0, 1));
        r = at::cat({ident, r.narrow(ax, 0, std::max<int64_t>(t.size(ax) - 1, 0))}, ax);
      }
      if (rev) r = r.flip({ax});
      c.out[0] = r.to(x.scalar_type()).contiguous();
      return;
    }
    require_gpu_dtype(x, {at::kFloat, at::kDouble, at::kInt, at::kLong}, c.node.op.c_str());
    at::Tensor xc = materialize(c, x);
    c.out[0] = c.alloc_out(0);
    int64_t outer = 1, inner = 1;
    for (int64_t i = 0; i < ax; ++i) outer *= xc.size(i);
    for (int64_t i = ax + 1; i < xc.dim(); ++i) inner *= xc.size(i);
    k::scan(prod, dt_of(xc), xc.data_ptr(), c.out[0].data_ptr(), outer, xc.size(ax), inner, excl, rev,
            stream_of(c));
  };
  return d;
}

// ---------------------------------------------------------------- depthwise conv
struct DwGeom {
  int64_t N, H, W, C, M, KH, KW, OH, OW, sh, sw, dh, dw, pt, pl, pb, pr;
};

void window(int64_t in, int64_t k, int64_t s, int64_t d, bool same, int64_t& out, int64_t& pb, int64_t& pa) {
  const int64_t eff = (k - 1) * d + 1;
  if (in < 0) { out = -1; pb = pa = 0; return; }
  if (same) {
    out = (in + s - 1) / s;
    const int64_t total = std::max<int64_t>((out - 1) * s + eff - in, 0);
    pb = total / 2;
    pa = total - pb;
  } else {
    out = in >= eff ? (in - eff) / s + 1 : 0;
    pb = pa = 0;
  }
}

DwGeom dw_geom(const Node& n, const std::vector<int64_t>& x, const std::vector<int64_t>& w) {
  TFA_CHECK(n.attr_s("data_format", std::string("NHWC")) == "NHWC", n.op, ": only NHWC is supported");
  auto st = n.attr_ilist("strides", {1, 1, 1, 1});
  auto dl = n.attr_ilist("dilations", {1, 1, 1, 1});
  TFA_CHECK(st.size() == 4 && st[0] == 1 && st[3] == 1, n.op, ": strides must be [1,sh,sw,1]");
  std::string pad = n.attr_s("padding");
  TFA_CHECK(pad == "SAME" || pad == "VALID", n.op, ": unsupported padding '", pad, "'");
  DwGeom g;
  g.N = x[0]; g.H = x[1]; g.W = x[2]; g.C = x[3];
  g.KH = w[0]; g.KW = w[1]; g.M = w[3];
  TFA_CHECK(w[2] == g.C || g.C < 0 || w[2] < 0, n.op, ": filter channels ", w[2], " != input channels ", g.C);
  g.sh = st[1]; g.sw = st[2];
  g.dh = dl.size() == 4 ? dl[1] : 1;
  g.dw = dl.size() == 4 ? dl[2] : 1;
  window(g.H, g.KH, g.sh, g.dh, pad == "SAME", g.OH, g.pt, g.pb);
  window(g.W, g.KW, g.sw, g.dw, pad == "SAME", g.OW, g.pl, g.pr);
  return g;
}

}  // namespace

void register_extra_ops(OpRegistry& r) {
  OpDef pad = make_pad();
  r.add("Pad", pad);
  r.add("PadV2", pad);
  r.add("MirrorPad", pad);
  r.add("Split", make_split(false));
  r.add("SplitV", make_split(true));
  r.add("Cumsum", make_scan(false));
  r.add("Cumprod", make_scan(true));

  // ---- LeakyRelu
  OpDef leaky;
  leaky.infer = [](InferCtx& c) { infer_like(c); };
  leaky.rows = [](InferCtx& c) { c.rows_like(0); };
  leaky.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    const double alpha = c.node.attr_f("alpha", 0.2f);
    if (!c.gpu) { c.out[0] = at::where(x >= 0, x, x * alpha).contiguous(); return; }
    require_gpu_dtype(x, {at::kFloat, at::kDouble}, "LeakyRelu");
    at::Tensor xc = materialize(c, x);
    c.out[0] = c.alloc_out(0);
    k::leaky_relu(dt_of(xc), xc.data_ptr(), c.out[0].data_ptr(), xc.numel(), alpha, stream_of(c));
  };
  r.add("LeakyRelu", leaky);

  // ---- ClipByValue(t, clip_value_min, clip_value_max)
  OpDef clip;
  clip.infer = [](InferCtx& c) {
    const TensorInfo& t = c.input(0);
    for (int i = 1; i <= 2; ++i)
      TFA_CHECK(c.input(i).dtype == t.dtype, "ClipByValue: bounds must have the tensor's dtype");
    c.set(0, t.dtype, t.shape);
  };
  clip.rows = [](InferCtx& c) { c.rows_elementwise(); };
  clip.compute = [](ExecCtx& c) {
    at::Tensor t = c.input(0);
    if (!c.gpu) {
      c.out[0] = at::minimum(at::maximum(t, c.input(1)), c.input(2)).expand(t.sizes()).contiguous();
      return;
    }
    require_gpu_dtype(t, {at::kFloat, at::kDouble, at::kInt, at::kLong}, "ClipByValue");
    gpu_binary(c, k::BinOp::MAX, t, c.input(1));
    at::Tensor lo = c.out[0];
    gpu_binary(c, k::BinOp::MIN, lo, c.input(2));
  };
  r.add("ClipByValue", clip);

  // ---- ReverseV2(tensor, axis)
  OpDef rev;
  rev.host_inputs = {1};
  rev.infer = [](InferCtx& c) { infer_like(c); };
  rev.rows = [](InferCtx& c) {
    auto av = c.ivalue(1);
    const int rk = c.input(0).shape.rank();
    bool axis0 = !av;
    if (av)
      for (auto a : *av) axis0 = axis0 || (rk > 0 && norm_axis(a, rk) == 0);
    rows_unless_axis0(c, axis0);
  };
  rev.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    std::vector<int64_t> axes;
    for (auto a : c.host_ivalue(1)) axes.push_back(norm_axis(a, x.dim()));
    if (!c.gpu) { c.out[0] = x.flip(axes).contiguous(); return; }
    at::Tensor xc = materialize(c, x);
    c.out[0] = c.alloc_out(0);
    if (!xc.numel()) return;
    TFA_CHECK(xc.dim() >= 1 && xc.dim() <= k::kMaxRank, "ReverseV2: rank ", xc.dim(), " not supported");
    std::vector<int64_t> dims = xc.sizes().vec(), ss = xc.strides().vec(), ds = c.out[0].strides().vec();
    const char* base = static_cast<const char*>(xc.data_ptr());
    for (auto a : axes) {
      base += (dims[a] - 1) * ss[a] * xc.element_size();
      ss[a] = -ss[a];
    }
    k::strided_copy(xc.element_size(), static_cast<int>(dims.size()), dims.data(), base, ss.data(),
                    c.out[0].data_ptr(), ds.data(), stream_of(c));
  };
  r.add("ReverseV2", rev);

  // ---- DepthwiseConv2dNative(input [N,H,W,C], filter [KH,KW,C,M])
  OpDef dw;
  dw.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    const TensorInfo& w = c.input(1);
    if (x.shape.unknown_rank || w.shape.unknown_rank) { c.set(0, x.dtype, Shape({-1, -1, -1, -1})); return; }
    TFA_CHECK(x.shape.rank() == 4 && w.shape.rank() == 4, c.node.op, " needs rank-4 input and filter");
    DwGeom g = dw_geom(c.node, x.shape.dims, w.shape.dims);
    c.set(0, x.dtype, Shape({g.N, g.OH, g.OW, (g.C < 0 || g.M < 0) ? -1 : g.C * g.M}));
  };
  dw.rows = [](InferCtx& c) { rows_unless_axis0(c, false); };
  dw.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0), w = c.input(1);
    DwGeom g = dw_geom(c.node, x.sizes().vec(), w.sizes().vec());
    if (!c.gpu) {
      at::Tensor xn = at::constant_pad_nd(x.permute({0, 3, 1, 2}), {g.pl, g.pr, g.pt, g.pb}, 0);
      // [KH,KW,C,M] -> [C*M, 1, KH, KW] (output channel c*M+m)
      at::Tensor wn = w.permute({2, 3, 0, 1}).reshape({g.C * g.M, 1, g.KH, g.KW});
      std::vector<int64_t> stride{g.sh, g.sw}, padz{0, 0}, dil{g.dh, g.dw};
      at::Tensor y = at::conv2d(xn, wn, c10::optional<at::Tensor>(), at::IntArrayRef(stride),
                                at::IntArrayRef(padz), at::IntArrayRef(dil), g.C);
      c.out[0] = y.permute({0, 2, 3, 1}).contiguous();
      return;
    }
    require_gpu_dtype(x, {at::kFloat}, "DepthwiseConv2dNative");
    at::Tensor xc = materialize(c, x), wc = materialize(c, w);
    c.out[0] = c.alloc_out(0);
    k::DepthwiseArgs a;
    a.N = g.N; a.H = g.H; a.W = g.W; a.C = g.C; a.M = g.M; a.KH = g.KH; a.KW = g.KW;
    a.OH = g.OH; a.OW = g.OW; a.sh = g.sh; a.sw = g.sw; a.dh = g.dh; a.dw = g.dw;
    a.pad_t = g.pt; a.pad_l = g.pl;
    a.x = xc.data_ptr(); a.w = wc.data_ptr(); a.y = c.out[0].data_ptr();
    k::depthwise_conv2d_nhwc(a, stream_of(c));
  };
  r.add("DepthwiseConv2dNative", dw);

  // ---- LRN (across the channel / last dim)
  OpDef lrn;
  lrn.infer = [](InferCtx& c) { infer_like(c); };
  lrn.rows = [](InferCtx& c) { rows_unless_axis0(c, c.input(0).shape.rank() < 2); };
  lrn.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    const int64_t radius = c.node.attr_i("depth_radius", 5);
    const double bias = c.node.attr_f("bias", 1.f), alpha = c.node.attr_f("alpha", 1.f),
                 beta = c.node.attr_f("beta", 0.5f);
    const int64_t C = x.size(-1);
    if (!c.gpu) {
      at::Tensor sq = (x.to(at::kDouble) * x.to(at::kDouble));
      at::Tensor cs = at::cumsum(at::constant_pad_nd(sq, {radius + 1, radius}, 0), -1);
      at::Tensor win = cs.narrow(-1, 2 * radius + 1, C) - cs.narrow(-1, 0, C);
      c.out[0] = (x.to(at::kDouble) / at::pow(bias + alpha * win, beta)).to(x.scalar_type()).contiguous();
      return;
    }
    require_gpu_dtype(x, {at::kFloat, at::kDouble}, "LRN");
    at::Tensor xc = materialize(c, x);
    c.out[0] = c.alloc_out(0);
    k::lrn(dt_of(xc), xc.data_ptr(), c.out[0].data_ptr(), xc.numel(), C, static_cast<int>(radius), bias, alpha,
           beta, stream_of(c));
  };
  r.add("LRN", lrn);

  // ---- GatherNd(params, indices)
  OpDef gnd;
  gnd.infer = [](InferCtx& c) {
    const TensorInfo& p = c.input(0);
    const TensorInfo& ix = c.input(1);
    if (p.shape.unknown_rank || ix.shape.unknown_rank || ix.shape.dims.empty() || ix.shape.dims.back() < 0) {
      c.set(0, p.dtype, Shape::unknown());
      return;
    }
    const int64_t K = ix.shape.dims.back();
    TFA_CHECK(K <= p.shape.rank(), "GatherNd: index depth ", K, " > params rank ", p.shape.rank());
    std::vector<int64_t> dims(ix.shape.dims.begin(), ix.shape.dims.end() - 1);
    for (int64_t d = K; d < p.shape.rank(); ++d) dims.push_back(p.shape.dims[d]);
    c.set(0, p.dtype, Shape(dims));
  };
  gnd.rows = [](InferCtx& c) {
    if (c.all_const()) { c.out[0].row = RowClass::CONST; return; }
    const bool ok = c.input(0).row == RowClass::CONST && c.input(1).row == RowClass::ROW &&
                    c.input(1).shape.rank() >= 2;
    c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  gnd.compute = [](ExecCtx& c) {
    at::Tensor p = c.input(0), ix = c.input(1);
    const int64_t K = ix.size(-1);
    int64_t inner = 1;
    for (int64_t d = K; d < p.dim(); ++d) inner *= p.size(d);
    const int64_t nidx = ix.numel() / std::max<int64_t>(K, 1);
    if (!c.gpu) {
      at::Tensor flat_ix = ix.reshape({nidx, K}).to(at::kLong);
      at::Tensor off = at::zeros({nidx}, at::kLong);
      int64_t stride = 1;
      for (int64_t d = K - 1; d >= 0; --d) {
        at::Tensor v = flat_ix.select(1, d);
        TFA_CHECK((v >= 0).all().item<bool>() && (v < p.size(d)).all().item<bool>(),
                  "GatherNd: index out of range for dim ", d, " of size ", p.size(d));
        off = off + v * stride;
        stride *= p.size(d);
      }
      at::Tensor rows = p.contiguous().reshape({stride, inner}).index_select(0, off);
      c.out[0] = rows.reshape(c.out_shape().dims).contiguous();
      return;
    }
    at::Tensor pc = materialize(c, p), ic = materialize(c, ix);
    TFA_CHECK(ic.scalar_type() == at::kInt || ic.scalar_type() == at::kLong, "GatherNd: indices must be int32/int64");
    c.out[0] = c.alloc_out(0);
    k::GatherNdArgs a;
    a.K = static_cast<int>(K);
    int64_t stride = 1;
    for (int64_t d = K - 1; d >= 0; --d) {
      a.dims[d] = pc.size(d);
      a.strides[d] = stride;
      stride *= pc.size(d);
    }
    k::gather_nd(pc.element_size(), dt_of(ic), pc.data_ptr(), ic.data_ptr(), c.out[0].data_ptr(), nidx, inner, a,
                 stream_of(c));
  };
  r.add("GatherNd", gnd);
}

}  // namespace tfa

// NN ops: BiasAdd, Softmax, Conv2D, pooling, FusedBatchNorm (inference), TopKV2.
//
// These are the ops of the CNN-scoring workloads (frozen VGG / Inception
// GraphDefs; reference: src/main/python/tensorframes_snippets/read_image.py:56-118).
// Layout is TF's default NHWC.
#include <cmath>
#include <limits>

#include "ops_common.h"

namespace tfa {


namespace {

bool nchw(const Node& n) { return n.attr_s("data_format", std::string("NHWC")) == "NCHW"; }

void window_out(int64_t in, int64_t k, int64_t s, int64_t d, bool same, int64_t& out,
                int64_t& pad_before, int64_t& pad_after) {
  int64_t eff = (k - 1) * d + 1;
  if (in < 0) { out = -1; pad_before = pad_after = 0; return; }
  if (same) {
    out = (in + s - 1) / s;
    int64_t total = std::max<int64_t>((out - 1) * s + eff - in, 0);
    pad_before = total / 2;
    pad_after = total - pad_before;
  } else {
    out = in >= eff ? (in - eff) / s + 1 : 0;
    pad_before = pad_after = 0;
  }
}

bool is_same(const Node& n) {
  std::string p = n.attr_s("padding");
  TFA_CHECK(p == "SAME" || p == "VALID", n.op, ": unsupported padding '", p, "'");
  return p == "SAME";
}

struct Conv2DGeom {
  int64_t N, H, W, C, KH, KW, OC, OH, OW, sh, sw, dh, dw, pt, pb, pl, pr;
};

Conv2DGeom conv_geom(const Node& n, const std::vector<int64_t>& x, const std::vector<int64_t>& w) {
  TFA_CHECK(!nchw(n), n.op, ": only data_format NHWC is supported");
  auto st = n.attr_ilist("strides", {1, 1, 1, 1});
  auto dl = n.attr_ilist("dilations", {1, 1, 1, 1});
  TFA_CHECK(st.size() == 4 && st[0] == 1 && st[3] == 1, n.op, ": strides must be [1,sh,sw,1]");
  Conv2DGeom g;
  g.N = x[0]; g.H = x[1]; g.W = x[2]; g.C = x[3];
  g.KH = w[0]; g.KW = w[1]; g.OC = w[3];
  TFA_CHECK(w[2] == g.C || g.C < 0 || w[2] < 0, n.op, ": filter in-channels ", w[2], " != input channels ", g.C);
  g.sh = st[1]; g.sw = st[2];
  g.dh = dl.size() == 4 ? dl[1] : 1;
  g.dw = dl.size() == 4 ? dl[2] : 1;
  bool same = is_same(n);
  window_out(g.H, g.KH, g.sh, g.dh, same, g.OH, g.pt, g.pb);
  window_out(g.W, g.KW, g.sw, g.dw, same, g.OW, g.pl, g.pr);
  return g;
}

struct PoolGeom {
  int64_t N, H, W, C, KH, KW, sh, sw, OH, OW, pt, pb, pl, pr;
};

PoolGeom pool_geom(const Node& n, const std::vector<int64_t>& x) {
  TFA_CHECK(!nchw(n), n.op, ": only data_format NHWC is supported");
  auto ks = n.attr_ilist("ksize");
  auto st = n.attr_ilist("strides");
  TFA_CHECK(ks.size() == 4 && ks[0] == 1 && ks[3] == 1, n.op, ": ksize must be [1,kh,kw,1]");
  TFA_CHECK(st.size() == 4 && st[0] == 1 && st[3] == 1, n.op, ": strides must be [1,sh,sw,1]");
  PoolGeom g;
  g.N = x[0]; g.H = x[1]; g.W = x[2]; g.C = x[3];
  g.KH = ks[1]; g.KW = ks[2]; g.sh = st[1]; g.sw = st[2];
  bool same = is_same(n);
  window_out(g.H, g.KH, g.sh, 1, same, g.OH, g.pt, g.pb);
  window_out(g.W, g.KW, g.sw, 1, same, g.OW, g.pl, g.pr);
  return g;
}

void rows_batch(InferCtx& c) {
  // NHWC ops are row-local over N when their parameters are constant
  if (c.all_const()) { for (auto& o : c.out) o.row = RowClass::CONST; return; }
  bool ok = c.input(0).row == RowClass::ROW;
  for (size_t i = 1; i < c.in.size(); ++i) ok = ok && c.in[i]->row == RowClass::CONST;
  for (auto& o : c.out) o.row = ok ? RowClass::ROW : RowClass::MIXED;
}

// the planner's Winograd filter: device-resident, f32, [C/4][16][OCP][4]
const void* wino_filter_ptr(const at::Tensor& u, int64_t KH, int64_t KW, int64_t C, int64_t OC) {
  const int kind = k::conv_wino_kind(KH, KW, 1, 1, 1, 1, C, OC);
  TFA_CHECK(kind != 0 && u.is_cuda() && u.scalar_type() == at::kFloat && u.is_contiguous() &&
                u.numel() == k::conv_wino_filter_elems(kind, C, OC),
            "internal: Winograd filter layout");
  return u.data_ptr();
}

}  // namespace

// planner-fused pool step (GPU): Pool -> BiasAdd -> Relu/Relu6 in one pass,
// written into `out`, possibly a channel slice of a concat output
void run_pool_fused(ExecCtx& c, bool is_max, const at::Tensor& x0, const at::Tensor* bias, int act,
                    const at::Tensor& out) {
  at::Tensor x = materialize(c, x0);
  require_gpu_dtype(x, {at::kFloat}, c.node.op.c_str());
  PoolGeom g = pool_geom(c.node, x.sizes().vec());
  TFA_CHECK(out.dim() == 4 && out.size(0) == g.N && out.size(1) == g.OH && out.size(2) == g.OW &&
                out.size(3) == g.C && out.stride(3) == 1 && out.stride(1) == out.stride(2) * g.OW &&
                out.stride(0) == out.stride(1) * g.OH,
            "internal: fused pool output layout");
  if (!out.numel()) return;
  k::PoolArgs a;
  a.N = g.N; a.H = g.H; a.W = g.W; a.C = g.C; a.OH = g.OH; a.OW = g.OW;
  a.KH = g.KH; a.KW = g.KW; a.sh = g.sh; a.sw = g.sw; a.pad_t = g.pt; a.pad_l = g.pl;
  a.is_max = is_max;
  a.x = x.data_ptr();
  a.y = out.data_ptr();
  if (bias) {
    TFA_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == g.C,
              "internal: fused pool bias");
    a.bias = bias->data_ptr();
  }
  a.act = act;
  a.ldc = out.stride(2) == g.C ? 0 : out.stride(2);
  k::pool2d_nhwc(DType::F32, a, stream_of(c));
}

// shared with the planner's fused conv epilogue
void run_conv2d(ExecCtx& c, const at::Tensor& x0, const at::Tensor& w0, const at::Tensor* bias,
                int act, at::Tensor& out, const std::vector<EpiStep>* epi, const at::Tensor* wino, bool pool2,
                const int* pool_in) {
  if (pool_in) {
    TFA_CHECK(c.gpu && !epi && !wino && !pool2 && x0.dim() == 4 && w0.dim() == 4 && w0.size(0) == 1 &&
                  w0.size(1) == 1,
              "internal: pooled-input conv step");
    require_gpu_dtype(x0, {at::kFloat}, "Conv2D");
    at::Tensor x = materialize(c, x0), w = materialize(c, w0);
    const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), OC = w.size(3);
    const int64_t PH = (H - pool_in[0]) / pool_in[2] + 1, PW = (W - pool_in[1]) / pool_in[3] + 1;
    TFA_CHECK(H >= pool_in[0] && W >= pool_in[1] && w.size(2) == C, "internal: pooled-input conv geometry");
    TFA_CHECK(out.dim() == 4 && out.size(0) == N && out.size(1) == PH && out.size(2) == PW && out.size(3) == OC &&
                  out.stride(3) == 1 && out.stride(1) == PW * out.stride(2) && out.stride(0) == PH * out.stride(1),
              "internal: pooled-input conv output");
    if (out.numel() == 0) return;
    const int64_t ldc = out.stride(2);
    if (pool_in[0] == 3 && pool_in[1] == 3 && k::pool_conv1x1_eligible(N, H, W, C, PH, PW, OC, ldc, act) &&
        (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0) {
      k::PoolConvArgs a;
      a.N = N; a.H = H; a.W = W; a.C = C; a.PH = PH; a.PW = PW;
      a.pkh = pool_in[0]; a.pkw = pool_in[1]; a.psh = pool_in[2]; a.psw = pool_in[3];
      a.OC = OC; a.ldc = ldc;
      a.x = x.data_ptr(); a.w = w.data_ptr(); a.y = out.data_ptr();
      a.bias = bias ? bias->data_ptr() : nullptr;
      a.act = act;
      k::set_last_conv_algo("maxpool3x3+conv1x1");
      k::pool_conv1x1(a, stream_of(c));
      return;
    }
    at::Tensor pooled = c.alloc({N, PH, PW, C}, x.options());
    k::PoolArgs pa;
    pa.N = N; pa.H = H; pa.W = W; pa.C = C; pa.OH = PH; pa.OW = PW;
    pa.KH = pool_in[0]; pa.KW = pool_in[1]; pa.sh = pool_in[2]; pa.sw = pool_in[3]; pa.pad_t = 0; pa.pad_l = 0;
    pa.is_max = true;
    pa.x = x.data_ptr();
    pa.y = pooled.data_ptr();
    k::pool2d_nhwc(DType::F32, pa, stream_of(c));
    run_conv2d(c, pooled, w, bias, act, out);
    return;
  }
  Conv2DGeom g = conv_geom(c.node, x0.sizes().vec(), w0.sizes().vec());
  TFA_CHECK(!pool2 || (c.gpu && !epi && g.OH % 2 == 0 && g.OW % 2 == 0), "internal: pooled conv step");
  if (!c.gpu) {
    at::Tensor x = x0.permute({0, 3, 1, 2});
    x = at::constant_pad_nd(x, {g.pl, g.pr, g.pt, g.pb}, 0);
    at::Tensor w = w0.permute({3, 2, 0, 1});
    std::vector<int64_t> stride{g.sh, g.sw}, pad{0, 0}, dil{g.dh, g.dw};
    at::Tensor y = at::conv2d(x, w, c10::optional<at::Tensor>(), at::IntArrayRef(stride),
                              at::IntArrayRef(pad), at::IntArrayRef(dil), 1);
    y = y.permute({0, 2, 3, 1});
    if (bias) y = y + *bias;
    y = apply_act_host(y, act);
    if (epi) y = apply_epi_host(y.reshape({-1, g.OC}), epi).reshape(y.sizes());
    out = y.contiguous();
    return;
  }
  require_gpu_dtype(x0, {at::kFloat}, "Conv2D");
  at::Tensor x = materialize(c, x0), w = materialize(c, w0);
  if (out.numel() == 0) return;
  if (pool2) {
    TFA_CHECK(out.dim() == 4 && out.size(0) == g.N && out.size(1) == g.OH / 2 && out.size(2) == g.OW / 2 &&
                  out.size(3) == g.OC,
              "internal: pooled conv output shape");
  }
  k::ConvArgs a;
  a.N = g.N; a.H = g.H; a.W = g.W; a.C = g.C;
  a.KH = g.KH; a.KW = g.KW; a.OC = g.OC; a.OH = g.OH; a.OW = g.OW;
  a.sh = g.sh; a.sw = g.sw; a.dh = g.dh; a.dw = g.dw; a.pad_t = g.pt; a.pad_l = g.pl;
  a.x = x.data_ptr(); a.w = w.data_ptr(); a.y = out.data_ptr();
  a.bias = bias ? bias->data_ptr() : nullptr;
  a.act = act;
  a.epi = epi_prog(epi);
  // `out` may be a channel slice of a wider NHWC tensor (concat write-into-slice)
  TFA_CHECK(out.stride(3) == 1 && out.stride(1) == out.size(2) * out.stride(2) &&
                out.stride(0) == out.size(1) * out.stride(1),
            "Conv2D: output must be NHWC-contiguous up to the channel stride");
  a.ldc = out.stride(2);
  if (wino) a.wino = wino_filter_ptr(*wino, g.KH, g.KW, g.C, g.OC);
  at::Tensor conv_out;  // pool2 without a pooled epilogue: the conv's own output, pooled after
  if (pool2) {
    a.pool2 = k::conv2d_pool2_direct(a);
    if (!a.pool2) {
      conv_out = c.alloc({g.N, g.OH, g.OW, g.OC}, x.options());
      a.y = conv_out.data_ptr();
      a.ldc = g.OC;
    }
  }
  at::Tensor work;
  if (size_t ws = k::conv2d_workspace_bytes(DType::F32, a)) {
    work = c.alloc({static_cast<int64_t>(ws)}, x.options().dtype(at::kByte));
    a.workspace = work.data_ptr();
  }
  k::conv2d_nhwc(DType::F32, a, stream_of(c));
  if (conv_out.defined()) {
    k::PoolArgs pa;
    pa.N = g.N; pa.H = g.OH; pa.W = g.OW; pa.C = g.OC; pa.OH = g.OH / 2; pa.OW = g.OW / 2;
    pa.KH = 2; pa.KW = 2; pa.sh = 2; pa.sw = 2; pa.pad_t = 0; pa.pad_l = 0;
    pa.is_max = true;
    pa.x = conv_out.data_ptr();
    pa.y = out.data_ptr();
    pa.ldc = out.stride(2) == g.OC ? 0 : out.stride(2);
    k::pool2d_nhwc(DType::F32, pa, stream_of(c));
  }
}

void run_conv2d_siblings(ExecCtx& c, const at::Tensor& x0, const at::Tensor& w0, const at::Tensor* bias, int act,
                         std::vector<at::Tensor>& outs, const std::vector<int>& acts, const at::Tensor* wino) {
  TFA_CHECK(c.gpu, "Conv2D siblings: GPU plans only");
  TFA_CHECK(!outs.empty() && outs.size() <= static_cast<size_t>(k::kMaxOutSegs), "Conv2D siblings: 1..",
            k::kMaxOutSegs, " outputs");
  Conv2DGeom g = conv_geom(c.node, x0.sizes().vec(), w0.sizes().vec());
  require_gpu_dtype(x0, {at::kFloat}, "Conv2D");
  at::Tensor x = materialize(c, x0), w = materialize(c, w0);
  k::ConvArgs a;
  a.N = g.N; a.H = g.H; a.W = g.W; a.C = g.C;
  a.KH = g.KH; a.KW = g.KW; a.OC = g.OC; a.OH = g.OH; a.OW = g.OW;
  a.sh = g.sh; a.sw = g.sw; a.dh = g.dh; a.dw = g.dw; a.pad_t = g.pt; a.pad_l = g.pl;
  a.x = x.data_ptr(); a.w = w.data_ptr();
  a.bias = bias ? bias->data_ptr() : nullptr;
  a.act = act;
  int64_t begin = 0;
  a.seg.n = static_cast<int>(outs.size());
  for (size_t k = 0; k < outs.size(); ++k) {
    const at::Tensor& o = outs[k];
    TFA_CHECK(o.dim() == 4 && o.size(0) == g.N && o.size(1) == g.OH && o.size(2) == g.OW,
              "Conv2D siblings: output ", k, " has the wrong spatial shape");
    TFA_CHECK(o.stride(3) == 1 && o.stride(1) == o.size(2) * o.stride(2) && o.stride(0) == o.size(1) * o.stride(1),
              "Conv2D siblings: outputs must be NHWC-contiguous up to the channel stride");
    a.seg.begin[k] = begin;
    a.seg.ptr[k] = o.data_ptr();
    a.seg.ldc[k] = o.stride(2);
    a.seg.act[k] = k < acts.size() ? acts[k] : act;
    begin += o.size(3);
  }
  a.seg.begin[outs.size()] = begin;
  TFA_CHECK(begin == g.OC, "Conv2D siblings: outputs cover ", begin, " channels of ", g.OC);
  a.y = outs[0].data_ptr();
  a.ldc = outs[0].stride(2);
  if (wino) a.wino = wino_filter_ptr(*wino, g.KH, g.KW, g.C, g.OC);
  if (g.N * g.OH * g.OW == 0) return;
  at::Tensor work;
  if (size_t ws = k::conv2d_workspace_bytes(DType::F32, a)) {
    work = c.alloc({static_cast<int64_t>(ws)}, x.options().dtype(at::kByte));
    a.workspace = work.data_ptr();
  }
  k::conv2d_nhwc(DType::F32, a, stream_of(c));
}

void register_nn_ops(OpRegistry& r) {
  // ---- BiasAdd
  OpDef bias;
  bias.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    const TensorInfo& b = c.input(1);
    TFA_CHECK(x.dtype == b.dtype, "BiasAdd: dtype mismatch");
    TFA_CHECK(b.shape.rank() == 1 || b.shape.unknown_rank, "BiasAdd: bias must be a vector");
    c.set(0, x.dtype, x.shape);
  };
  bias.rows = [](InferCtx& c) { c.rows_elementwise(); };
  bias.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0), b = c.input(1);
    bool cf = nchw(c.node);
    at::Tensor bb = b;
    if (cf && x.dim() > 2) {
      std::vector<int64_t> s(x.dim(), 1);
      s[1] = b.size(0);
      bb = b.reshape(s);
    }
    if (!c.gpu) { c.out[0] = (x + bb).contiguous(); return; }
    require_gpu_dtype(x, {at::kFloat, at::kDouble, at::kInt, at::kLong}, "BiasAdd");
    at::Tensor xc = materialize(c, x), bc = materialize(c, bb);
    c.out[0] = c.alloc_out(0);
    int64_t n = xc.numel();
    if (!n) return;
    if (!cf || x.dim() <= 2) {
      TFA_CHECK(bc.numel() == x.size(-1), "BiasAdd: bias length ", bc.numel(), " != last dim ", x.size(-1));
      k::binary(k::BinOp::ADD, dt_of(xc), xc.data_ptr(), bc.data_ptr(), c.out[0].data_ptr(), n, 3,
                x.size(-1), nullptr, stream_of(c));
    } else {
      k::Bcast bcd = make_bcast(x.sizes().vec(), xc, bc);
      k::binary(k::BinOp::ADD, dt_of(xc), xc.data_ptr(), bc.data_ptr(), c.out[0].data_ptr(), n, 4,
                1, &bcd, stream_of(c));
    }
  };
  r.add("BiasAdd", bias);
  r.add("BiasAddV1", bias);

  // ---- Softmax / LogSoftmax (last axis)
  auto make_softmax = [](bool log) {
    OpDef d;
    d.infer = [](InferCtx& c) { infer_like(c); };
    d.rows = [](InferCtx& c) {
      c.rows_like(0);
      if (c.out[0].row == RowClass::ROW && c.input(0).shape.rank() < 2) c.out[0].row = RowClass::MIXED;
    };
    d.compute = [log](ExecCtx& c) {
      at::Tensor x = c.input(0);
      if (!c.gpu) { c.out[0] = (log ? at::log_softmax(x, -1) : at::softmax(x, -1)).contiguous(); return; }
      require_gpu_dtype(x, {at::kFloat, at::kDouble}, "Softmax");
      at::Tensor xc = materialize(c, x);
      c.out[0] = c.alloc_out(0);
      int64_t cols = xc.dim() ? xc.size(-1) : 1;
      if (xc.numel()) k::softmax(dt_of(xc), log, xc.data_ptr(), c.out[0].data_ptr(), xc.numel() / cols, cols, stream_of(c));
    };
    return d;
  };
  r.add("Softmax", make_softmax(false));
  r.add("LogSoftmax", make_softmax(true));

  // ---- Conv2D
  OpDef conv;
  conv.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    const TensorInfo& w = c.input(1);
    TFA_CHECK(x.dtype == w.dtype, "Conv2D: dtype mismatch");
    if (x.shape.unknown_rank || w.shape.unknown_rank) {
      c.set(0, x.dtype, Shape({-1, -1, -1, -1}));
      return;
    }
    TFA_CHECK(x.shape.rank() == 4 && w.shape.rank() == 4, "Conv2D needs rank-4 input and filter");
    Conv2DGeom g = conv_geom(c.node, x.shape.dims, w.shape.dims);
    c.set(0, x.dtype, Shape({g.N, g.OH, g.OW, g.OC}));
  };
  conv.rows = rows_batch;
  conv.compute = [](ExecCtx& c) {
    at::Tensor out = c.gpu ? c.alloc_out(0) : at::Tensor();
    run_conv2d(c, c.input(0), c.input(1), nullptr, 0, out);
    c.out[0] = out;
  };
  r.add("Conv2D", conv);

  // ---- MaxPool / AvgPool
  auto make_pool = [](bool is_max) {
    OpDef d;
    d.infer = [](InferCtx& c) {
      const TensorInfo& x = c.input(0);
      if (x.shape.unknown_rank) { c.set(0, x.dtype, Shape({-1, -1, -1, -1})); return; }
      TFA_CHECK(x.shape.rank() == 4, c.node.op, " needs a rank-4 input");
      PoolGeom g = pool_geom(c.node, x.shape.dims);
      c.set(0, x.dtype, Shape({g.N, g.OH, g.OW, g.C}));
    };
    d.rows = rows_batch;
    d.compute = [is_max](ExecCtx& c) {
      at::Tensor x = c.input(0);
      PoolGeom g = pool_geom(c.node, x.sizes().vec());
      if (!c.gpu) {
        at::Tensor xn = x.permute({0, 3, 1, 2});
        at::Tensor y;
        if (is_max) {
          double lo = -std::numeric_limits<double>::infinity();
          at::Tensor xp = at::constant_pad_nd(xn, {g.pl, g.pr, g.pt, g.pb}, lo);
          y = at::max_pool2d(xp, {g.KH, g.KW}, {g.sh, g.sw});
        } else {
          at::Tensor xp = at::constant_pad_nd(xn, {g.pl, g.pr, g.pt, g.pb}, 0);
          at::Tensor ones = at::constant_pad_nd(at::ones_like(xn.narrow(1, 0, 1)), {g.pl, g.pr, g.pt, g.pb}, 0);
          at::Tensor s = at::avg_pool2d(xp, {g.KH, g.KW}, {g.sh, g.sw});
          at::Tensor cnt = at::avg_pool2d(ones, {g.KH, g.KW}, {g.sh, g.sw});
          y = s / cnt;
        }
        c.out[0] = y.permute({0, 2, 3, 1}).contiguous();
        return;
      }
      require_gpu_dtype(x, {at::kFloat}, c.node.op.c_str());
      at::Tensor xc = materialize(c, x);
      c.out[0] = c.alloc_out(0);
      if (!c.out[0].numel()) return;
      k::PoolArgs a;
      a.N = g.N; a.H = g.H; a.W = g.W; a.C = g.C; a.OH = g.OH; a.OW = g.OW;
      a.KH = g.KH; a.KW = g.KW; a.sh = g.sh; a.sw = g.sw; a.pad_t = g.pt; a.pad_l = g.pl;
      a.is_max = is_max;
      a.x = xc.data_ptr();
      a.y = c.out[0].data_ptr();
      k::pool2d_nhwc(DType::F32, a, stream_of(c));
    };
    return d;
  };
  r.add("MaxPool", make_pool(true));
  r.add("AvgPool", make_pool(false));

  // ---- ResizeBilinear / ResizeNearestNeighbor (images [N,H,W,C], size int32[2])
  auto make_resize = [](bool bilinear) {
    OpDef d;
    d.host_inputs = {1};
    d.infer = [bilinear](InferCtx& c) {
      const TensorInfo& x = c.input(0);
      DType odt = bilinear ? DType::F32 : x.dtype;
      auto sz = c.ivalue(1);
      int64_t oh = sz ? (*sz).at(0) : -1, ow = sz ? (*sz).at(1) : -1;
      if (sz) TFA_CHECK(sz->size() == 2 && oh > 0 && ow > 0, c.node.op, ": size must be 2 positive ints");
      if (x.shape.unknown_rank) { c.set(0, odt, Shape({-1, oh, ow, -1})); return; }
      TFA_CHECK(x.shape.rank() == 4, c.node.op, " needs a rank-4 [batch,height,width,channels] input");
      c.set(0, odt, Shape({x.shape.dims[0], oh, ow, x.shape.dims[3]}));
    };
    d.rows = rows_batch;
    d.compute = [bilinear](ExecCtx& c) {
      at::Tensor x = c.input(0);
      auto sz = c.host_ivalue(1);
      TFA_CHECK(sz.size() == 2 && sz[0] > 0 && sz[1] > 0, c.node.op, ": size must be 2 positive ints");
      const bool align = c.node.attr_b("align_corners", false);
      const bool half = c.node.attr_b("half_pixel_centers", false);
      TFA_CHECK(!(align && half), c.node.op, ": align_corners and half_pixel_centers are exclusive");
      const int64_t H = x.size(1), W = x.size(2), OH = sz[0], OW = sz[1];
      auto scale = [&](int64_t in, int64_t out) {
        return (align && out > 1) ? float(in - 1) / float(out - 1) : float(in) / float(out);
      };
      const float sh = scale(H, OH), sw = scale(W, OW);
      const int mode = align ? 1 : (half ? 2 : 0);
      if (!c.gpu) {
        // oracle: same formulas in float on the host
        auto idx = [&](int64_t out, int64_t in, float s) {
          at::Tensor d = at::arange(out, at::kFloat);
          return mode == 2 ? (d + 0.5f) * s - 0.5f : d * s;
        };
        at::Tensor fy = idx(OH, H, sh), fx = idx(OW, W, sw);
        if (!bilinear) {
          auto pick = [&](const at::Tensor& f, int64_t out, int64_t in, float s) {
            at::Tensor d = at::arange(out, at::kFloat);
            at::Tensor v = mode == 1 ? at::round(d * s) : (mode == 2 ? at::floor((d + 0.5f) * s) : at::floor(d * s));
            return v.to(at::kLong).clamp(0, in - 1);
          };
          at::Tensor iy = pick(fy, OH, H, sh), ix = pick(fx, OW, W, sw);
          c.out[0] = x.index_select(1, iy).index_select(2, ix).contiguous();
          return;
        }
        at::Tensor xf = x.to(at::kFloat);
        at::Tensor y0 = at::floor(fy).to(at::kLong).clamp_min(0), y1 = at::ceil(fy).to(at::kLong).clamp_max(H - 1);
        at::Tensor x0 = at::floor(fx).to(at::kLong).clamp_min(0), x1 = at::ceil(fx).to(at::kLong).clamp_max(W - 1);
        y0 = y0.clamp_max(H - 1);
        x0 = x0.clamp_max(W - 1);
        at::Tensor ly = (fy - at::floor(fy)).view({1, OH, 1, 1}), lx = (fx - at::floor(fx)).view({1, 1, OW, 1});
        at::Tensor top = xf.index_select(1, y0), bot = xf.index_select(1, y1);
        at::Tensor tl = top.index_select(2, x0), tr = top.index_select(2, x1);
        at::Tensor bl = bot.index_select(2, x0), br = bot.index_select(2, x1);
        at::Tensor t = tl + (tr - tl) * lx, b = bl + (br - bl) * lx;
        c.out[0] = (t + (b - t) * ly).contiguous();
        return;
      }
      at::Tensor xc = materialize(c, x);
      c.out[0] = c.alloc_out(0);
      if (!c.out[0].numel()) return;
      k::ResizeArgs a;
      a.N = xc.size(0); a.H = H; a.W = W; a.C = xc.size(3); a.OH = OH; a.OW = OW;
      a.sh = sh; a.sw = sw; a.mode = mode;
      a.x = xc.data_ptr(); a.y = c.out[0].data_ptr();
      if (bilinear) k::resize_bilinear(dt_of(xc), a, stream_of(c));
      else k::resize_nearest(xc.element_size(), a, stream_of(c));
    };
    return d;
  };
  r.add("ResizeBilinear", make_resize(true));
  r.add("ResizeNearestNeighbor", make_resize(false));

  // ---- image decoders: host ops. Shapes/dtypes are inferred here so graphs
  // containing them analyze; the decode itself runs in the Python host stage
  // (tensorframes_amd/ops/host_ops.py), which feeds the decoded uint8 HWC
  // tensor in place of the node's output (reference example:
  // src/main/python/tensorframes_snippets/read_image.py:42,165).
  auto make_decode = [](const char* op) {
    OpDef d;
    d.stateful = true;  // never constant-folded
    d.host_only = true;
    d.infer = [](InferCtx& c) {
      TFA_CHECK(c.input(0).dtype == DType::STRING, c.node.op, ": contents must be a string tensor");
      int64_t ch = c.node.attr_i("channels", 0);
      DType odt = DType::U8;
      if (c.node.op == "DecodePng" || c.node.op == "DecodeImage") {
        int dt = static_cast<int>(c.node.attr_i("dtype", 4));
        odt = static_cast<DType>(dt);
      }
      c.set(0, odt, Shape({-1, -1, ch > 0 ? ch : -1}));
    };
    d.compute = [op](ExecCtx& c) {
      TFA_CHECK(false, op, " (node '", c.node.name, "') is a host op: it is decoded on the host by the "
                "map_rows host stage; feed its output or use map_rows with a binary column");
    };
    return d;
  };
  for (const char* op : {"DecodeJpeg", "DecodePng", "DecodeImage", "DecodeBmp"}) r.add(op, make_decode(op));

  // ---- FusedBatchNorm (inference): y = x*s + b with s = scale/sqrt(var+eps)
  auto make_bn = [](int nout) {
    OpDef d;
    d.num_outputs = [nout](const Node&) { return nout; };
    d.host_inputs = {1, 2, 3, 4};
    d.infer = [](InferCtx& c) {
      TFA_CHECK(!c.node.attr_b("is_training", true) || true, "");
      infer_like(c);
      for (size_t i = 1; i < c.out.size(); ++i) c.set(static_cast<int>(i), c.input(1).dtype, c.input(1).shape);
    };
    d.rows = rows_batch;
    d.compute = [](ExecCtx& c) {
      TFA_CHECK(!c.node.attr_b("is_training", true), c.node.op,
                ": only inference mode (is_training=false) is supported");
      TFA_CHECK(!nchw(c.node), c.node.op, ": only NHWC is supported");
      float eps = c.node.attr_f("epsilon", 1e-4f);
      auto host = [&](int i) {
        const TensorInfo* t = c.in_info->at(i);
        return (t->value ? *t->value : c.input(i).to(at::kCPU)).to(at::kDouble);
      };
      at::Tensor scale = host(1), offset = host(2), mean = host(3), var = host(4);
      at::Tensor s = scale * at::rsqrt(var + eps);
      at::Tensor b = offset - mean * s;
      at::Tensor x = c.input(0);
      for (size_t i = 1; i < c.out.size(); ++i) c.out[i] = c.input(std::min<int>(static_cast<int>(i) + 2, 4));
      if (!c.gpu) {
        c.out[0] = (x * s.to(x.scalar_type()) + b.to(x.scalar_type())).contiguous();
        return;
      }
      require_gpu_dtype(x, {at::kFloat, at::kDouble}, c.node.op.c_str());
      at::Tensor xc = materialize(c, x);
      at::Tensor sd = s.to(xc.scalar_type()).to(xc.device(), true);
      at::Tensor bd = b.to(xc.scalar_type()).to(xc.device(), true);
      c.out[0] = c.alloc_out(0);
      if (xc.numel())
        k::channel_affine(dt_of(xc), xc.data_ptr(), sd.data_ptr(), bd.data_ptr(), c.out[0].data_ptr(),
                          xc.numel(), xc.size(-1), 0, stream_of(c));
    };
    return d;
  };
  r.add("FusedBatchNorm", make_bn(5));
  r.add("FusedBatchNormV2", make_bn(5));
  r.add("FusedBatchNormV3", make_bn(6));

  // ---- TopKV2 (input, k) -> values, indices(int32)
  OpDef topk;
  topk.num_outputs = [](const Node&) { return 2; };
  topk.host_inputs = {1};
  topk.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto kv = c.ivalue(1);
    if (x.shape.unknown_rank) {
      c.set(0, x.dtype, Shape::unknown());
      c.set(1, DType::I32, Shape::unknown());
      return;
    }
    std::vector<int64_t> d = x.shape.dims;
    TFA_CHECK(!d.empty(), "TopKV2 needs rank >= 1");
    int64_t kk = kv ? (*kv)[0] : -1;
    TFA_CHECK(kk < 0 || d.back() < 0 || kk <= d.back(), "TopKV2: k=", kk, " > last dim ", d.back());
    d.back() = kk;
    c.set(0, x.dtype, Shape(d));
    c.set(1, DType::I32, Shape(d));
  };
  topk.rows = [](InferCtx& c) {
    c.rows_default();
    if (c.input(0).row == RowClass::ROW && c.input(0).shape.rank() >= 2 && c.input(1).row == RowClass::CONST)
      for (auto& o : c.out) o.row = RowClass::ROW;
  };
  topk.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    int64_t kk = c.host_ivalue(1)[0];
    if (!c.gpu) {
      auto res = at::topk(x, kk, -1, true, true);
      // TF breaks ties by lower index first; ATen's stable sort gives the same
      auto srt = at::sort(x, /*stable=*/true, -1, /*descending=*/true);
      c.out[0] = std::get<0>(srt).narrow(-1, 0, kk).contiguous();
      c.out[1] = std::get<1>(srt).narrow(-1, 0, kk).to(at::kInt).contiguous();
      (void)res;
      return;
    }
    require_gpu_dtype(x, {at::kFloat, at::kDouble, at::kInt, at::kLong}, "TopKV2");
    at::Tensor xc = materialize(c, x);
    c.out[0] = c.alloc_out(0);
    c.out[1] = c.alloc_out(1);
    int64_t cols = xc.size(-1);
    if (c.out[0].numel())
      k::topk(dt_of(xc), xc.data_ptr(), c.out[0].data_ptr(), c.out[1].data_ptr<int32_t>(),
              xc.numel() / cols, cols, static_cast<int>(kk), stream_of(c));
  };
  r.add("TopKV2", topk);
}

}  // namespace tfa

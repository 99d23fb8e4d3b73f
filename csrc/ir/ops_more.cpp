// More TF-1.x ops of frozen inference graphs: BroadcastTo, DepthToSpace /
// SpaceToDepth, SpaceToBatchND / BatchToSpaceND (the dilated-conv rewrite TF 1.x
// emits for atrous convolutions), Conv2DBackpropInput (tf.nn.conv2d_transpose,
// decoder / upsampling layers), L2Loss, SoftmaxCrossEntropyWithLogits and
// SparseSoftmaxCrossEntropyWithLogits (evaluation losses).
// (The reference ran whatever op a user's GraphDef held through libtensorflow;
// reference: src/main/scala/org/tensorframes/impl/TensorFlowOps.scala:76-95.)
//
// Same contract as the other op files: CPU compute through ATen (the oracle),
// GPU compute through the HIP kernels (the data movement ops are strided
// copies of permuted views, the losses compose softmax / one-hot / elementwise
// / reduction kernels); no ATen fallback on device tensors.
#include "ops_common.h"

namespace tfa {

void gpu_binary(ExecCtx& c, k::BinOp op, const at::Tensor& a0, const at::Tensor& b0);

namespace {

std::string data_format(const Node& n) { return n.attr_s("data_format", std::string("NHWC")); }

// ---------------------------------------------------------------- BroadcastTo
OpDef make_broadcast_to() {
  OpDef d;
  d.host_inputs = {1};
  d.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto sv = c.ivalue(1);
    if (!sv) {
      c.set(0, x.dtype, Shape::unknown());
      return;
    }
    std::vector<int64_t> out = *sv;
    if (!x.shape.unknown_rank) {
      TFA_CHECK(x.shape.rank() <= static_cast<int64_t>(out.size()), "BroadcastTo: input rank ", x.shape.rank(),
                " exceeds target rank ", out.size());
      const int64_t off = static_cast<int64_t>(out.size()) - x.shape.rank();
      for (int64_t i = 0; i < x.shape.rank(); ++i) {
        const int64_t d = x.shape.dims[i];
        TFA_CHECK(d < 0 || d == 1 || d == out[off + i], "BroadcastTo: dim ", i, " of size ", d,
                  " cannot broadcast to ", out[off + i]);
      }
    }
    c.set(0, x.dtype, Shape(out));
  };
  d.rows = [](InferCtx& c) {
    if (c.all_const()) {
      c.out[0].row = RowClass::CONST;
      return;
    }
    // a ROW input keeps its row dim when the target rank equals its own
    const TensorInfo& x = c.input(0);
    const bool ok = x.row == RowClass::ROW && !x.shape.unknown_rank && !c.out[0].shape.unknown_rank &&
                    x.shape.rank() == c.out[0].shape.rank() && x.shape.rank() > 0 && x.shape.dims[0] != 1;
    c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  d.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    std::vector<int64_t> shape = c.out_shape().dims;
    at::Tensor v = x.expand(shape);
    if (!c.gpu) {
      c.out[0] = v.contiguous();
      return;
    }
    c.out[0] = c.alloc_out(0);
    if (c.out[0].numel()) gpu_copy(v, c.out[0], stream_of(c));
  };
  return d;
}

// ---------------------------------------------------------------- DepthToSpace / SpaceToDepth (NHWC)
OpDef make_depth_space(bool to_space) {
  OpDef d;
  d.infer = [to_space](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    TFA_CHECK(data_format(c.node) == "NHWC", c.node.op, ": only data_format NHWC is supported");
    const int64_t b = c.node.attr_i("block_size");
    TFA_CHECK(b >= 2, c.node.op, ": block_size must be >= 2");
    if (x.shape.unknown_rank) {
      c.set(0, x.dtype, Shape({-1, -1, -1, -1}));
      return;
    }
    TFA_CHECK(x.shape.rank() == 4, c.node.op, " needs a rank-4 NHWC input");
    auto s = x.shape.dims;
    auto mul = [](int64_t v, int64_t f) { return v < 0 ? v : v * f; };
    if (to_space) {
      TFA_CHECK(s[3] < 0 || s[3] % (b * b) == 0, "DepthToSpace: depth ", s[3], " not divisible by block_size^2");
      c.set(0, x.dtype, Shape({s[0], mul(s[1], b), mul(s[2], b), s[3] < 0 ? -1 : s[3] / (b * b)}));
    } else {
      TFA_CHECK((s[1] < 0 || s[1] % b == 0) && (s[2] < 0 || s[2] % b == 0),
                "SpaceToDepth: height/width must be divisible by block_size");
      c.set(0, x.dtype, Shape({s[0], s[1] < 0 ? -1 : s[1] / b, s[2] < 0 ? -1 : s[2] / b, mul(s[3], b * b)}));
    }
  };
  d.rows = [](InferCtx& c) { c.rows_like(0); };
  d.compute = [to_space](ExecCtx& c) {
    at::Tensor x = c.gpu ? materialize(c, c.input(0)) : c.input(0).contiguous();
    const int64_t b = c.node.attr_i("block_size");
    const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
    // both directions move the same 6-d index space [N, h, by, w, bx, c]
    at::Tensor src;
    if (to_space) {
      const int64_t Co = C / (b * b);
      src = x.reshape({N, H, W, b, b, Co}).permute({0, 1, 3, 2, 4, 5});  // [N, H, by, W, bx, Co]
    } else {
      src = x.reshape({N, H / b, b, W / b, b, C}).permute({0, 1, 3, 2, 4, 5});  // [N, H/b, W/b, by, bx, C]
    }
    if (!c.gpu) {
      c.out[0] = src.contiguous().reshape(c.out_shape().dims);
      return;
    }
    c.out[0] = c.alloc_out(0);
    if (c.out[0].numel()) gpu_copy(src, c.out[0].view(src.sizes()), stream_of(c));
  };
  return d;
}

// ---------------------------------------------------------------- SpaceToBatchND / BatchToSpaceND
struct BlockGeom {
  std::vector<int64_t> block;                     // M block sizes
  std::vector<std::pair<int64_t, int64_t>> pads;  // M (before, after): paddings or crops
};

BlockGeom block_geom(const std::vector<int64_t>& bs, const std::vector<int64_t>& pv, const char* op) {
  BlockGeom g;
  g.block = bs;
  TFA_CHECK(!bs.empty() && pv.size() == 2 * bs.size(), op, ": block_shape [M] and paddings/crops [M, 2] mismatch");
  for (size_t i = 0; i < bs.size(); ++i) {
    TFA_CHECK(bs[i] >= 1, op, ": block sizes must be >= 1");
    TFA_CHECK(pv[2 * i] >= 0 && pv[2 * i + 1] >= 0, op, ": paddings/crops must be non-negative");
    g.pads.push_back({pv[2 * i], pv[2 * i + 1]});
  }
  return g;
}

OpDef make_space_to_batch() {
  OpDef d;
  d.host_inputs = {1, 2};
  d.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto bv = c.ivalue(1), pv = c.ivalue(2);
    if (x.shape.unknown_rank || !bv || !pv) {
      c.set(0, x.dtype, Shape::unknown());
      return;
    }
    BlockGeom g = block_geom(*bv, *pv, "SpaceToBatchND");
    const int64_t M = static_cast<int64_t>(g.block.size());
    TFA_CHECK(x.shape.rank() >= M + 1, "SpaceToBatchND: input rank too small for ", M, " block dims");
    std::vector<int64_t> out = x.shape.dims;
    int64_t prod = 1;
    for (int64_t i = 0; i < M; ++i) {
      prod *= g.block[i];
      int64_t& s = out[i + 1];
      if (s >= 0) {
        s += g.pads[i].first + g.pads[i].second;
        TFA_CHECK(s % g.block[i] == 0, "SpaceToBatchND: padded dim ", i + 1, " (", s, ") not divisible by ",
                  g.block[i]);
        s /= g.block[i];
      }
    }
    if (out[0] >= 0) out[0] *= prod;
    c.set(0, x.dtype, Shape(out));
  };
  d.rows = [](InferCtx& c) { c.rows_default(); };
  d.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    BlockGeom g = block_geom(c.host_ivalue(1), c.host_ivalue(2), "SpaceToBatchND");
    const int64_t M = static_cast<int64_t>(g.block.size()), R = x.dim();
    // padded input [N, P1..PM, rest...]
    std::vector<int64_t> psz = x.sizes().vec();
    for (int64_t i = 0; i < M; ++i) psz[i + 1] += g.pads[i].first + g.pads[i].second;
    // view the padded tensor as [N, P1/b1, b1, ..., PM/bM, bM, rest] and move the b's first
    std::vector<int64_t> vsz{psz[0]}, perm;
    for (int64_t i = 0; i < M; ++i) {
      vsz.push_back(psz[i + 1] / g.block[i]);
      vsz.push_back(g.block[i]);
    }
    for (int64_t i = M + 1; i < R; ++i) vsz.push_back(psz[i]);
    for (int64_t i = 0; i < M; ++i) perm.push_back(2 + 2 * i);  // b_i
    perm.push_back(0);                                          // N
    for (int64_t i = 0; i < M; ++i) perm.push_back(1 + 2 * i);  // P_i / b_i
    for (int64_t i = 2 * M + 1; i < static_cast<int64_t>(vsz.size()); ++i) perm.push_back(i);
    if (!c.gpu) {
      at::Tensor p = pool_zeros(psz, x.options());
      at::Tensor inner = p;
      for (int64_t i = 0; i < M; ++i) inner = inner.narrow(i + 1, g.pads[i].first, x.size(i + 1));
      inner.copy_(x);
      c.out[0] = p.view(vsz).permute(perm).contiguous().reshape(c.out_shape().dims);
      return;
    }
    at::Tensor p = pool_empty(psz, x.options());
    k::fill(dt_of(p), p.data_ptr(), p.numel(), 0.0, stream_of(c));
    at::Tensor inner = p;
    for (int64_t i = 0; i < M; ++i) inner = inner.narrow(i + 1, g.pads[i].first, x.size(i + 1));
    if (x.numel()) gpu_copy(x, inner, stream_of(c));
    c.out[0] = c.alloc_out(0);
    at::Tensor src = p.view(vsz).permute(perm);
    if (c.out[0].numel()) gpu_copy(src, c.out[0].view(src.sizes()), stream_of(c));
  };
  return d;
}

OpDef make_batch_to_space() {
  OpDef d;
  d.host_inputs = {1, 2};
  d.infer = [](InferCtx& c) {
    const TensorInfo& x = c.input(0);
    auto bv = c.ivalue(1), cv = c.ivalue(2);
    if (x.shape.unknown_rank || !bv || !cv) {
      c.set(0, x.dtype, Shape::unknown());
      return;
    }
    BlockGeom g = block_geom(*bv, *cv, "BatchToSpaceND");
    const int64_t M = static_cast<int64_t>(g.block.size());
    TFA_CHECK(x.shape.rank() >= M + 1, "BatchToSpaceND: input rank too small for ", M, " block dims");
    std::vector<int64_t> out = x.shape.dims;
    int64_t prod = 1;
    for (int64_t i = 0; i < M; ++i) prod *= g.block[i];
    if (out[0] >= 0) {
      TFA_CHECK(out[0] % prod == 0, "BatchToSpaceND: batch ", out[0], " not divisible by the block product ", prod);
      out[0] /= prod;
    }
    for (int64_t i = 0; i < M; ++i) {
      int64_t& s = out[i + 1];
      if (s >= 0) {
        s = s * g.block[i] - g.pads[i].first - g.pads[i].second;
        TFA_CHECK(s >= 0, "BatchToSpaceND: crops larger than the dimension");
      }
    }
    c.set(0, x.dtype, Shape(out));
  };
  d.rows = [](InferCtx& c) { c.rows_default(); };
  d.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    BlockGeom g = block_geom(c.host_ivalue(1), c.host_ivalue(2), "BatchToSpaceND");
    const int64_t M = static_cast<int64_t>(g.block.size()), R = x.dim();
    int64_t prod = 1;
    for (int64_t b : g.block) prod *= b;
    const int64_t N = x.size(0) / prod;
    // x viewed as [b1..bM, N, S1..SM, rest], moved to [N, S1, b1, ..., SM, bM, rest]
    std::vector<int64_t> vsz(g.block), perm{M};
    vsz.push_back(N);
    for (int64_t i = 1; i < R; ++i) vsz.push_back(x.size(i));
    for (int64_t i = 0; i < M; ++i) {
      perm.push_back(M + 1 + i);  // S_i
      perm.push_back(i);          // b_i
    }
    for (int64_t i = 2 * M + 1; i < static_cast<int64_t>(vsz.size()); ++i) perm.push_back(i);
    std::vector<int64_t> full{N};  // uncropped output
    for (int64_t i = 0; i < M; ++i) full.push_back(x.size(i + 1) * g.block[i]);
    for (int64_t i = M + 1; i < R; ++i) full.push_back(x.size(i));
    at::Tensor xc = c.gpu ? materialize(c, x) : x.contiguous();
    at::Tensor moved = xc.view(vsz).permute(perm);
    auto crop = [&](at::Tensor t) {
      for (int64_t i = 0; i < M; ++i)
        t = t.narrow(i + 1, g.pads[i].first, full[i + 1] - g.pads[i].first - g.pads[i].second);
      return t;
    };
    if (!c.gpu) {
      c.out[0] = crop(moved.contiguous().view(full)).contiguous();
      return;
    }
    at::Tensor tmp = pool_empty(full, x.options());
    if (tmp.numel()) gpu_copy(moved, tmp.view(moved.sizes()), stream_of(c));
    c.out[0] = c.alloc_out(0);
    if (c.out[0].numel()) gpu_copy(crop(tmp), c.out[0], stream_of(c));
  };
  return d;
}

// ---------------------------------------------------------------- Conv2DBackpropInput
// dx = conv2d_transpose(dy, W): on the GPU, dy is scattered with the forward
// stride into a zero buffer padded by (effective kernel - 1 - forward pad) and
// convolved (stride 1, the forward dilation, VALID) with W flipped in space and
// with its channel axes swapped, on the f32 MFMA implicit-GEMM conv kernel.
struct TransposedGeom {
  int64_t N, H, W, IC, OH, OW, OC, KH, KW, sh, sw, dh, dw, pt, pl;
};

TransposedGeom transposed_geom(const Node& n, const std::vector<int64_t>& in_sizes, const std::vector<int64_t>& w,
                               const std::vector<int64_t>& dy) {
  TFA_CHECK(data_format(n) == "NHWC", n.op, ": only data_format NHWC is supported");
  TFA_CHECK(in_sizes.size() == 4 && w.size() == 4 && dy.size() == 4, n.op, ": rank-4 sizes/filter/out_backprop");
  auto st = n.attr_ilist("strides", {1, 1, 1, 1});
  auto dl = n.attr_ilist("dilations", {1, 1, 1, 1});
  TFA_CHECK(st.size() == 4 && st[0] == 1 && st[3] == 1, n.op, ": strides must be [1,sh,sw,1]");
  std::string pad = n.attr_s("padding");
  TFA_CHECK(pad == "SAME" || pad == "VALID", n.op, ": unsupported padding '", pad, "'");
  TransposedGeom g;
  g.N = in_sizes[0]; g.H = in_sizes[1]; g.W = in_sizes[2]; g.IC = in_sizes[3];
  g.KH = w[0]; g.KW = w[1]; g.OC = w[3];
  TFA_CHECK(w[2] == g.IC, n.op, ": filter in-channels ", w[2], " != input_sizes channels ", g.IC);
  g.sh = st[1]; g.sw = st[2];
  g.dh = dl.size() == 4 ? dl[1] : 1; g.dw = dl.size() == 4 ? dl[2] : 1;
  auto fwd = [&](int64_t in, int64_t k, int64_t s, int64_t d, int64_t& out, int64_t& pb) {
    const int64_t eff = (k - 1) * d + 1;
    if (pad == "SAME") {
      out = (in + s - 1) / s;
      pb = std::max<int64_t>((out - 1) * s + eff - in, 0) / 2;
    } else {
      out = in >= eff ? (in - eff) / s + 1 : 0;
      pb = 0;
    }
  };
  fwd(g.H, g.KH, g.sh, g.dh, g.OH, g.pt);
  fwd(g.W, g.KW, g.sw, g.dw, g.OW, g.pl);
  TFA_CHECK(dy[1] == g.OH && dy[2] == g.OW && dy[3] == g.OC && (dy[0] == g.N || dy[0] < 0), n.op,
            ": out_backprop shape [", dy[0], ",", dy[1], ",", dy[2], ",", dy[3], "] does not match the forward conv of ",
            "input_sizes (expected spatial ", g.OH, "x", g.OW, ", channels ", g.OC, ")");
  return g;
}

OpDef make_conv2d_backprop_input() {
  OpDef d;
  d.host_inputs = {0};
  d.infer = [](InferCtx& c) {
    auto sv = c.ivalue(0);
    const TensorInfo& dy = c.input(2);
    TFA_CHECK(dy.dtype == c.input(1).dtype, "Conv2DBackpropInput: filter/out_backprop dtype mismatch");
    if (!sv) {
      c.set(0, dy.dtype, Shape({-1, -1, -1, -1}));
      return;
    }
    TFA_CHECK(sv->size() == 4, "Conv2DBackpropInput: input_sizes must have 4 values");
    std::vector<int64_t> out = *sv;
    // the batch follows out_backprop (input_sizes often carries the traced batch)
    if (!dy.shape.unknown_rank && dy.shape.rank() == 4) out[0] = dy.shape.dims[0];
    c.set(0, dy.dtype, Shape(out));
  };
  d.rows = [](InferCtx& c) {
    if (c.all_const()) { c.out[0].row = RowClass::CONST; return; }
    const bool ok = c.input(2).row == RowClass::ROW && c.input(1).row == RowClass::CONST;
    c.out[0].row = ok ? RowClass::ROW : RowClass::MIXED;
  };
  d.compute = [](ExecCtx& c) {
    at::Tensor w = c.input(1), dy = c.input(2);
    std::vector<int64_t> sizes = c.host_ivalue(0);
    sizes[0] = dy.size(0);
    TransposedGeom g = transposed_geom(c.node, sizes, w.sizes().vec(), dy.sizes().vec());
    const int64_t ekh = (g.KH - 1) * g.dh + 1, ekw = (g.KW - 1) * g.dw + 1;
    if (!c.gpu) {  // oracle: ATen's transposed conv, then TF's asymmetric crop
      at::Tensor y = at::conv_transpose2d(dy.permute({0, 3, 1, 2}), w.permute({3, 2, 0, 1}), {}, {g.sh, g.sw},
                                          {0, 0}, {0, 0}, 1, {g.dh, g.dw});
      // positions past the last window (VALID / stride remainders) receive nothing
      const int64_t lack_h = std::max<int64_t>(g.pt + g.H - y.size(2), 0);
      const int64_t lack_w = std::max<int64_t>(g.pl + g.W - y.size(3), 0);
      if (lack_h || lack_w) y = at::constant_pad_nd(y, {0, lack_w, 0, lack_h}, 0);
      y = y.narrow(2, g.pt, g.H).narrow(3, g.pl, g.W);
      c.out[0] = y.permute({0, 2, 3, 1}).contiguous();
      return;
    }
    require_gpu_dtype(dy, {at::kFloat}, "Conv2DBackpropInput");
    hipStream_t s = stream_of(c);
    c.out[0] = c.alloc_out(0);
    if (!c.out[0].numel()) return;
    // zero buffer [N, H + ekh - 1, W + ekw - 1, OC] with dy scattered at stride (sh, sw)
    const int64_t PH = g.H + ekh - 1, PW = g.W + ekw - 1;
    at::Tensor buf = pool_empty({g.N, PH, PW, g.OC}, dy.options());
    k::fill(DType::F32, buf.data_ptr(), buf.numel(), 0.0, s);
    const int64_t top = ekh - 1 - g.pt, left = ekw - 1 - g.pl;
    if (dy.numel()) {
      at::Tensor dst = buf.slice(1, top, top + (g.OH - 1) * g.sh + 1, g.sh)
                           .slice(2, left, left + (g.OW - 1) * g.sw + 1, g.sw);
      gpu_copy(dy, dst, s);
    }
    // W'[kh][kw][oc][ic] = W[KH-1-kh][KW-1-kw][ic][oc] (negative source strides)
    at::Tensor wc = materialize(c, w);
    at::Tensor wf = pool_empty({g.KH, g.KW, g.OC, g.IC}, wc.options());
    {
      const int64_t dims[4] = {g.KH, g.KW, g.OC, g.IC};
      const int64_t sst[4] = {-g.KW * g.IC * g.OC, -g.IC * g.OC, 1, g.OC};
      const int64_t dst_st[4] = {g.KW * g.OC * g.IC, g.OC * g.IC, g.IC, 1};
      const float* src0 = wc.data_ptr<float>() + ((g.KH - 1) * g.KW + (g.KW - 1)) * g.IC * g.OC;
      k::strided_copy(4, 4, dims, src0, sst, wf.data_ptr(), dst_st, s);
    }
    k::ConvArgs a;
    a.N = g.N; a.H = PH; a.W = PW; a.C = g.OC;
    a.KH = g.KH; a.KW = g.KW; a.OC = g.IC; a.OH = g.H; a.OW = g.W;
    a.sh = a.sw = 1; a.dh = g.dh; a.dw = g.dw; a.pad_t = a.pad_l = 0;
    a.x = buf.data_ptr(); a.w = wf.data_ptr(); a.y = c.out[0].data_ptr();
    a.bias = nullptr; a.act = 0;
    at::Tensor work;
    if (size_t ws = k::conv2d_workspace_bytes(DType::F32, a)) {
      work = pool_empty({static_cast<int64_t>(ws)}, buf.options().dtype(at::kByte));
      a.workspace = work.data_ptr();
    }
    k::conv2d_nhwc(DType::F32, a, s);
  };
  return d;
}

// ---------------------------------------------------------------- L2Loss
OpDef make_l2loss() {
  OpDef d;
  d.infer = [](InferCtx& c) { c.set(0, c.input(0).dtype, Shape(std::vector<int64_t>{})); };
  d.rows = [](InferCtx& c) { c.rows_default(); };
  d.compute = [](ExecCtx& c) {
    at::Tensor x = c.input(0);
    if (!c.gpu) {
      c.out[0] = (x * x).sum().mul(0.5).to(x.scalar_type());
      return;
    }
    require_gpu_dtype(x, {at::kFloat, at::kDouble}, "L2Loss");
    at::Tensor xc = materialize(c, x);
    const DType dt = dt_of(xc);
    c.out[0] = c.alloc_out(0);
    at::Tensor sq = pool_empty_like(xc);
    at::Tensor half = pool_empty({}, xc.options());
    k::fill(dt, half.data_ptr(), 1, 0.5, stream_of(c));
    if (xc.numel() == 0) {
      k::fill(dt, c.out[0].data_ptr(), 1, 0.0, stream_of(c));
      return;
    }
    k::unary(k::UnOp::SQUARE, dt, xc.data_ptr(), sq.data_ptr(), xc.numel(), stream_of(c));
    at::Tensor s = pool_empty({}, xc.options());
    size_t ws = k::reduce_workspace_bytes(dt, 1, xc.numel(), 1);
    at::Tensor work;
    if (ws) work = pool_empty({static_cast<int64_t>(ws)}, xc.options().dtype(at::kByte));
    k::reduce(k::RedOp::SUM, dt, sq.data_ptr(), s.data_ptr(), 1, xc.numel(), 1, ws ? work.data_ptr() : nullptr,
              stream_of(c));
    k::binary(k::BinOp::MUL, dt, s.data_ptr(), half.data_ptr(), c.out[0].data_ptr(), 1, 1, 1, nullptr,
              stream_of(c));
  };
  return d;
}

// ---------------------------------------------------------------- softmax cross-entropy
// loss[b] = -sum_c labels[b,c] * log_softmax(features)[b,c]; backprop = softmax - labels
void xent_gpu(ExecCtx& c, const at::Tensor& feat, const at::Tensor& labels_dense) {
  const DType dt = dt_of(feat);
  const int64_t B = feat.size(0), C = feat.size(1);
  hipStream_t s = stream_of(c);
  c.out[0] = c.alloc_out(0);
  c.out[1] = c.alloc_out(1);
  if (B == 0) return;
  at::Tensor lsm = pool_empty_like(feat);
  k::softmax(dt, true, feat.data_ptr(), lsm.data_ptr(), B, C, s);
  at::Tensor prod = pool_empty_like(feat);
  k::binary(k::BinOp::MUL, dt, labels_dense.data_ptr(), lsm.data_ptr(), prod.data_ptr(), B * C, 0, 1, nullptr, s);
  at::Tensor neg = pool_empty({B}, feat.options());
  size_t ws = k::reduce_workspace_bytes(dt, B, C, 1);
  at::Tensor work;
  if (ws) work = pool_empty({static_cast<int64_t>(ws)}, feat.options().dtype(at::kByte));
  k::reduce(k::RedOp::SUM, dt, prod.data_ptr(), neg.data_ptr(), B, C, 1, ws ? work.data_ptr() : nullptr, s);
  k::unary(k::UnOp::NEG, dt, neg.data_ptr(), c.out[0].data_ptr(), B, s);
  at::Tensor sm = pool_empty_like(feat);
  k::softmax(dt, false, feat.data_ptr(), sm.data_ptr(), B, C, s);
  k::binary(k::BinOp::SUB, dt, sm.data_ptr(), labels_dense.data_ptr(), c.out[1].data_ptr(), B * C, 0, 1, nullptr, s);
}

OpDef make_xent(bool sparse) {
  OpDef d;
  d.num_outputs = [](const Node&) { return 2; };
  d.infer = [sparse](InferCtx& c) {
    const TensorInfo& f = c.input(0);
    const TensorInfo& l = c.input(1);
    if (sparse)
      TFA_CHECK(l.dtype == DType::I32 || l.dtype == DType::I64, c.node.op, ": labels must be int32/int64");
    else
      TFA_CHECK(l.dtype == f.dtype, c.node.op, ": features and labels dtypes differ");
    int64_t B = -1, C = -1;
    if (!f.shape.unknown_rank) {
      TFA_CHECK(f.shape.rank() == 2, c.node.op, ": features must be [batch, classes]");
      B = f.shape.dims[0];
      C = f.shape.dims[1];
    }
    if (!l.shape.unknown_rank) {
      TFA_CHECK(l.shape.rank() == (sparse ? 1 : 2), c.node.op, ": labels rank ", l.shape.rank());
      if (B < 0) B = l.shape.dims[0];
      TFA_CHECK(l.shape.dims[0] < 0 || B < 0 || l.shape.dims[0] == B, c.node.op, ": batch sizes differ");
      if (!sparse) {
        TFA_CHECK(l.shape.dims[1] < 0 || C < 0 || l.shape.dims[1] == C, c.node.op, ": class counts differ");
        if (C < 0) C = l.shape.dims[1];
      }
    }
    c.set(0, f.dtype, Shape({B}));
    c.set(1, f.dtype, Shape({B, C}));
  };
  d.rows = [](InferCtx& c) {  // one loss / gradient row per input row
    RowClass r = RowClass::MIXED;
    if (c.all_const()) r = RowClass::CONST;
    else if (c.input(0).row == RowClass::ROW && c.input(1).row == RowClass::ROW) r = RowClass::ROW;
    for (auto& o : c.out) o.row = r;
  };
  d.compute = [sparse](ExecCtx& c) {
    at::Tensor f = c.input(0), l = c.input(1);
    if (!c.gpu) {
      at::Tensor dense = sparse ? at::one_hot(l.to(at::kLong), f.size(1)).to(f.scalar_type()) : l;
      at::Tensor lsm = at::log_softmax(f, 1);
      c.out[0] = (-(dense * lsm).sum(1)).contiguous();
      c.out[1] = (at::softmax(f, 1) - dense).contiguous();
      return;
    }
    require_gpu_dtype(f, {at::kFloat, at::kDouble}, c.node.op.c_str());
    at::Tensor fc = materialize(c, f);
    at::Tensor dense;
    if (sparse) {
      at::Tensor lc = materialize(c, l);
      dense = pool_empty_like(fc);
      if (fc.numel())
        k::one_hot(dt_of(fc), dt_of(lc), lc.data_ptr(), dense.data_ptr(), fc.size(0), fc.size(1), 1.0, 0.0,
                   stream_of(c));
    } else {
      dense = materialize(c, l);
    }
    xent_gpu(c, fc, dense);
  };
  return d;
}

}  // namespace

void register_more_ops(OpRegistry& r) {
  r.add("BroadcastTo", make_broadcast_to());
  r.add("DepthToSpace", make_depth_space(true));
  r.add("SpaceToDepth", make_depth_space(false));
  r.add("SpaceToBatchND", make_space_to_batch());
  r.add("BatchToSpaceND", make_batch_to_space());
  r.add("Conv2DBackpropInput", make_conv2d_backprop_input());
  r.add("L2Loss", make_l2loss());
  r.add("SoftmaxCrossEntropyWithLogits", make_xent(false));
  r.add("SparseSoftmaxCrossEntropyWithLogits", make_xent(true));
}

}  // namespace tfa

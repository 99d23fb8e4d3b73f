// Helpers shared by the op registrations (ops_array.cpp, ops_math.cpp, ops_nn.cpp).
//
// Every op has one compute function that runs on CPU tensors through ATen
// (the oracle / constant-folding path) and on device tensors through the
// tensorframes_amd HIP kernels (kernels/kernels.h). There is no ATen fallback
// on the device path: an unsupported device case raises.
#pragma once

#include <ATen/ATen.h>
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../kernels/kernels.h"
#include "../runtime/device_pool.h"
#include "graph.h"

namespace tfa {

inline hipStream_t stream_of(const ExecCtx& c) { return static_cast<hipStream_t>(c.stream); }

// one op of an elementwise chain absorbed into a GEMM/conv epilogue (the
// planner's match; k::EpiCode / k::EpiOperand): `t` holds the tensor operand
// (per-column [N], per-row [M,1], full, or a 1-element runtime scalar)
struct EpiStep {
  int code = k::EPI_ADD, kind = k::EPO_NONE, act = k::ACT_NONE;
  double s = 0;
  at::Tensor t;
};

// fills the kernel-side program (device pointers of contiguous operands)
inline k::EpiProg epi_prog(const std::vector<EpiStep>* epi) {
  k::EpiProg p;
  if (!epi) return p;
  TFA_CHECK(static_cast<int>(epi->size()) <= k::kMaxEpi, "epilogue chain too long");
  for (const EpiStep& e : *epi) {
    k::EpiOp& o = p.op[p.n++];
    o.code = e.code;
    o.kind = e.kind;
    o.act = e.act;
    o.s = e.s;
    if (e.t.defined()) {
      TFA_CHECK(e.t.is_contiguous(), "epilogue operand must be contiguous");
      o.p = e.t.data_ptr();
    }
  }
  return p;
}

inline at::Tensor apply_act_host(const at::Tensor& r, int act);

// host (ATen) form of the chain over a result r (2-D view [rows, N])
inline at::Tensor apply_epi_host(at::Tensor r, const std::vector<EpiStep>* epi) {
  if (!epi) return r;
  const int64_t N = r.size(-1);
  for (const EpiStep& e : *epi) {
    at::Tensor x;
    switch (e.kind) {
      case k::EPO_SCALAR: x = at::scalar_tensor(e.s, r.options()); break;
      case k::EPO_SCALAR_PTR: x = e.t.reshape({}); break;
      case k::EPO_COL: x = e.t.reshape({N}); break;
      case k::EPO_ROW: x = e.t.reshape({r.numel() / N, 1}); break;
      case k::EPO_FULL: x = e.t.reshape(r.sizes()); break;
      default: break;
    }
    switch (e.code) {
      case k::EPI_ADD: r = r + x; break;
      case k::EPI_SUB: r = r - x; break;
      case k::EPI_RSUB: r = x - r; break;
      case k::EPI_MUL: r = r * x; break;
      case k::EPI_DIV: r = r / x; break;
      case k::EPI_RDIV: r = x / r; break;
      case k::EPI_MAX: r = at::maximum(r, x.expand_as(r)); break;
      case k::EPI_MIN: r = at::minimum(r, x.expand_as(r)); break;
      case k::EPI_ACT: r = apply_act_host(r, e.act); break;
      case k::EPI_NEG: r = -r; break;
      case k::EPI_SQUARE: r = r * r; break;
      case k::EPI_ABS: r = at::abs(r); break;
      default: break;
    }
  }
  return r;
}

// MatMul / Conv2D with a fused epilogue (bias [N], activation, absorbed chain);
// shared by the ops and the planner's fused steps
void run_gemm(ExecCtx& c, const at::Tensor& a0, const at::Tensor& b0, bool ta, bool tb,
              const at::Tensor* bias, int act, at::Tensor& out, const std::vector<EpiStep>* epi = nullptr);
// sibling convs fused along OC (GPU): w0 = the members' filters concatenated
// along OC, outs[k] = member k's output (NHWC, possibly a channel slice)
// wino: the planner's Winograd F(2x2,3x3) filter of w0 (conv_wino_filter), or null
void run_conv2d_siblings(ExecCtx& c, const at::Tensor& x0, const at::Tensor& w0, const at::Tensor* bias, int act,
                         std::vector<at::Tensor>& outs, const std::vector<int>& acts,
                         const at::Tensor* wino = nullptr);
// pool2: `out` is the 2x2 / stride-2 VALID max pool of the conv's activated
// output (planner-fused); the Winograd epilogue pools its own output tiles,
// any other kernel path runs the conv into a temporary and the pool after it
// pool_in (planner-fused MaxPool -> 1x1 conv): x0 is the pool's input and
// pool_in = {kh, kw, sh, sw} its VALID window; the conv reads the pooled values
// without the pooled tensor reaching HBM (kernels/conv_smallc.hip), or, where
// that kernel does not apply, pools into a temporary first
void run_conv2d(ExecCtx& c, const at::Tensor& x0, const at::Tensor& w0, const at::Tensor* bias,
                int act, at::Tensor& out, const std::vector<EpiStep>* epi = nullptr,
                const at::Tensor* wino = nullptr, bool pool2 = false, const int* pool_in = nullptr);
// MaxPool/AvgPool with a fused bias + activation, into `out` (GPU; `out` may
// be a channel slice of a concat output)
void run_pool_fused(ExecCtx& c, bool is_max, const at::Tensor& x0, const at::Tensor* bias, int act,
                    const at::Tensor& out);

// host (ATen) form of a fused epilogue activation (k::Act codes); same
// formulas as the standalone ops
inline at::Tensor apply_act_host(const at::Tensor& r, int act) {
  switch (act) {
    case k::ACT_RELU: return at::clamp_min(r, 0);
    case k::ACT_RELU6: return at::clamp(r, 0, 6);
    case k::ACT_SIGMOID: return at::sigmoid(r);
    case k::ACT_TANH: return at::tanh(r);
    case k::ACT_ELU: return at::where(r > 0, r, at::expm1(r));
    case k::ACT_SELU: return at::selu(r);
    case k::ACT_SOFTPLUS: return at::where(r > 20, r, at::log1p(at::exp(r)));
    default: return r;
  }
}
inline DType dt_of(const at::Tensor& t) { return from_scalar_type(t.scalar_type()); }

inline int64_t norm_axis(int64_t a, int64_t rank, const char* what = "axis") {
  int64_t r = a < 0 ? a + rank : a;
  TFA_CHECK(r >= 0 && r < std::max<int64_t>(rank, 1), what, " ", a, " out of range for rank ", rank);
  return r;
}

// Copy an arbitrarily strided device view into another (same sizes). Device only.
void gpu_copy(const at::Tensor& src, const at::Tensor& dst, hipStream_t s);
// Contiguous copy of a (view) tensor on its device (ATen on CPU, our kernel on GPU).
at::Tensor materialize(const ExecCtx& c, const at::Tensor& view);
// Device-side broadcast descriptor for operands already expanded to `out` sizes.
k::Bcast make_bcast(const std::vector<int64_t>& out, const at::Tensor& a, const at::Tensor& b,
                    const at::Tensor* c = nullptr);

inline void require_gpu_dtype(const at::Tensor& t, std::initializer_list<at::ScalarType> ok,
                              const char* op) {
  for (auto s : ok)
    if (t.scalar_type() == s) return;
  TFA_CHECK(false, op, ": dtype ", c10::toString(t.scalar_type()), " is not supported on the GPU path");
}

// Common infer: same dtype/shape as input i.
inline void infer_like(InferCtx& c, int i = 0) {
  c.set(0, c.input(i).dtype, c.input(i).shape);
}

}  // namespace tfa

// Device-side helpers shared by the tensorframes_amd HIP kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <type_traits>
#include <utility>

#include "kernels.h"

namespace tfa {
namespace k {

constexpr int kWave = 64;  // CDNA wavefront

// Memory-bound grid sizing: enough blocks to fill 256 CUs several times over,
// grid-stride for the rest.
inline int ew_grid(int64_t work_items, int block = 256, int max_blocks = 256 * 8) {
  int64_t b = (work_items + block - 1) / block;
  if (b < 1) b = 1;
  if (b > max_blocks) b = max_blocks;
  return static_cast<int>(b);
}

// Division by a launch-constant divisor without the integer-divide sequence
// (a 64-bit `%`/`/` is ~100 VALU instructions on CDNA; an implicit-GEMM conv
// decomposes every output-row index into (n, oh, ow)). Round-up magic number:
// n / d == (umulhi(n, m) + n) >> s for every 32-bit n, d in [1, 2^31)
// (checked exhaustively on edge cases in tests/test_fastdiv.py).
struct FastDivU32 {
  uint32_t d = 1, m = 1, s = 0;
};
inline FastDivU32 make_fastdiv(uint32_t d) {
  FastDivU32 f;
  f.d = d;
  f.s = 0;
  while ((uint64_t(1) << f.s) < d) ++f.s;
  f.m = static_cast<uint32_t>(((uint64_t(1) << 32) * ((uint64_t(1) << f.s) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDivU32& f) {
  const uint32_t hi = __umulhi(n, f.m);
  return static_cast<uint32_t>((static_cast<uint64_t>(hi) + n) >> f.s);
}

// the cheap epilogue activations (none / relu / relu6): kernels branch once
// on `act` between an epilogue built from this and one built from act_apply,
// so the transcendental forms do not bloat the common hot epilogue
template <typename T>
__device__ __forceinline__ T act_fast(T v, int act) {
  if (act == ACT_RELU) return v > T(0) ? v : T(0);
  if (act == ACT_RELU6) return v > T(0) ? (v < T(6) ? v : T(6)) : T(0);
  return v;
}

// epilogue activation (codes: enum Act in kernels.h); `act` is uniform per
// launch, so the switch is a scalar branch
template <typename T>
__device__ __forceinline__ T act_apply(T v, int act) {
  switch (act) {
    case ACT_RELU: return v > T(0) ? v : T(0);
    case ACT_RELU6: return v > T(0) ? (v < T(6) ? v : T(6)) : T(0);
    case ACT_SIGMOID: return T(1) / (T(1) + exp(-v));
    case ACT_TANH: return tanh(v);
    case ACT_ELU: return v > T(0) ? v : expm1(v);
    case ACT_SELU: {
      const T alpha = T(1.6732632423543772848170429916717), scale = T(1.0507009873554804934193349852946);
      return v > T(0) ? scale * v : scale * alpha * expm1(v);
    }
    case ACT_SOFTPLUS: return v > T(20) ? v : log1p(exp(v));
    default: return v;
  }
}

// f(std::integral_constant<int, I>) for I = 0..N-1, expanded at compile time.
// Accumulator tiles must be indexed with constants: one loop the unroller gives
// up on (a big epilogue body) demotes the whole accumulator array to scratch,
// and the k loop then stores every accumulator to scratch once per k tile.
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// the absorbed elementwise chain of a GEMM/conv epilogue at output (row, col)
// of batch offset `boff` (elements); operands are contiguous [.., M, N]
template <typename T>
__device__ __forceinline__ T epi_apply(const EpiProg& e, T v, int64_t row, int64_t col, int64_t N, int64_t boff) {
  for (int k = 0; k < e.n; ++k) {
    const EpiOp& o = e.op[k];
    const T* p = static_cast<const T*>(o.p);
    T x = T(0);
    switch (o.kind) {
      case EPO_SCALAR: x = T(o.s); break;
      case EPO_SCALAR_PTR: x = p[0]; break;
      case EPO_COL: x = p[col]; break;
      case EPO_ROW: x = p[row]; break;
      case EPO_FULL: x = p[boff + row * N + col]; break;
      default: break;
    }
    switch (o.code) {
      case EPI_ADD: v = v + x; break;
      case EPI_SUB: v = v - x; break;
      case EPI_RSUB: v = x - v; break;
      case EPI_MUL: v = v * x; break;
      case EPI_DIV: v = v / x; break;
      case EPI_RDIV: v = x / v; break;
      // NaN-propagating, like the unfused Maximum/Minimum kernels
      case EPI_MAX: v = (v != v || x != x) ? v + x : (v > x ? v : x); break;
      case EPI_MIN: v = (v != v || x != x) ? v + x : (v < x ? v : x); break;
      case EPI_ACT: v = act_apply(v, o.act); break;
      case EPI_NEG: v = -v; break;
      case EPI_SQUARE: v = v * v; break;
      case EPI_ABS: v = v < T(0) ? -v : v; break;
      default: break;
    }
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Broadcast index math: linear output index -> operand offset.
__device__ __forceinline__ int64_t bcast_offset(int64_t i, int rank, const int64_t* dims,
                                                const int64_t* strides) {
  int64_t off = 0;
  for (int d = rank - 1; d >= 0; --d) {
    int64_t q = i / dims[d];
    int64_t r = i - q * dims[d];
    off += r * strides[d];
    i = q;
  }
  return off;
}

}  // namespace k
}  // namespace tfa

#define TFA_LAUNCH_CHECK(what)                                                        \
  do {                                                                                \
    hipError_t _e = hipGetLastError();                                                \
    if (_e != hipSuccess) {                                                           \
      throw ::tfa::GraphError(::tfa::str_cat("HIP launch of ", what, " failed: ",     \
                                             hipGetErrorString(_e)));                 \
    }                                                                                 \
  } while (0)

// Kernels of the wider TF op set: padding (constant / reflect / symmetric),
// cumulative scans, LeakyRelu, depthwise convolution, local response
// normalisation, GatherNd and Where (coordinates of true elements).
//
// All grid-stride over <= 2048 blocks of 256 threads; scans along the last
// axis use one block per row with wave-level (64-lane) prefix sums.
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

template <typename E>
__global__ __launch_bounds__(256) void pad_kernel(const E* __restrict__ x, E* __restrict__ y, int64_t n,
                                                  PadArgs a, E cval) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t rem = i, src = 0;
    bool inside = true;
    for (int d = a.rank - 1; d >= 0; --d) {
      const int64_t od = rem % a.out_dims[d];
      rem /= a.out_dims[d];
      int64_t s = od - a.before[d];
      const int64_t len = a.in_dims[d];
      if (s < 0 || s >= len) {
        if (a.mode == 0) {
          inside = false;
        } else if (a.mode == 1) {  // REFLECT: edge not repeated
          s = s < 0 ? -s : 2 * (len - 1) - s;
        } else {  // SYMMETRIC: edge repeated
          s = s < 0 ? -s - 1 : 2 * len - 1 - s;
        }
      }
      src += s * a.in_strides[d];
    }
    y[i] = inside ? x[src] : cval;
  }
}

// ---- scans
template <typename T>
__device__ __forceinline__ T scan_op(T a, T b, bool prod) { return prod ? a * b : a + b; }

template <typename T>
__device__ __forceinline__ T wave_inclusive(T v, int lane, bool prod) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T u = __shfl_up(v, o, 64);
    if (lane >= o) v = scan_op(v, u, prod);
  }
  return v;
}

// one block per row of [rows, n] (inner == 1), chunks of 256 elements carried across
template <typename T>
__global__ __launch_bounds__(256) void scan_rows(const T* __restrict__ x, T* __restrict__ y, int64_t rows,
                                                 int64_t n, bool prod, bool exclusive, bool reverse) {
  __shared__ T wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T ident = prod ? T(1) : T(0);
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const T* xr = x + r * n;
    T* yr = y + r * n;
    T carry = ident;
    for (int64_t base = 0; base < n; base += 256) {
      const int64_t j = base + tid;
      const int64_t src = reverse ? n - 1 - j : j;
      T v = j < n ? xr[src] : ident;
      T inc = wave_inclusive(v, lane, prod);
      T exc_w = __shfl_up(inc, 1, 64);  // exclusive within the wave
      if (lane == 0) exc_w = ident;
      if (lane == 63) wsum[wave] = inc;
      __syncthreads();
      T wpre = ident;
      for (int w = 0; w < wave; ++w) wpre = scan_op(wpre, wsum[w], prod);
      T total = ident;
      for (int w = 0; w < 4; ++w) total = scan_op(total, wsum[w], prod);
      const T pre = scan_op(carry, wpre, prod);
      if (j < n) yr[src] = exclusive ? scan_op(pre, exc_w, prod) : scan_op(pre, inc, prod);
      carry = scan_op(carry, total, prod);
      __syncthreads();
    }
  }
}

// general [outer, n, inner]: one thread per (outer, inner) line
template <typename T>
__global__ __launch_bounds__(256) void scan_lines(const T* __restrict__ x, T* __restrict__ y, int64_t outer,
                                                  int64_t n, int64_t inner, bool prod, bool exclusive,
                                                  bool reverse) {
  const int64_t lines = outer * inner;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < lines; l += stride) {
    const int64_t o = l / inner, in = l % inner;
    T acc = prod ? T(1) : T(0);
    for (int64_t t = 0; t < n; ++t) {
      const int64_t j = reverse ? n - 1 - t : t;
      const int64_t idx = (o * n + j) * inner + in;
      const T v = x[idx];
      if (exclusive) {
        y[idx] = acc;
        acc = scan_op(acc, v, prod);
      } else {
        acc = scan_op(acc, v, prod);
        y[idx] = acc;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void leaky_relu_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                         T alpha) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const T v = x[i];
    y[i] = v >= T(0) ? v : v * alpha;
  }
}

// depthwise NHWC: y[n,oh,ow,c*M+m] = sum_{kh,kw} x[n,ih,iw,c] * w[kh,kw,c,m]
__global__ __launch_bounds__(256) void depthwise_kernel(DepthwiseArgs a, int64_t total) {
  const float* x = static_cast<const float*>(a.x);
  const float* w = static_cast<const float*>(a.w);
  float* y = static_cast<float*>(a.y);
  const int64_t OC = a.C * a.M;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t oc = i % OC;
    int64_t t = i / OC;
    const int64_t ow = t % a.OW;
    t /= a.OW;
    const int64_t oh = t % a.OH;
    const int64_t nn = t / a.OH;
    const int64_t c = oc / a.M, m = oc % a.M;
    float acc = 0.f;
    for (int64_t kh = 0; kh < a.KH; ++kh) {
      const int64_t ih = oh * a.sh - a.pad_t + kh * a.dh;
      if (ih < 0 || ih >= a.H) continue;
      for (int64_t kw = 0; kw < a.KW; ++kw) {
        const int64_t iw = ow * a.sw - a.pad_l + kw * a.dw;
        if (iw < 0 || iw >= a.W) continue;
        acc = fmaf(x[((nn * a.H + ih) * a.W + iw) * a.C + c], w[((kh * a.KW + kw) * a.C + c) * a.M + m], acc);
      }
    }
    y[i] = acc;
  }
}

// LRN over the channel (last) dim
template <typename T>
__global__ __launch_bounds__(256) void lrn_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, int64_t C,
                                                  int radius, float bias, float alpha, float beta) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t c = i % C;
    const int64_t row = i - c;
    const int64_t lo = c - radius < 0 ? 0 : c - radius, hi = c + radius >= C ? C - 1 : c + radius;
    double sq = 0.0;
    for (int64_t j = lo; j <= hi; ++j) {
      const double v = (double)x[row + j];
      sq += v * v;
    }
    y[i] = (T)((double)x[i] / pow((double)bias + (double)alpha * sq, (double)beta));
  }
}

template <typename E, typename I>
__global__ __launch_bounds__(256) void gather_nd_kernel(const E* __restrict__ p, const I* __restrict__ idx,
                                                        E* __restrict__ out, int64_t nidx, int64_t inner,
                                                        GatherNdArgs a) {
  const int64_t total = nidx * inner;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t r = i / inner, in = i % inner;
    int64_t off = 0;
    bool ok = true;
    for (int d = 0; d < a.K; ++d) {
      const int64_t v = (int64_t)idx[r * a.K + d];
      ok = ok && v >= 0 && v < a.dims[d];
      off += v * a.strides[d];
    }
    out[i] = ok ? p[off * inner + in] : E{};
  }
}

// Where: coordinates of nonzero elements, row-major order, from an inclusive
// int64 scan of the mask
__global__ __launch_bounds__(256) void where_kernel(const uint8_t* __restrict__ mask, const int64_t* __restrict__ pos,
                                                    int64_t* __restrict__ out, int64_t n, WhereArgs a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (!mask[i]) continue;
    const int64_t row = pos[i] - 1;
    int64_t rem = i;
    for (int d = a.rank - 1; d >= 0; --d) {
      out[row * a.rank + d] = rem % a.dims[d];
      rem /= a.dims[d];
    }
  }
}

__global__ __launch_bounds__(256) void mask_to_i64(const uint8_t* __restrict__ m, int64_t* __restrict__ o, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) o[i] = m[i] ? 1 : 0;
}

template <typename T>
void scan_t(bool prod, const void* x, void* y, int64_t outer, int64_t n, int64_t inner, bool exclusive,
            bool reverse, hipStream_t s) {
  if (inner == 1) {
    const int blocks = (int)std::min<int64_t>(outer, 4096);
    hipLaunchKernelGGL((scan_rows<T>), dim3(blocks), dim3(256), 0, s, (const T*)x, (T*)y, outer, n, prod, exclusive,
                       reverse);
  } else {
    hipLaunchKernelGGL((scan_lines<T>), dim3(ew_grid(outer * inner)), dim3(256), 0, s, (const T*)x, (T*)y, outer, n,
                       inner, prod, exclusive, reverse);
  }
}

}  // namespace

void pad_nd(int64_t elem_size, const PadArgs& a, const void* x, void* y, uint64_t cbits, hipStream_t s) {
  TFA_CHECK(a.rank >= 1 && a.rank <= kMaxRank, "pad: bad rank ", a.rank);
  int64_t n = 1;
  for (int d = 0; d < a.rank; ++d) {
    n *= a.out_dims[d];
    if (a.mode != 0)
      TFA_CHECK(a.before[d] <= a.in_dims[d] - (a.mode == 1 ? 1 : 0) &&
                    a.out_dims[d] - a.in_dims[d] - a.before[d] <= a.in_dims[d] - (a.mode == 1 ? 1 : 0),
                "MirrorPad: paddings must not exceed the dimension size");
  }
  if (n <= 0) return;
  const dim3 g(ew_grid(n)), b(256);
  switch (elem_size) {
    case 1: hipLaunchKernelGGL((pad_kernel<uint8_t>), g, b, 0, s, (const uint8_t*)x, (uint8_t*)y, n, a, (uint8_t)cbits); break;
    case 2: hipLaunchKernelGGL((pad_kernel<uint16_t>), g, b, 0, s, (const uint16_t*)x, (uint16_t*)y, n, a, (uint16_t)cbits); break;
    case 4: hipLaunchKernelGGL((pad_kernel<uint32_t>), g, b, 0, s, (const uint32_t*)x, (uint32_t*)y, n, a, (uint32_t)cbits); break;
    case 8: hipLaunchKernelGGL((pad_kernel<uint64_t>), g, b, 0, s, (const uint64_t*)x, (uint64_t*)y, n, a, (uint64_t)cbits); break;
    default: TFA_CHECK(false, "pad: element size ", elem_size);
  }
  TFA_LAUNCH_CHECK("pad");
}

void scan(bool prod, DType dt, const void* x, void* y, int64_t outer, int64_t n, int64_t inner, bool exclusive,
          bool reverse, hipStream_t s) {
  if (outer * n * inner <= 0) return;
  switch (dt) {
    case DType::F32: scan_t<float>(prod, x, y, outer, n, inner, exclusive, reverse, s); break;
    case DType::F64: scan_t<double>(prod, x, y, outer, n, inner, exclusive, reverse, s); break;
    case DType::I32: scan_t<int32_t>(prod, x, y, outer, n, inner, exclusive, reverse, s); break;
    case DType::I64: scan_t<int64_t>(prod, x, y, outer, n, inner, exclusive, reverse, s); break;
    default: TFA_CHECK(false, "scan: dtype ", dtype_name(dt), " not supported");
  }
  TFA_LAUNCH_CHECK("scan");
}

void leaky_relu(DType dt, const void* x, void* y, int64_t n, double alpha, hipStream_t s) {
  if (n <= 0) return;
  if (dt == DType::F32)
    hipLaunchKernelGGL((leaky_relu_kernel<float>), dim3(ew_grid(n)), dim3(256), 0, s, (const float*)x, (float*)y, n,
                       (float)alpha);
  else if (dt == DType::F64)
    hipLaunchKernelGGL((leaky_relu_kernel<double>), dim3(ew_grid(n)), dim3(256), 0, s, (const double*)x, (double*)y,
                       n, alpha);
  else
    TFA_CHECK(false, "LeakyRelu: dtype ", dtype_name(dt), " not supported");
  TFA_LAUNCH_CHECK("leaky_relu");
}

void depthwise_conv2d_nhwc(const DepthwiseArgs& a, hipStream_t s) {
  const int64_t total = a.N * a.OH * a.OW * a.C * a.M;
  if (total <= 0) return;
  hipLaunchKernelGGL(depthwise_kernel, dim3(ew_grid(total)), dim3(256), 0, s, a, total);
  TFA_LAUNCH_CHECK("depthwise_conv2d");
}

void lrn(DType dt, const void* x, void* y, int64_t n, int64_t C, int radius, double bias, double alpha, double beta,
         hipStream_t s) {
  if (n <= 0) return;
  if (dt == DType::F32)
    hipLaunchKernelGGL((lrn_kernel<float>), dim3(ew_grid(n)), dim3(256), 0, s, (const float*)x, (float*)y, n, C,
                       radius, (float)bias, (float)alpha, (float)beta);
  else if (dt == DType::F64)
    hipLaunchKernelGGL((lrn_kernel<double>), dim3(ew_grid(n)), dim3(256), 0, s, (const double*)x, (double*)y, n, C,
                       radius, (float)bias, (float)alpha, (float)beta);
  else
    TFA_CHECK(false, "LRN: dtype ", dtype_name(dt), " not supported");
  TFA_LAUNCH_CHECK("lrn");
}

void gather_nd(int64_t elem_size, DType idt, const void* params, const void* idx, void* out, int64_t nidx,
               int64_t inner, const GatherNdArgs& a, hipStream_t s) {
  const int64_t total = nidx * inner;
  if (total <= 0) return;
  TFA_CHECK(a.K >= 0 && a.K <= kMaxRank, "GatherNd: index depth ", a.K);
#define TFA_GND(E)                                                                                         \
  if (idt == DType::I32)                                                                                   \
    hipLaunchKernelGGL((gather_nd_kernel<E, int32_t>), dim3(ew_grid(total)), dim3(256), 0, s, (const E*)params, \
                       (const int32_t*)idx, (E*)out, nidx, inner, a);                                     \
  else                                                                                                     \
    hipLaunchKernelGGL((gather_nd_kernel<E, int64_t>), dim3(ew_grid(total)), dim3(256), 0, s, (const E*)params, \
                       (const int64_t*)idx, (E*)out, nidx, inner, a)
  switch (elem_size) {
    case 1: TFA_GND(uint8_t); break;
    case 2: TFA_GND(uint16_t); break;
    case 4: TFA_GND(uint32_t); break;
    case 8: TFA_GND(uint64_t); break;
    default: TFA_CHECK(false, "GatherNd: element size ", elem_size);
  }
#undef TFA_GND
  TFA_LAUNCH_CHECK("gather_nd");
}

// ---- batched copy: up to kMaxCopyPieces contiguous pieces into one buffer
// in ONE launch (a row concatenation of many small device tensors costs one
// kernel, not one DMA call per piece). blockIdx.y = piece; 16-byte accesses
// when the piece's source and destination are 16-byte aligned.
__global__ __launch_bounds__(256) void batched_copy_kernel(CopyPieces pc, char* __restrict__ dst) {
  const int p = blockIdx.y;
  const char* src = static_cast<const char*>(pc.src[p]);
  char* d = dst + pc.dst_off[p];
  const int64_t nb = pc.bytes[p];
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
    const int64_t n16 = nb / 16;
    for (int64_t i = tid; i < n16; i += stride)
      reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(src)[i];
    for (int64_t i = n16 * 16 + tid; i < nb; i += stride) d[i] = src[i];
  } else {
    for (int64_t i = tid; i < nb; i += stride) d[i] = src[i];
  }
}

void batched_copy(const CopyPieces& pc, void* dst, hipStream_t s) {
  TFA_CHECK(pc.n >= 0 && pc.n <= kMaxCopyPieces, "batched_copy: at most ", kMaxCopyPieces, " pieces");
  if (pc.n == 0) return;
  int64_t mx = 0;
  for (int i = 0; i < pc.n; ++i) {
    TFA_CHECK(pc.bytes[i] >= 0, "batched_copy: negative size");
    mx = std::max(mx, pc.bytes[i]);
  }
  if (mx == 0) return;
  const int gx = static_cast<int>(std::min<int64_t>((mx / 16 + 255) / 256 + 1, 1024));
  hipLaunchKernelGGL(batched_copy_kernel, dim3(gx, pc.n), dim3(256), 0, s, pc, static_cast<char*>(dst));
  TFA_LAUNCH_CHECK("batched_copy");
}

void mask_prefix(const uint8_t* mask, int64_t* pos, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(mask_to_i64, dim3(ew_grid(n)), dim3(256), 0, s, mask, pos, n);
  scan_t<int64_t>(false, pos, pos, 1, n, 1, false, false, s);
  TFA_LAUNCH_CHECK("mask_prefix");
}

void where_coords(const uint8_t* mask, const int64_t* pos, int64_t* out, int64_t n, const WhereArgs& a,
                  hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(where_kernel, dim3(ew_grid(n)), dim3(256), 0, s, mask, pos, out, n, a);
  TFA_LAUNCH_CHECK("where");
}

}  // namespace k
}  // namespace tfa

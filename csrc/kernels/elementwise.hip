// Elementwise + data-movement kernels for gfx950.
//
// Memory-bound: 16-byte vector loads/stores per lane (dwordx4), 4 vectors per
// lane in flight, one block of 256 threads (4 waves) per 1024 vectors (the
// binary/unary hot paths; other kernels grid-stride over <= 2048 blocks), the hot arithmetic ops
// specialised at compile time (Add/Sub/Mul/Div/Max/Min on f32/f64 for the
// same-shape, scalar and row-broadcast forms), the rest through a wave-uniform
// op switch.
#include <cmath>
#include <cstdlib>

#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

template <typename T, int VEC>
struct alignas(sizeof(T) * VEC) Vec {
  T v[VEC];
};

template <typename T>
__device__ __forceinline__ T ipow(T base, T e) {
  if (e < 0) return base == 1 ? T(1) : (base == -1 ? ((e & 1) ? T(-1) : T(1)) : T(0));
  T r = 1;
  while (e) {
    if (e & 1) r *= base;
    base *= base;
    e >>= 1;
  }
  return r;
}

template <typename T>
__device__ __forceinline__ T bin_arith(int op, T a, T b) {
  constexpr bool F = std::is_floating_point<T>::value;
  switch (op) {
    case (int)BinOp::ADD: return a + b;
    case (int)BinOp::SUB: return a - b;
    case (int)BinOp::MUL: return a * b;
    case (int)BinOp::DIV:
      if constexpr (F) return a / b;
      else return b == 0 ? T(0) : T(a / b);
    case (int)BinOp::FLOORDIV:
      if constexpr (F) return floor(a / b);
      else {
        if (b == 0) return T(0);
        T q = a / b;
        if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
        return q;
      }
    case (int)BinOp::FLOORMOD:
      if constexpr (F) {
        T r = fmod(a, b);
        if (r != 0 && ((r < 0) != (b < 0))) r += b;
        return r;
      } else {
        if (b == 0) return T(0);
        T r = a % b;
        if (r != 0 && ((r < 0) != (b < 0))) r += b;
        return r;
      }
    case (int)BinOp::TRUNCMOD:
      if constexpr (F) return fmod(a, b);
      else return b == 0 ? T(0) : T(a % b);
    case (int)BinOp::MAX:
      if constexpr (F) return (a != a || b != b) ? (a + b) : (a > b ? a : b);
      else return a > b ? a : b;
    case (int)BinOp::MIN:
      if constexpr (F) return (a != a || b != b) ? (a + b) : (a < b ? a : b);
      else return a < b ? a : b;
    case (int)BinOp::POW:
      if constexpr (F) return pow(a, b);
      else return ipow(a, b);
    case (int)BinOp::SQDIFF: { T d = a - b; return d * d; }
    case (int)BinOp::ATAN2:
      if constexpr (F) return atan2(a, b);
      else return T(atan2((double)a, (double)b));
    case (int)BinOp::DIVNONAN:
      if constexpr (F) return b == T(0) ? T(0) : a / b;
      else return b == 0 ? T(0) : T(a / b);
    case (int)BinOp::LAND: return T(a && b);
    case (int)BinOp::LOR: return T(a || b);
  }
  return a;
}

template <typename T>
__device__ __forceinline__ uint8_t bin_cmp(int op, T a, T b) {
  switch (op) {
    case (int)BinOp::EQ: return a == b;
    case (int)BinOp::NE: return a != b;
    case (int)BinOp::LT: return a < b;
    case (int)BinOp::LE: return a <= b;
    case (int)BinOp::GT: return a > b;
    case (int)BinOp::GE: return a >= b;
    case (int)BinOp::LAND: return (a != T(0)) && (b != T(0));
    case (int)BinOp::LOR: return (a != T(0)) || (b != T(0));
  }
  return 0;
}

// compile-time specialised op (OPC >= 0) or runtime switch
template <typename T, typename TO, int OPC>
__device__ __forceinline__ TO apply_bin(int op, T a, T b) {
  if constexpr (std::is_same<TO, uint8_t>::value && !std::is_same<T, uint8_t>::value) {
    return bin_cmp<T>(op, a, b);
  } else if constexpr (std::is_same<T, uint8_t>::value) {
    return bin_cmp<T>(op, a, b);
  } else if constexpr (OPC >= 0) {
    return bin_arith<T>(OPC, a, b);
  } else {
    return bin_arith<T>(op, a, b);
  }
}

// MODE: 0 same shape, 1 b scalar, 2 a scalar, 3 row broadcast (b[i % inner])
template <typename T, typename TO, int MODE, int VEC, int OPC>
__global__ __launch_bounds__(256) void binary_vec_kernel(int op, const T* __restrict__ a,
                                                         const T* __restrict__ b,
                                                         TO* __restrict__ out, int64_t n,
                                                         int64_t inner) {
  const int64_t nvec = n / VEC;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  T sa = MODE == 2 ? a[0] : T(0);
  T sb = MODE == 1 ? b[0] : T(0);
  // U vectors per lane per step, all loads issued before any use: 4x the
  // bytes in flight of one-vector-per-step (HBM needs ~64 KB in flight per CU;
  // with the uncapped grid, 1M x 128 f32 Add 5.3 -> 5.8 TB/s, scripts/hbm_probe.py)
  constexpr int U = VEC > 1 ? 4 : 1;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < nvec; base += stride * U) {
    Vec<T, VEC> va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i >= nvec) break;
      if (MODE != 2) va[u] = reinterpret_cast<const Vec<T, VEC>*>(a)[i];
      if (MODE == 0 || MODE == 2) vb[u] = reinterpret_cast<const Vec<T, VEC>*>(b)[i];
      if (MODE == 3) vb[u] = *reinterpret_cast<const Vec<T, VEC>*>(b + ((i * VEC) % inner));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i >= nvec) break;
      Vec<TO, VEC> vo;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        T x = MODE == 2 ? sa : va[u].v[j];
        T y = MODE == 1 ? sb : vb[u].v[j];
        vo.v[j] = apply_bin<T, TO, OPC>(op, x, y);
      }
      reinterpret_cast<Vec<TO, VEC>*>(out)[i] = vo;
    }
  }
  // tail
  for (int64_t i = nvec * VEC + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    T x = MODE == 2 ? sa : a[i];
    T y = MODE == 1 ? sb : (MODE == 3 ? b[i % inner] : b[i]);
    out[i] = apply_bin<T, TO, OPC>(op, x, y);
  }
}

template <typename T, typename TO>
__global__ __launch_bounds__(256) void binary_bcast_kernel(int op, const T* __restrict__ a,
                                                           const T* __restrict__ b,
                                                           TO* __restrict__ out, int64_t n,
                                                           Bcast bc) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t oa = bcast_offset(i, bc.rank, bc.dims, bc.sa);
    int64_t ob = bcast_offset(i, bc.rank, bc.dims, bc.sb);
    out[i] = apply_bin<T, TO, -1>(op, a[oa], b[ob]);
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// block cap of the unrolled streaming kernels: effectively none (one block per
// 256 x 4 vectors). Measured on MI355X, f32 Add of 4M x 128 (scripts/hbm_probe.py):
// 2048 blocks (grid-stride) 5.0 TB/s, 16384 5.3, uncapped 5.7 (ATen 6.1); 1M x 128:
// 5.6 / 5.8 / 5.8 (ATen 6.0). TFA_EW_MAX_BLOCKS overrides.
int ew_max_blocks() {
  static const int v = static_cast<int>(std::min<int64_t>(env_positive("TFA_EW_MAX_BLOCKS", 1 << 22), 1 << 30));
  return v;
}

template <typename T, typename TO, int MODE, int OPC>
void launch_vec(int op, const T* a, const T* b, TO* out, int64_t n, int64_t inner, hipStream_t s) {
  constexpr int VEC = 16 / sizeof(T);
  bool vec_ok = aligned16(a) && aligned16(b) && aligned16(out) &&
                (MODE != 3 || inner % VEC == 0) && (sizeof(TO) * VEC) % sizeof(TO) == 0;
  if (std::is_same<TO, uint8_t>::value && !aligned16(out)) vec_ok = false;
  if (vec_ok) {
    hipLaunchKernelGGL((binary_vec_kernel<T, TO, MODE, VEC, OPC>), dim3(ew_grid((n / VEC + 3) / 4, 256, ew_max_blocks())),
                       dim3(256), 0, s, op, a, b, out, n, inner);
  } else {
    hipLaunchKernelGGL((binary_vec_kernel<T, TO, MODE, 1, OPC>), dim3(ew_grid(n)), dim3(256), 0, s,
                       op, a, b, out, n, inner);
  }
}

template <typename T, typename TO, int MODE>
void launch_mode_hot(BinOp op, const T* a, const T* b, TO* out, int64_t n, int64_t inner, hipStream_t s) {
  switch (op) {
    case BinOp::ADD: return launch_vec<T, TO, MODE, (int)BinOp::ADD>((int)op, a, b, out, n, inner, s);
    case BinOp::SUB: return launch_vec<T, TO, MODE, (int)BinOp::SUB>((int)op, a, b, out, n, inner, s);
    case BinOp::MUL: return launch_vec<T, TO, MODE, (int)BinOp::MUL>((int)op, a, b, out, n, inner, s);
    case BinOp::DIV: return launch_vec<T, TO, MODE, (int)BinOp::DIV>((int)op, a, b, out, n, inner, s);
    default: return launch_vec<T, TO, MODE, -1>((int)op, a, b, out, n, inner, s);
  }
}

template <typename T, typename TO>
void binary_typed(BinOp op, const void* a, const void* b, void* out, int64_t n, int mode,
                  int64_t inner, const Bcast* bc, hipStream_t s) {
  const T* pa = static_cast<const T*>(a);
  const T* pb = static_cast<const T*>(b);
  TO* po = static_cast<TO*>(out);
  constexpr bool hot = std::is_floating_point<T>::value && !std::is_same<TO, uint8_t>::value;
  switch (mode) {
    case 0:
      if constexpr (hot) launch_mode_hot<T, TO, 0>(op, pa, pb, po, n, inner, s);
      else launch_vec<T, TO, 0, -1>((int)op, pa, pb, po, n, inner, s);
      break;
    case 1:
      if constexpr (hot) launch_mode_hot<T, TO, 1>(op, pa, pb, po, n, inner, s);
      else launch_vec<T, TO, 1, -1>((int)op, pa, pb, po, n, inner, s);
      break;
    case 2: launch_vec<T, TO, 2, -1>((int)op, pa, pb, po, n, inner, s); break;
    case 3:
      if constexpr (hot) launch_mode_hot<T, TO, 3>(op, pa, pb, po, n, inner, s);
      else launch_vec<T, TO, 3, -1>((int)op, pa, pb, po, n, inner, s);
      break;
    default:
      TFA_CHECK(bc != nullptr, "binary: broadcast descriptor missing");
      hipLaunchKernelGGL((binary_bcast_kernel<T, TO>), dim3(ew_grid(n)), dim3(256), 0, s, (int)op,
                         pa, pb, po, n, *bc);
  }
}

bool is_cmp_op(BinOp op) {
  return op == BinOp::EQ || op == BinOp::NE || op == BinOp::LT || op == BinOp::LE ||
         op == BinOp::GT || op == BinOp::GE || op == BinOp::LAND || op == BinOp::LOR;
}

// ------------------------------------------------------------------ unary
template <typename T>
__device__ __forceinline__ T un_apply(int op, T x) {
  constexpr bool F = std::is_floating_point<T>::value;
  using C = typename std::conditional<F, T, double>::type;  // compute type for transcendental
  C xc = C(x);
  switch (op) {
    case (int)UnOp::NEG: return -x;
    case (int)UnOp::ABS: return x < 0 ? -x : x;
    case (int)UnOp::SQUARE: return x * x;
    case (int)UnOp::SQRT: return T(sqrt(xc));
    case (int)UnOp::RSQRT: return T(C(1) / sqrt(xc));
    case (int)UnOp::EXP: return T(exp(xc));
    case (int)UnOp::LOG: return T(log(xc));
    case (int)UnOp::LOG1P: return T(log1p(xc));
    case (int)UnOp::EXPM1: return T(expm1(xc));
    case (int)UnOp::RECIP:
      if constexpr (F) return T(1) / x;
      else return x == 0 ? T(0) : T(1 / x);
    case (int)UnOp::RELU: return x > T(0) ? x : T(0);
    case (int)UnOp::RELU6: return x > T(0) ? (x < T(6) ? x : T(6)) : T(0);
    case (int)UnOp::ELU: return x > T(0) ? x : T(expm1(xc));
    case (int)UnOp::SELU: {
      const C alpha = C(1.6732632423543772848170429916717), scale = C(1.0507009873554804934193349852946);
      return T(x > T(0) ? scale * xc : scale * alpha * expm1(xc));
    }
    case (int)UnOp::SIGMOID: return T(C(1) / (C(1) + exp(-xc)));
    case (int)UnOp::TANH: return T(tanh(xc));
    case (int)UnOp::SOFTPLUS: return T(xc > C(20) ? xc : log1p(exp(xc)));
    case (int)UnOp::SOFTSIGN: return T(xc / (C(1) + fabs(xc)));
    case (int)UnOp::FLOOR: return F ? T(floor(xc)) : x;
    case (int)UnOp::CEIL: return F ? T(ceil(xc)) : x;
    case (int)UnOp::ROUND: return F ? T(rint(xc)) : x;
    case (int)UnOp::SIGN: return T((x > T(0)) - (x < T(0)));
    case (int)UnOp::SIN: return T(sin(xc));
    case (int)UnOp::COS: return T(cos(xc));
    case (int)UnOp::TAN: return T(tan(xc));
    case (int)UnOp::NOT: return T(!x);
    case (int)UnOp::ERF: return T(erf(xc));
    case (int)UnOp::IDENTITY: return x;
  }
  return x;
}

template <typename T, int VEC>
__global__ __launch_bounds__(256) void unary_kernel(int op, const T* __restrict__ x,
                                                    T* __restrict__ y, int64_t n) {
  const int64_t nvec = n / VEC;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  constexpr int U = VEC > 1 ? 4 : 1;  // loads of U vectors in flight per lane (see binary_vec_kernel)
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < nvec; base += stride * U) {
    Vec<T, VEC> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i >= nvec) break;
      v[u] = reinterpret_cast<const Vec<T, VEC>*>(x)[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i >= nvec) break;
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[u].v[j] = un_apply<T>(op, v[u].v[j]);
      reinterpret_cast<Vec<T, VEC>*>(y)[i] = v[u];
    }
  }
  for (int64_t i = nvec * VEC + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = un_apply<T>(op, x[i]);
}

template <typename T>
__global__ __launch_bounds__(256) void unary_pred_kernel(int op, const T* __restrict__ x,
                                                         uint8_t* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    T v = x[i];
    uint8_t r = 0;
    if constexpr (std::is_floating_point<T>::value) {
      if (op == (int)UnOp::ISNAN) r = isnan(v);
      else if (op == (int)UnOp::ISINF) r = isinf(v);
      else r = isfinite(v);
    } else {
      r = op == (int)UnOp::ISFINITE;
    }
    y[i] = r;
  }
}

template <typename T>
void unary_typed(UnOp op, const void* x, void* y, int64_t n, hipStream_t s) {
  if (op == UnOp::ISNAN || op == UnOp::ISINF || op == UnOp::ISFINITE) {
    hipLaunchKernelGGL((unary_pred_kernel<T>), dim3(ew_grid(n)), dim3(256), 0, s, (int)op,
                       static_cast<const T*>(x), static_cast<uint8_t*>(y), n);
    return;
  }
  constexpr int VEC = 16 / sizeof(T);
  if (aligned16(x) && aligned16(y))
    hipLaunchKernelGGL((unary_kernel<T, VEC>), dim3(ew_grid((n / VEC + 3) / 4, 256, ew_max_blocks())), dim3(256), 0, s,
                       (int)op, static_cast<const T*>(x), static_cast<T*>(y), n);
  else
    hipLaunchKernelGGL((unary_kernel<T, 1>), dim3(ew_grid(n)), dim3(256), 0, s, (int)op,
                       static_cast<const T*>(x), static_cast<T*>(y), n);
}

// ------------------------------------------------------------------ cast / fill / range
// TO_BOOL: BOOL and U8 share uint8_t storage; only a cast to BOOL is `x != 0`
template <typename F, typename T, bool TO_BOOL = false>
__global__ __launch_bounds__(256) void cast_kernel(const F* __restrict__ x, T* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if constexpr (TO_BOOL)
      y[i] = x[i] != F(0);
    else
      y[i] = static_cast<T>(x[i]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void fill_kernel(T* __restrict__ y, int64_t n, T v) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = v;
}

template <typename T>
__global__ __launch_bounds__(256) void range_kernel(T* __restrict__ y, int64_t n, double s, double d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = static_cast<T>(s + d * (double)i);
}

template <typename T>
__global__ __launch_bounds__(256) void select_kernel(const uint8_t* __restrict__ c, const T* __restrict__ a,
                                                     const T* __restrict__ b, T* __restrict__ out,
                                                     int64_t n, Bcast bc) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t oc = bcast_offset(i, bc.rank, bc.dims, bc.sc);
    int64_t oa = bcast_offset(i, bc.rank, bc.dims, bc.sa);
    int64_t ob = bcast_offset(i, bc.rank, bc.dims, bc.sb);
    out[i] = c[oc] ? a[oa] : b[ob];
  }
}

// ------------------------------------------------------------------ data movement
struct CopyDesc {
  int rank;
  int64_t dims[kMaxRank];
  int64_t ss[kMaxRank];
  int64_t ds[kMaxRank];
};

template <typename E, typename I>
__global__ __launch_bounds__(256) void strided_copy_kernel(const E* __restrict__ src, E* __restrict__ dst,
                                                           I n, CopyDesc d) {
  const I stride = (I)gridDim.x * blockDim.x;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    I rem = i;
    int64_t so = 0, dof = 0;
    for (int k2 = d.rank - 1; k2 >= 0; --k2) {
      const I dim = (I)d.dims[k2];
      const I q = rem / dim;
      const I r = rem - q * dim;
      so += (int64_t)r * d.ss[k2];
      dof += (int64_t)r * d.ds[k2];
      rem = q;
    }
    dst[dof] = src[so];
  }
}

template <typename E, typename I>
__global__ __launch_bounds__(256) void gather_kernel(const E* __restrict__ params, const I* __restrict__ idx,
                                                     E* __restrict__ out, int64_t outer, int64_t axis_dim,
                                                     int64_t nidx, int64_t inner) {
  const int64_t n = outer * nidx * inner;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t in_ = i % inner;
    int64_t t = i / inner;
    int64_t j = t % nidx;
    int64_t o = t / nidx;
    int64_t ix = static_cast<int64_t>(idx[j]);
    out[i] = (ix >= 0 && ix < axis_dim) ? params[(o * axis_dim + ix) * inner + in_] : E{};
  }
}

template <typename T, typename I>
__global__ __launch_bounds__(256) void one_hot_kernel(const I* __restrict__ idx, T* __restrict__ out,
                                                      int64_t n, int64_t depth, T on, T off) {
  const int64_t total = n * depth;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride)
    out[i] = (static_cast<int64_t>(idx[i / depth]) == i % depth) ? on : off;
}

template <typename T>
__global__ __launch_bounds__(256) void channel_affine_kernel(const T* __restrict__ x, const T* __restrict__ sc,
                                                             const T* __restrict__ sh, T* __restrict__ y,
                                                             int64_t n, int64_t C, int act) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t c = i % C;
    y[i] = act_apply<T>(x[i] * sc[c] + sh[c], act);
  }
}

template <int ES>
struct ElemOf;
template <> struct ElemOf<1> { using T = uint8_t; };
template <> struct ElemOf<2> { using T = uint16_t; };
template <> struct ElemOf<4> { using T = uint32_t; };
template <> struct ElemOf<8> { using T = uint64_t; };

}  // namespace

// ====================================================================== host API
#define TFA_DISPATCH_NUM(dt, NAME, ...)                                               \
  switch (dt) {                                                                       \
    case DType::F32: { using NAME = float; __VA_ARGS__; break; }                      \
    case DType::F64: { using NAME = double; __VA_ARGS__; break; }                     \
    case DType::I32: { using NAME = int32_t; __VA_ARGS__; break; }                    \
    case DType::I64: { using NAME = int64_t; __VA_ARGS__; break; }                    \
    default: TFA_CHECK(false, "dtype ", dtype_name(dt), " not supported by this kernel"); \
  }

void binary(BinOp op, DType dt, const void* a, const void* b, void* out, int64_t n, int mode,
            int64_t inner, const Bcast* bc, hipStream_t s) {
  if (n <= 0) return;
  TFA_CHECK(mode != 3 || (inner > 0 && n % inner == 0), "binary: bad row-broadcast inner ", inner);
  if (dt == DType::BOOL) {
    TFA_CHECK(is_cmp_op(op), "binary: only logical/comparison ops on bool");
    binary_typed<uint8_t, uint8_t>(op, a, b, out, n, mode, inner, bc, s);
  } else if (is_cmp_op(op)) {
    TFA_DISPATCH_NUM(dt, T, binary_typed<T, uint8_t>(op, a, b, out, n, mode, inner, bc, s));
  } else {
    TFA_DISPATCH_NUM(dt, T, binary_typed<T, T>(op, a, b, out, n, mode, inner, bc, s));
  }
  TFA_LAUNCH_CHECK("binary");
}

void unary(UnOp op, DType dt, const void* x, void* y, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  if (dt == DType::BOOL) {
    TFA_CHECK(op == UnOp::NOT || op == UnOp::IDENTITY, "unary: op not supported on bool");
    unary_typed<uint8_t>(op, x, y, n, s);
  } else {
    TFA_DISPATCH_NUM(dt, T, unary_typed<T>(op, x, y, n, s));
  }
  TFA_LAUNCH_CHECK("unary");
}

template <typename F>
static void cast_from(DType to, const void* x, void* y, int64_t n, hipStream_t s) {
  const F* px = static_cast<const F*>(x);
  switch (to) {
    case DType::F32: hipLaunchKernelGGL((cast_kernel<F, float>), dim3(ew_grid(n)), dim3(256), 0, s, px, (float*)y, n); break;
    case DType::F64: hipLaunchKernelGGL((cast_kernel<F, double>), dim3(ew_grid(n)), dim3(256), 0, s, px, (double*)y, n); break;
    case DType::I32: hipLaunchKernelGGL((cast_kernel<F, int32_t>), dim3(ew_grid(n)), dim3(256), 0, s, px, (int32_t*)y, n); break;
    case DType::I64: hipLaunchKernelGGL((cast_kernel<F, int64_t>), dim3(ew_grid(n)), dim3(256), 0, s, px, (int64_t*)y, n); break;
    case DType::BOOL: hipLaunchKernelGGL((cast_kernel<F, uint8_t, true>), dim3(ew_grid(n)), dim3(256), 0, s, px, (uint8_t*)y, n); break;
    case DType::U8: hipLaunchKernelGGL((cast_kernel<F, uint8_t>), dim3(ew_grid(n)), dim3(256), 0, s, px, (uint8_t*)y, n); break;
    case DType::I8: hipLaunchKernelGGL((cast_kernel<F, int8_t>), dim3(ew_grid(n)), dim3(256), 0, s, px, (int8_t*)y, n); break;
    case DType::I16: hipLaunchKernelGGL((cast_kernel<F, int16_t>), dim3(ew_grid(n)), dim3(256), 0, s, px, (int16_t*)y, n); break;
    default: TFA_CHECK(false, "cast to ", dtype_name(to), " not supported on GPU");
  }
}

void cast(DType from, DType to, const void* x, void* y, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  switch (from) {
    case DType::F32: cast_from<float>(to, x, y, n, s); break;
    case DType::F64: cast_from<double>(to, x, y, n, s); break;
    case DType::I32: cast_from<int32_t>(to, x, y, n, s); break;
    case DType::I64: cast_from<int64_t>(to, x, y, n, s); break;
    case DType::BOOL:
    case DType::U8: cast_from<uint8_t>(to, x, y, n, s); break;
    case DType::I8: cast_from<int8_t>(to, x, y, n, s); break;
    case DType::I16: cast_from<int16_t>(to, x, y, n, s); break;
    default: TFA_CHECK(false, "cast from ", dtype_name(from), " not supported on GPU");
  }
  TFA_LAUNCH_CHECK("cast");
}

void fill(DType dt, void* out, int64_t n, double value, hipStream_t s) {
  if (n <= 0) return;
  switch (dt) {
    case DType::BOOL:
    case DType::U8:
      hipLaunchKernelGGL((fill_kernel<uint8_t>), dim3(ew_grid(n)), dim3(256), 0, s, (uint8_t*)out, n,
                         (uint8_t)value);
      break;
    default:
      TFA_DISPATCH_NUM(dt, T, hipLaunchKernelGGL((fill_kernel<T>), dim3(ew_grid(n)), dim3(256), 0, s,
                                                 (T*)out, n, (T)value));
  }
  TFA_LAUNCH_CHECK("fill");
}

void range(DType dt, void* out, int64_t n, double start, double delta, hipStream_t s) {
  if (n <= 0) return;
  TFA_DISPATCH_NUM(dt, T, hipLaunchKernelGGL((range_kernel<T>), dim3(ew_grid(n)), dim3(256), 0, s,
                                             (T*)out, n, start, delta));
  TFA_LAUNCH_CHECK("range");
}

void select(DType dt, const void* cond, const void* a, const void* b, void* out, int64_t n,
            const Bcast& bc, hipStream_t s) {
  if (n <= 0) return;
  if (dt == DType::BOOL) {
    hipLaunchKernelGGL((select_kernel<uint8_t>), dim3(ew_grid(n)), dim3(256), 0, s, (const uint8_t*)cond,
                       (const uint8_t*)a, (const uint8_t*)b, (uint8_t*)out, n, bc);
  } else {
    TFA_DISPATCH_NUM(dt, T, hipLaunchKernelGGL((select_kernel<T>), dim3(ew_grid(n)), dim3(256), 0, s,
                                               (const uint8_t*)cond, (const T*)a, (const T*)b, (T*)out, n, bc));
  }
  TFA_LAUNCH_CHECK("select");
}

namespace {
template <typename E>
void strided_copy_e(const CopyDesc& d, int64_t n, const void* src, void* dst, hipStream_t s) {
  if (n < (int64_t(1) << 31))
    hipLaunchKernelGGL((strided_copy_kernel<E, uint32_t>), dim3(ew_grid(n)), dim3(256), 0, s, (const E*)src, (E*)dst,
                       (uint32_t)n, d);
  else
    hipLaunchKernelGGL((strided_copy_kernel<E, int64_t>), dim3(ew_grid(n)), dim3(256), 0, s, (const E*)src, (E*)dst,
                       n, d);
}
}  // namespace

// Host-side normalisation before the launch: size-1 dims are dropped, dims
// that are contiguous in BOTH operands are merged, and a unit-stride inner
// dim is widened to 16-byte elements when sizes/alignment allow (a channel
// concat of NHWC tensors becomes a rank-2 float4 copy).
void strided_copy(int64_t elem_size, int rank, const int64_t* dims, const void* src,
                  const int64_t* src_strides, void* dst, const int64_t* dst_strides, hipStream_t s) {
  TFA_CHECK(rank >= 1 && rank <= kMaxRank, "strided_copy: bad rank ", rank);
  CopyDesc d;
  d.rank = 0;
  int64_t n = 1;
  for (int i = 0; i < rank; ++i) {
    n *= dims[i];
    if (dims[i] == 1) continue;
    if (d.rank > 0 && d.ss[d.rank - 1] == src_strides[i] * dims[i] && d.ds[d.rank - 1] == dst_strides[i] * dims[i]) {
      d.dims[d.rank - 1] *= dims[i];  // merge into the previous (outer) dim
      d.ss[d.rank - 1] = src_strides[i];
      d.ds[d.rank - 1] = dst_strides[i];
      continue;
    }
    d.dims[d.rank] = dims[i];
    d.ss[d.rank] = src_strides[i];
    d.ds[d.rank] = dst_strides[i];
    ++d.rank;
  }
  if (n <= 0) return;
  if (d.rank == 0) {  // single element
    d.rank = 1;
    d.dims[0] = 1;
    d.ss[0] = d.ds[0] = 1;
  }
  // widen a unit-stride inner dim to 16-byte elements
  const int last = d.rank - 1;
  if (elem_size < 16 && d.ss[last] == 1 && d.ds[last] == 1) {
    const int64_t f = 16 / elem_size;
    bool ok = d.dims[last] % f == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
              (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
    for (int i = 0; ok && i < last; ++i) ok = d.ss[i] % f == 0 && d.ds[i] % f == 0;
    if (ok) {
      d.dims[last] /= f;
      for (int i = 0; i < last; ++i) {
        d.ss[i] /= f;
        d.ds[i] /= f;
      }
      strided_copy_e<uint4>(d, n / f, src, dst, s);
      TFA_LAUNCH_CHECK("strided_copy");
      return;
    }
  }
  switch (elem_size) {
    case 1: strided_copy_e<uint8_t>(d, n, src, dst, s); break;
    case 2: strided_copy_e<uint16_t>(d, n, src, dst, s); break;
    case 4: strided_copy_e<uint32_t>(d, n, src, dst, s); break;
    case 8: strided_copy_e<uint64_t>(d, n, src, dst, s); break;
    default: TFA_CHECK(false, "strided_copy: element size ", elem_size);
  }
  TFA_LAUNCH_CHECK("strided_copy");
}

template <typename E>
static void gather_e(DType idt, const void* params, const void* idx, void* out, int64_t outer,
                     int64_t axis_dim, int64_t nidx, int64_t inner, hipStream_t s) {
  int64_t n = outer * nidx * inner;
  if (idt == DType::I32)
    hipLaunchKernelGGL((gather_kernel<E, int32_t>), dim3(ew_grid(n)), dim3(256), 0, s, (const E*)params,
                       (const int32_t*)idx, (E*)out, outer, axis_dim, nidx, inner);
  else if (idt == DType::I64)
    hipLaunchKernelGGL((gather_kernel<E, int64_t>), dim3(ew_grid(n)), dim3(256), 0, s, (const E*)params,
                       (const int64_t*)idx, (E*)out, outer, axis_dim, nidx, inner);
  else
    TFA_CHECK(false, "gather: indices must be int32/int64");
}

void gather(int64_t elem_size, DType idt, const void* params, const void* idx, void* out,
            int64_t outer, int64_t axis_dim, int64_t nidx, int64_t inner, hipStream_t s) {
  if (outer * nidx * inner <= 0) return;
  switch (elem_size) {
    case 1: gather_e<uint8_t>(idt, params, idx, out, outer, axis_dim, nidx, inner, s); break;
    case 2: gather_e<uint16_t>(idt, params, idx, out, outer, axis_dim, nidx, inner, s); break;
    case 4: gather_e<uint32_t>(idt, params, idx, out, outer, axis_dim, nidx, inner, s); break;
    case 8: gather_e<uint64_t>(idt, params, idx, out, outer, axis_dim, nidx, inner, s); break;
    default: TFA_CHECK(false, "gather: element size ", elem_size);
  }
  TFA_LAUNCH_CHECK("gather");
}

void one_hot(DType dt, DType idt, const void* idx, void* out, int64_t n, int64_t depth, double on,
             double off, hipStream_t s) {
  if (n * depth <= 0) return;
  TFA_CHECK(idt == DType::I32 || idt == DType::I64 || idt == DType::U8, "one_hot: bad index dtype");
  TFA_DISPATCH_NUM(dt, T, {
    if (idt == DType::I32)
      hipLaunchKernelGGL((one_hot_kernel<T, int32_t>), dim3(ew_grid(n * depth)), dim3(256), 0, s,
                         (const int32_t*)idx, (T*)out, n, depth, (T)on, (T)off);
    else if (idt == DType::I64)
      hipLaunchKernelGGL((one_hot_kernel<T, int64_t>), dim3(ew_grid(n * depth)), dim3(256), 0, s,
                         (const int64_t*)idx, (T*)out, n, depth, (T)on, (T)off);
    else
      hipLaunchKernelGGL((one_hot_kernel<T, uint8_t>), dim3(ew_grid(n * depth)), dim3(256), 0, s,
                         (const uint8_t*)idx, (T*)out, n, depth, (T)on, (T)off);
  });
  TFA_LAUNCH_CHECK("one_hot");
}

void channel_affine(DType dt, const void* x, const void* scale, const void* shift, void* y,
                    int64_t n, int64_t C, int act, hipStream_t s) {
  if (n <= 0) return;
  TFA_CHECK(C > 0 && n % C == 0, "channel_affine: bad channel count");
  if (dt == DType::F32)
    hipLaunchKernelGGL((channel_affine_kernel<float>), dim3(ew_grid(n)), dim3(256), 0, s, (const float*)x,
                       (const float*)scale, (const float*)shift, (float*)y, n, C, act);
  else if (dt == DType::F64)
    hipLaunchKernelGGL((channel_affine_kernel<double>), dim3(ew_grid(n)), dim3(256), 0, s, (const double*)x,
                       (const double*)scale, (const double*)shift, (double*)y, n, C, act);
  else
    TFA_CHECK(false, "channel_affine: float types only");
  TFA_LAUNCH_CHECK("channel_affine");
}

}  // namespace k
}  // namespace tfa

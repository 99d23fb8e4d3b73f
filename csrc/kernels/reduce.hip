// Reductions for gfx950: Sum/Prod/Min/Max/Mean/All/Any over [outer, r, inner],
// arg-min/max, row softmax, row top-k, segment reductions.
//
// All float sums accumulate in f64 and every multi-block reduction goes
// through a fixed-order partial-slab pass (no float atomics), so results are
// bitwise reproducible run to run.
#include <cstdlib>
#include <cfloat>
#include <climits>
#include <cmath>

#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

template <typename T> struct AccT { using type = double; };
template <> struct AccT<int32_t> { using type = int64_t; };
template <> struct AccT<int64_t> { using type = int64_t; };
template <> struct AccT<uint8_t> { using type = int64_t; };

template <typename A>
__device__ __forceinline__ A big_pos() {
  if constexpr (std::is_floating_point<A>::value) return INFINITY;
  else return LLONG_MAX;
}
template <typename A>
__device__ __forceinline__ A big_neg() {
  if constexpr (std::is_floating_point<A>::value) return -INFINITY;
  else return LLONG_MIN;
}

template <int OP, typename A>
__device__ __forceinline__ A ident() {
  if constexpr (OP == (int)RedOp::SUM || OP == (int)RedOp::MEAN || OP == (int)RedOp::ANY) return A(0);
  else if constexpr (OP == (int)RedOp::PROD || OP == (int)RedOp::ALL) return A(1);
  else if constexpr (OP == (int)RedOp::MIN) return big_pos<A>();
  else return big_neg<A>();
}

template <int OP, typename A>
__device__ __forceinline__ A combine(A a, A b) {
  if constexpr (OP == (int)RedOp::SUM || OP == (int)RedOp::MEAN) return a + b;
  else if constexpr (OP == (int)RedOp::PROD) return a * b;
  else if constexpr (OP == (int)RedOp::MIN || OP == (int)RedOp::ALL) return b < a ? b : a;
  else return b > a ? b : a;
}

template <int OP, typename A>
__device__ __forceinline__ A wave_reduce(A v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = combine<OP, A>(v, __shfl_xor(v, off, 64));
  return v;
}

template <int OP, typename T, typename A>
__device__ __forceinline__ T finish(A v, int64_t count) {
  if constexpr (OP == (int)RedOp::MEAN) {
    if constexpr (std::is_floating_point<A>::value) return T(v / A(count));
    else return T(v / count);  // truncating, like TF integer Mean
  } else {
    return T(v);
  }
}

// ---- row reduce (inner == 1): one wave per row
template <typename T, int OP, int VEC>
__global__ __launch_bounds__(256) void row_reduce_wave(const T* __restrict__ x, T* __restrict__ y,
                                                       int64_t outer, int64_t r) {
  using A = typename AccT<T>::type;
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < outer; row += waves) {
    const T* p = x + row * r;
    A acc = ident<OP, A>();
    if (VEC > 1) {
      int64_t nv = r / VEC;
      for (int64_t i = lane; i < nv; i += 64) {
        struct alignas(sizeof(T) * VEC) V { T v[VEC]; } v = reinterpret_cast<const V*>(p)[i];
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc = combine<OP, A>(acc, A(v.v[j]));
      }
      for (int64_t i = nv * VEC + lane; i < r; i += 64) acc = combine<OP, A>(acc, A(p[i]));
    } else {
      for (int64_t i = lane; i < r; i += 64) acc = combine<OP, A>(acc, A(p[i]));
    }
    acc = wave_reduce<OP, A>(acc);
    if (lane == 0) y[row] = finish<OP, T, A>(acc, r);
  }
}

// ---- short rows (inner == 1, r <= kBlockRowBytes): one 1024-thread block per
// row, so a small full reduction (a per-partition Sum of 25k values) is one
// launch instead of a split pass plus a final pass
constexpr int64_t kBlockRowBytes = 256 << 10;
template <typename T, int OP>
__global__ __launch_bounds__(1024) void row_reduce_block(const T* __restrict__ x, T* __restrict__ y, int64_t r) {
  using A = typename AccT<T>::type;
  __shared__ A red[16];
  const T* p = x + (int64_t)blockIdx.x * r;
  A acc = ident<OP, A>();
  // 8 independent loads in flight per thread: one block has no other waves
  // to hide the HBM latency behind
  constexpr int U = 8;
  int64_t i = threadIdx.x;
  for (; i + (U - 1) * 1024 < r; i += U * 1024) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[i + u * 1024];
#pragma unroll
    for (int u = 0; u < U; ++u) acc = combine<OP, A>(acc, A(v[u]));
  }
  for (; i < r; i += 1024) acc = combine<OP, A>(acc, A(p[i]));
  acc = wave_reduce<OP, A>(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    A t = red[0];
#pragma unroll
    for (int w = 1; w < 16; ++w) t = combine<OP, A>(t, red[w]);
    y[blockIdx.x] = finish<OP, T, A>(t, r);
  }
}

// ---- column-style reduce over [outer, r, inner]; grid = (col_blocks, outer, S)
// Each thread owns one column and a contiguous slice of r. S > 1 writes
// partials part[s][outer][inner] (accumulator type), combined by col_final.
template <typename T, int OP>
__global__ __launch_bounds__(256) void col_reduce(const T* __restrict__ x, T* __restrict__ y,
                                                  typename AccT<T>::type* __restrict__ part,
                                                  int64_t outer, int64_t r, int64_t inner,
                                                  int64_t rows_per_split) {
  using A = typename AccT<T>::type;
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t o = blockIdx.y;
  const int64_t s = blockIdx.z;
  if (col >= inner) return;
  const int64_t r0 = s * rows_per_split;
  const int64_t r1 = min(r, r0 + rows_per_split);
  const T* p = x + (o * r) * inner + col;
  A acc0 = ident<OP, A>(), acc1 = ident<OP, A>(), acc2 = ident<OP, A>(), acc3 = ident<OP, A>();
  int64_t i = r0;
  for (; i + 4 <= r1; i += 4) {  // 4 independent chains keep 4 loads in flight
    acc0 = combine<OP, A>(acc0, A(p[(i + 0) * inner]));
    acc1 = combine<OP, A>(acc1, A(p[(i + 1) * inner]));
    acc2 = combine<OP, A>(acc2, A(p[(i + 2) * inner]));
    acc3 = combine<OP, A>(acc3, A(p[(i + 3) * inner]));
  }
  for (; i < r1; ++i) acc0 = combine<OP, A>(acc0, A(p[i * inner]));
  A acc = combine<OP, A>(combine<OP, A>(acc0, acc1), combine<OP, A>(acc2, acc3));
  if (part == nullptr) y[o * inner + col] = finish<OP, T, A>(acc, r);
  else part[(s * outer + o) * inner + col] = acc;
}

// Vectorised variant: each thread owns VEC adjacent columns (16-byte loads).
template <typename T, int OP, int VEC>
__global__ __launch_bounds__(256) void col_reduce_vec(const T* __restrict__ x, T* __restrict__ y,
                                                      typename AccT<T>::type* __restrict__ part,
                                                      int64_t outer, int64_t r, int64_t inner,
                                                      int64_t rows_per_split) {
  using A = typename AccT<T>::type;
  struct alignas(sizeof(T) * VEC) V { T v[VEC]; };
  const int64_t cg = (int64_t)blockIdx.x * 256 + threadIdx.x;  // column group
  const int64_t o = blockIdx.y;
  const int64_t s = blockIdx.z;
  if (cg * VEC >= inner) return;
  const int64_t r0 = s * rows_per_split;
  const int64_t r1 = min(r, r0 + rows_per_split);
  const V* p = reinterpret_cast<const V*>(x + (o * r) * inner) + cg;
  const int64_t rs = inner / VEC;  // row stride in vectors
  // 4 rows in flight per thread (4 x 16-byte loads issued before their use)
  constexpr int U = 4;
  A acc[U][VEC];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[u][j] = ident<OP, A>();
  int64_t i = r0;
  for (; i + U <= r1; i += U) {
    V v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[(i + u) * rs];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[u][j] = combine<OP, A>(acc[u][j], A(v[u].v[j]));
  }
  for (; i < r1; ++i) {
    V v0 = p[i * rs];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[0][j] = combine<OP, A>(acc[0][j], A(v0.v[j]));
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    A a = combine<OP, A>(combine<OP, A>(acc[0][j], acc[1][j]), combine<OP, A>(acc[2][j], acc[3][j]));
    int64_t col = cg * VEC + j;
    if (part == nullptr) y[o * inner + col] = finish<OP, T, A>(a, r);
    else part[(s * outer + o) * inner + col] = a;
  }
}

// ---- few long rows (inner == 1): grid = (S, outer), each block folds a
// contiguous slice of its row with all 256 threads, partial -> part[s][outer].
template <typename T, int OP>
__global__ __launch_bounds__(256) void row_split(const T* __restrict__ x,
                                                 typename AccT<T>::type* __restrict__ part,
                                                 int64_t outer, int64_t r, int64_t per_split) {
  using A = typename AccT<T>::type;
  __shared__ A red[4];
  const int64_t s = blockIdx.x, o = blockIdx.y;
  const int64_t r0 = s * per_split, r1 = min(r, r0 + per_split);
  const T* p = x + o * r;
  A acc = ident<OP, A>();
  for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) acc = combine<OP, A>(acc, A(p[i]));
  acc = wave_reduce<OP, A>(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    A t = combine<OP, A>(combine<OP, A>(red[0], red[1]), combine<OP, A>(red[2], red[3]));
    part[s * outer + o] = t;
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(256) void col_final(const typename AccT<T>::type* __restrict__ part,
                                                 T* __restrict__ y, int64_t n, int64_t S, int64_t r) {
  using A = typename AccT<T>::type;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    A acc = ident<OP, A>();
#pragma unroll 8
    for (int64_t s = 0; s < S; ++s) acc = combine<OP, A>(acc, part[s * n + i]);
    y[i] = finish<OP, T, A>(acc, r);
  }
}

// Fold S partial slabs [S][n] into G = ceil(S / F) slabs (F consecutive slabs
// per thread, fixed order), so the final pass is not one thread per column
// walking all S slabs: with n = 1024 columns and S = 2048 that serial walk
// took as long as streaming the 4 GB input.
template <typename T, int OP>
__global__ __launch_bounds__(256) void col_fold(const typename AccT<T>::type* __restrict__ part,
                                                typename AccT<T>::type* __restrict__ part2, int64_t n,
                                                int64_t S, int64_t F) {
  using A = typename AccT<T>::type;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s0 = (int64_t)blockIdx.y * F, s1 = min(S, s0 + F);
  A acc = ident<OP, A>();
#pragma unroll 8
  for (int64_t s = s0; s < s1; ++s) acc = combine<OP, A>(acc, part[s * n + i]);
  part2[(int64_t)blockIdx.y * n + i] = acc;
}

constexpr int64_t kFoldAbove = 64;  // fold first when more partial slabs than this
constexpr int64_t kFoldBy = 32;     // slabs per fold thread

inline int64_t fold_slabs(int64_t S) { return S > kFoldAbove ? (S + kFoldBy - 1) / kFoldBy : 0; }

// part [S][n] -> y (through one fold pass when S is large); part2 follows part in the workspace
template <typename T, int OP>
void final_pass(typename AccT<T>::type* part, T* y, int64_t n, int64_t S, int64_t r, hipStream_t s) {
  const int64_t G = fold_slabs(S);
  if (G > 0 && G <= 65535) {
    auto* part2 = part + S * n;
    hipLaunchKernelGGL((col_fold<T, OP>), dim3((unsigned)((n + 255) / 256), (unsigned)G), dim3(256), 0, s, part,
                       part2, n, S, kFoldBy);
    hipLaunchKernelGGL((col_final<T, OP>), dim3(ew_grid(n)), dim3(256), 0, s, part2, y, n, G, r);
    return;
  }
  hipLaunchKernelGGL((col_final<T, OP>), dim3(ew_grid(n)), dim3(256), 0, s, part, y, n, S, r);
}

struct RedPlan {
  bool row_wave;
  int64_t S;             // r splits (col path)
  int64_t col_blocks;
  int vec;
};

template <typename T>
RedPlan plan_reduce(int64_t outer, int64_t r, int64_t inner) {
  RedPlan p{};
  constexpr int VEC = 16 / sizeof(T) > 0 ? 16 / sizeof(T) : 1;
  if (inner == 1 && (outer >= 1024 || r <= 4096)) {
    p.row_wave = true;
    return p;
  }
  p.row_wave = false;
  if (inner == 1) {  // few long rows: split each row over S blocks
    p.vec = 1;
    p.col_blocks = 0;
    int64_t S = std::max<int64_t>(1, 2048 / std::max<int64_t>(outer, 1));
    p.S = std::min<int64_t>(std::min<int64_t>(S, std::max<int64_t>(1, r / 1024)), 65535);
    return p;
  }
  p.vec = (inner % VEC == 0) ? VEC : 1;
  int64_t cols = (inner + p.vec - 1) / p.vec;
  p.col_blocks = (cols + 255) / 256;
  int64_t blocks = p.col_blocks * outer;
  static const int64_t target = env_positive("TFA_RED_TARGET_BLOCKS", 2048);
  int64_t S = blocks >= target ? 1 : (target + blocks - 1) / blocks;
  int64_t max_s = std::max<int64_t>(1, r / 64);
  p.S = std::min<int64_t>(std::min<int64_t>(S, max_s), 65535);
  return p;
}

template <typename T, int OP>
void reduce_typed(const void* xv, void* yv, int64_t outer, int64_t r, int64_t inner, void* ws,
                  hipStream_t s) {
  using A = typename AccT<T>::type;
  const T* x = static_cast<const T*>(xv);
  T* y = static_cast<T*>(yv);
  RedPlan p = plan_reduce<T>(outer, r, inner);
  if (p.row_wave) {
    constexpr int VEC = 16 / sizeof(T);
    bool vec = (r % VEC == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
    int grid = (int)std::min<int64_t>((outer + 3) / 4, 4096);
    if (vec) hipLaunchKernelGGL((row_reduce_wave<T, OP, VEC>), dim3(grid), dim3(256), 0, s, x, y, outer, r);
    else hipLaunchKernelGGL((row_reduce_wave<T, OP, 1>), dim3(grid), dim3(256), 0, s, x, y, outer, r);
    return;
  }
  int64_t rows_per_split = (r + p.S - 1) / p.S;
  int64_t S = (r + rows_per_split - 1) / rows_per_split;
  if (inner == 1 && S > 1 && outer <= 64 && r * (int64_t)sizeof(T) <= kBlockRowBytes) {
    hipLaunchKernelGGL((row_reduce_block<T, OP>), dim3((unsigned)outer), dim3(1024), 0, s, x, y, r);
    return;
  }
  if (inner == 1) {
    TFA_CHECK(ws != nullptr || S == 1, "reduce: missing workspace");
    TFA_CHECK(outer <= 65535, "reduce: outer dim ", outer, " too large for the split-row path");
    A* part2 = static_cast<A*>(ws);
    if (S == 1) {
      hipLaunchKernelGGL((row_reduce_wave<T, OP, 1>), dim3((unsigned)((outer + 3) / 4)), dim3(256), 0, s, x, y, outer, r);
      return;
    }
    hipLaunchKernelGGL((row_split<T, OP>), dim3((unsigned)S, (unsigned)outer), dim3(256), 0, s, x, part2, outer, r,
                       rows_per_split);
    final_pass<T, OP>(part2, y, outer, S, r, s);
    return;
  }
  TFA_CHECK(outer <= 65535, "reduce: outer dim ", outer, " too large for the column path");
  A* part = S > 1 ? static_cast<A*>(ws) : nullptr;
  TFA_CHECK(S == 1 || ws != nullptr, "reduce: missing workspace");
  dim3 grid((unsigned)p.col_blocks, (unsigned)outer, (unsigned)S);
  bool vec_ok = p.vec > 1 && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  if (vec_ok) {
    constexpr int VEC = 16 / sizeof(T);
    hipLaunchKernelGGL((col_reduce_vec<T, OP, VEC>), grid, dim3(256), 0, s, x, y, part, outer, r, inner,
                       rows_per_split);
  } else {
    dim3 g2((unsigned)((inner + 255) / 256), (unsigned)outer, (unsigned)S);
    hipLaunchKernelGGL((col_reduce<T, OP>), g2, dim3(256), 0, s, x, y, part, outer, r, inner, rows_per_split);
  }
  if (S > 1) {
    final_pass<T, OP>(part, y, outer * inner, S, r, s);
  }
}

template <typename T>
void reduce_dispatch_op(RedOp op, const void* x, void* y, int64_t outer, int64_t r, int64_t inner,
                        void* ws, hipStream_t s) {
  switch (op) {
    case RedOp::SUM: reduce_typed<T, (int)RedOp::SUM>(x, y, outer, r, inner, ws, s); break;
    case RedOp::PROD: reduce_typed<T, (int)RedOp::PROD>(x, y, outer, r, inner, ws, s); break;
    case RedOp::MIN: reduce_typed<T, (int)RedOp::MIN>(x, y, outer, r, inner, ws, s); break;
    case RedOp::MAX: reduce_typed<T, (int)RedOp::MAX>(x, y, outer, r, inner, ws, s); break;
    case RedOp::MEAN: reduce_typed<T, (int)RedOp::MEAN>(x, y, outer, r, inner, ws, s); break;
    default: TFA_CHECK(false, "reduce: op needs bool input");
  }
}

// ---- arg reduce
template <typename T, typename O, bool MIN>
__global__ __launch_bounds__(256) void argreduce_row(const T* __restrict__ x, O* __restrict__ y,
                                                     int64_t outer, int64_t r) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < outer; row += waves) {
    const T* p = x + row * r;
    T best = p[0];
    int64_t bi = 0;
    for (int64_t i = lane; i < r; i += 64) {
      T v = p[i];
      bool better = MIN ? (v < best || (v == best && i < bi)) : (v > best || (v == best && i < bi));
      if (better) { best = v; bi = i; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      T ov = __shfl_xor(best, off, 64);
      int64_t oi = __shfl_xor(bi, off, 64);
      bool better = MIN ? (ov < best || (ov == best && oi < bi)) : (ov > best || (ov == best && oi < bi));
      if (better) { best = ov; bi = oi; }
    }
    if (lane == 0) y[row] = (O)bi;
  }
}

template <typename T, typename O, bool MIN>
__global__ __launch_bounds__(256) void argreduce_col(const T* __restrict__ x, O* __restrict__ y,
                                                     int64_t outer, int64_t r, int64_t inner) {
  const int64_t n = outer * inner;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
    int64_t o = t / inner, c = t % inner;
    const T* p = x + o * r * inner + c;
    T best = p[0];
    int64_t bi = 0;
    for (int64_t i = 1; i < r; ++i) {
      T v = p[i * inner];
      if (MIN ? v < best : v > best) { best = v; bi = i; }
    }
    y[t] = (O)bi;
  }
}

template <typename T, typename O>
void argreduce_typed(bool is_min, const void* xv, void* yv, int64_t outer, int64_t r, int64_t inner,
                     hipStream_t s) {
  const T* x = static_cast<const T*>(xv);
  O* y = static_cast<O*>(yv);
  if (inner == 1) {
    int grid = (int)std::min<int64_t>((outer + 3) / 4, 4096);
    if (is_min) hipLaunchKernelGGL((argreduce_row<T, O, true>), dim3(grid), dim3(256), 0, s, x, y, outer, r);
    else hipLaunchKernelGGL((argreduce_row<T, O, false>), dim3(grid), dim3(256), 0, s, x, y, outer, r);
  } else {
    int64_t n = outer * inner;
    if (is_min) hipLaunchKernelGGL((argreduce_col<T, O, true>), dim3(ew_grid(n)), dim3(256), 0, s, x, y, outer, r, inner);
    else hipLaunchKernelGGL((argreduce_col<T, O, false>), dim3(ew_grid(n)), dim3(256), 0, s, x, y, outer, r, inner);
  }
}

// ---- softmax (wave per row, 3 passes over an L2-resident row)
template <typename T, bool LOG>
__global__ __launch_bounds__(256) void softmax_rows(const T* __restrict__ x, T* __restrict__ y,
                                                    int64_t rows, int64_t cols) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += waves) {
    const T* p = x + row * cols;
    T* q = y + row * cols;
    T m = -INFINITY;
    for (int64_t i = lane; i < cols; i += 64) m = p[i] > m ? p[i] : m;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      T o = __shfl_xor(m, off, 64);
      m = o > m ? o : m;
    }
    T sum = 0;
    for (int64_t i = lane; i < cols; i += 64) sum += exp(p[i] - m);
    sum = wave_sum(sum);
    if (LOG) {
      T ls = log(sum);
      for (int64_t i = lane; i < cols; i += 64) q[i] = p[i] - m - ls;
    } else {
      T inv = T(1) / sum;
      for (int64_t i = lane; i < cols; i += 64) q[i] = exp(p[i] - m) * inv;
    }
  }
}

// ---- top-k: wave per row, k selection rounds ordered (value desc, index asc)
template <typename T>
__global__ __launch_bounds__(256) void topk_rows(const T* __restrict__ x, T* __restrict__ vals,
                                                 int32_t* __restrict__ idx, int64_t rows, int64_t cols,
                                                 int kk) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += waves) {
    const T* p = x + row * cols;
    T pv = 0;
    int64_t pi = -1;
    for (int j = 0; j < kk; ++j) {
      bool have = false;
      T bv = 0;
      int64_t bi = INT64_MAX;
      for (int64_t i = lane; i < cols; i += 64) {
        T v = p[i];
        // eligible: strictly after the previous pick in (value desc, index asc) order
        bool elig = pi < 0 || v < pv || (v == pv && i > pi);
        if (elig && (!have || v > bv || (v == bv && i < bi))) {
          have = true;
          bv = v;
          bi = i;
        }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        T ov = __shfl_xor(bv, off, 64);
        int64_t oi = __shfl_xor(bi, off, 64);
        int oh = __shfl_xor((int)have, off, 64);
        if (oh && (!have || ov > bv || (ov == bv && oi < bi))) {
          have = true;
          bv = ov;
          bi = oi;
        }
      }
      pv = bv;
      pi = bi;
      if (lane == 0) {
        vals[row * kk + j] = bv;
        idx[row * kk + j] = (int32_t)bi;
      }
    }
  }
}

// ---- unsorted segment reduce, deterministic LDS-private path.
// grid = (B row-blocks, col tiles); blockDim = TILE (one thread per column);
// each block folds its rows in order into LDS acc[seg][col], writes its slab.
template <typename T, typename I, int OP>
__global__ __launch_bounds__(256) void useg_private(const T* __restrict__ x, const I* __restrict__ ids,
                                                    typename AccT<T>::type* __restrict__ part,
                                                    int64_t n, int64_t inner, int64_t nseg,
                                                    int64_t rows_per_block) {
  using A = typename AccT<T>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  A* acc = reinterpret_cast<A*>(smem);
  const int tile = blockDim.x;
  const int64_t col = (int64_t)blockIdx.y * tile + threadIdx.x;
  for (int64_t sgi = 0; sgi < nseg; ++sgi) acc[sgi * tile + threadIdx.x] = ident<OP, A>();
  const int64_t r0 = blockIdx.x * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  if (col < inner) {
    // 8 rows of ids and values are loaded before they are folded, so the
    // global loads overlap instead of one latency per row; the fold itself
    // keeps the row order (deterministic)
    constexpr int U = 8;
    for (int64_t i = r0; i < r1; i += U) {
      int64_t sg[U];
      A v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = i + u < r1;
        sg[u] = ok ? (int64_t)ids[i + u] : -1;
        v[u] = ok ? A(x[(i + u) * inner + col]) : A(0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (sg[u] < 0 || sg[u] >= nseg) continue;
        A* a = &acc[sg[u] * tile + threadIdx.x];
        *a = combine<OP, A>(*a, v[u]);
      }
    }
    for (int64_t sgi = 0; sgi < nseg; ++sgi)
      part[((int64_t)blockIdx.x * nseg + sgi) * inner + col] = acc[sgi * tile + threadIdx.x];
  }
}

// folds the B partial slabs: a group of G lanes (G = pow2 <= 64) per output
// element strides over the slabs, then a fixed xor tree (deterministic)
template <typename T, int OP>
__global__ __launch_bounds__(256) void useg_final(const typename AccT<T>::type* __restrict__ part,
                                                  T* __restrict__ y, int64_t m, int64_t B, int G) {
  using A = typename AccT<T>::type;
  const int lane = threadIdx.x & 63;
  const int sub = lane % G;
  const int per_wave = 64 / G;
  const int64_t waves = (int64_t)gridDim.x * 4;
  for (int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * per_wave; base < m; base += waves * per_wave) {
    const int64_t i = base + lane / G;
    A acc = ident<OP, A>();
    if (i < m) {
      // 8 slabs' loads in flight per lane, folded in slab order (the same
      // order as one at a time: deterministic, bit-identical)
      constexpr int R = 8;
      for (int64_t b0 = sub; b0 < B; b0 += (int64_t)R * G) {
        A t[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int64_t b = b0 + (int64_t)r * G;
          t[r] = b < B ? part[b * m + i] : ident<OP, A>();
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (b0 + (int64_t)r * G < B) acc = combine<OP, A>(acc, t[r]);  // no padding term (-0.0 stays -0.0)
      }
    }
    for (int s = G / 2; s >= 1; s >>= 1) acc = combine<OP, A>(acc, __shfl_xor(acc, s, 64));
    if (i >= m || sub != 0) continue;
    if constexpr (OP == (int)RedOp::MIN || OP == (int)RedOp::MAX) {
      // TF: empty segments get the type's lowest (max) / highest (min) value
      if (acc == ident<OP, A>()) {
        if constexpr (std::is_floating_point<T>::value)
          acc = OP == (int)RedOp::MAX ? A(-std::numeric_limits<T>::max()) : A(std::numeric_limits<T>::max());
        else
          acc = OP == (int)RedOp::MAX ? A(std::numeric_limits<T>::lowest()) : A(std::numeric_limits<T>::max());
      }
    }
    y[i] = T(acc);
  }
}

// ---- CSR segment reduce over sorted rows: grid = (nseg, col tiles)
template <typename T, int OP>
__global__ __launch_bounds__(256) void seg_csr(const T* __restrict__ x, const int64_t* __restrict__ off,
                                               T* __restrict__ y, int64_t nseg, int64_t inner) {
  using A = typename AccT<T>::type;
  const int64_t sg = blockIdx.x;
  const int64_t col = (int64_t)blockIdx.y * blockDim.x + threadIdx.x;
  if (col >= inner) return;
  A acc = ident<OP, A>();
  for (int64_t i = off[sg]; i < off[sg + 1]; ++i) acc = combine<OP, A>(acc, A(x[i * inner + col]));
  y[sg * inner + col] = finish<OP, T, A>(acc, off[sg + 1] - off[sg]);
}

// ---- segment reduce over permuted rows: segment g = rows perm[off[g] .. off[g+1]),
// one wave per segment; for inner <= 64 the wave reads 64/inner_pad rows at
// once (lane = row slot x column) and folds them with a fixed xor tree
// (deterministic); wider rows loop over 64-column chunks
// TF: an empty segment of a Min/Max gets the type's highest / lowest value
template <typename T, int OP, typename A>
__device__ __forceinline__ T seg_empty_or(A acc, int64_t count) {
  if constexpr (OP == (int)RedOp::MIN || OP == (int)RedOp::MAX) {
    if (count == 0) {
      if constexpr (std::is_floating_point<T>::value)
        return OP == (int)RedOp::MAX ? -std::numeric_limits<T>::max() : std::numeric_limits<T>::max();
      else
        return OP == (int)RedOp::MAX ? std::numeric_limits<T>::lowest() : std::numeric_limits<T>::max();
    }
  }
  return finish<OP, T, A>(acc, count);
}

template <typename T, int OP>
__global__ __launch_bounds__(256) void seg_perm(const T* __restrict__ x, const int64_t* __restrict__ perm,
                                                const int64_t* __restrict__ off, T* __restrict__ y, int64_t nseg,
                                                int64_t inner, int inner_pad) {
  using A = typename AccT<T>::type;
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= nseg) return;  // the whole wave leaves together
  const int64_t b = off[g], e = off[g + 1];
  if (inner <= 64) {
    const int c = lane % inner_pad, rs = lane / inner_pad, R = 64 / inner_pad;
    A acc = ident<OP, A>();
    if (c < inner)
      for (int64_t j = b + rs; j < e; j += R) acc = combine<OP, A>(acc, A(x[perm[j] * inner + c]));
    for (int s = 32; s >= inner_pad; s >>= 1) acc = combine<OP, A>(acc, __shfl_xor(acc, s, 64));
    if (rs == 0 && c < inner) y[g * inner + c] = seg_empty_or<T, OP, A>(acc, e - b);
  } else {
    for (int64_t c = lane; c < inner; c += 64) {
      A acc = ident<OP, A>();
      for (int64_t j = b; j < e; ++j) acc = combine<OP, A>(acc, A(x[perm[j] * inner + c]));
      y[g * inner + c] = seg_empty_or<T, OP, A>(acc, e - b);
    }
  }
}

constexpr int64_t kUsegTile = 256;
constexpr int64_t kUsegLds = 64 * 1024;

int64_t useg_tile(int64_t inner) {
  int64_t t = ((inner + 63) / 64) * 64;
  return std::min<int64_t>(t, kUsegTile);
}

// row blocks of the LDS-private pass: at least 4 rows per segment and 32 per
// block, so the partial slabs (B x nseg x inner) stay well below the input
// they summarise; at most 8192 blocks and 256 MB of slabs
int64_t useg_rows_per_block(int64_t n, int64_t nseg, int64_t inner) {
  int64_t rpb = std::max<int64_t>(32, 4 * nseg);
  rpb = std::max<int64_t>(rpb, (n + 8191) / 8192);
  const int64_t max_blocks = std::max<int64_t>(1, (int64_t(256) << 20) / std::max<int64_t>(1, nseg * inner * 8));
  rpb = std::max<int64_t>(rpb, (n + max_blocks - 1) / max_blocks);
  return (rpb + 7) / 8 * 8;
}

int64_t useg_blocks(int64_t n, int64_t nseg, int64_t inner) {
  const int64_t rpb = useg_rows_per_block(n, nseg, inner);
  return std::max<int64_t>(1, (n + rpb - 1) / rpb);
}

}  // namespace

// ====================================================================== host API
size_t reduce_workspace_bytes(DType dt, int64_t outer, int64_t r, int64_t inner) {
  int64_t S = 1;
  switch (dt) {
    case DType::F32: { auto p = plan_reduce<float>(outer, r, inner); S = p.row_wave ? 1 : p.S; break; }
    case DType::F64: { auto p = plan_reduce<double>(outer, r, inner); S = p.row_wave ? 1 : p.S; break; }
    case DType::I32: { auto p = plan_reduce<int32_t>(outer, r, inner); S = p.row_wave ? 1 : p.S; break; }
    case DType::I64: { auto p = plan_reduce<int64_t>(outer, r, inner); S = p.row_wave ? 1 : p.S; break; }
    case DType::BOOL: { auto p = plan_reduce<uint8_t>(outer, r, inner); S = p.row_wave ? 1 : p.S; break; }
    default: return 0;
  }
  if (S <= 1) return 0;
  // accumulators are 8 bytes: S partial slabs + the folded ones
  return static_cast<size_t>(S + fold_slabs(S)) * outer * inner * 8;
}

void reduce(RedOp op, DType dt, const void* x, void* y, int64_t outer, int64_t r, int64_t inner,
            void* workspace, hipStream_t s) {
  if (outer * inner <= 0) return;
  TFA_CHECK(r > 0, "reduce: empty reduction handled by caller");
  switch (dt) {
    case DType::F32: reduce_dispatch_op<float>(op, x, y, outer, r, inner, workspace, s); break;
    case DType::F64: reduce_dispatch_op<double>(op, x, y, outer, r, inner, workspace, s); break;
    case DType::I32: reduce_dispatch_op<int32_t>(op, x, y, outer, r, inner, workspace, s); break;
    case DType::I64: reduce_dispatch_op<int64_t>(op, x, y, outer, r, inner, workspace, s); break;
    case DType::BOOL:
      if (op == RedOp::ALL) reduce_typed<uint8_t, (int)RedOp::ALL>(x, y, outer, r, inner, workspace, s);
      else if (op == RedOp::ANY) reduce_typed<uint8_t, (int)RedOp::ANY>(x, y, outer, r, inner, workspace, s);
      else TFA_CHECK(false, "reduce: only All/Any on bool");
      break;
    default: TFA_CHECK(false, "reduce: dtype ", dtype_name(dt), " not supported");
  }
  TFA_LAUNCH_CHECK("reduce");
}

void argreduce(bool is_min, DType dt, DType out_dt, const void* x, void* y, int64_t outer, int64_t r,
               int64_t inner, hipStream_t s) {
  if (outer * inner <= 0) return;
  TFA_CHECK(r > 0, "argreduce over an empty axis");
  TFA_CHECK(out_dt == DType::I32 || out_dt == DType::I64, "argreduce: output must be int32/int64");
  bool o64 = out_dt == DType::I64;
  switch (dt) {
    case DType::F32: o64 ? argreduce_typed<float, int64_t>(is_min, x, y, outer, r, inner, s) : argreduce_typed<float, int32_t>(is_min, x, y, outer, r, inner, s); break;
    case DType::F64: o64 ? argreduce_typed<double, int64_t>(is_min, x, y, outer, r, inner, s) : argreduce_typed<double, int32_t>(is_min, x, y, outer, r, inner, s); break;
    case DType::I32: o64 ? argreduce_typed<int32_t, int64_t>(is_min, x, y, outer, r, inner, s) : argreduce_typed<int32_t, int32_t>(is_min, x, y, outer, r, inner, s); break;
    case DType::I64: o64 ? argreduce_typed<int64_t, int64_t>(is_min, x, y, outer, r, inner, s) : argreduce_typed<int64_t, int32_t>(is_min, x, y, outer, r, inner, s); break;
    default: TFA_CHECK(false, "argreduce: dtype ", dtype_name(dt), " not supported");
  }
  TFA_LAUNCH_CHECK("argreduce");
}

void softmax(DType dt, bool log, const void* x, void* y, int64_t rows, int64_t cols, hipStream_t s) {
  if (rows * cols <= 0) return;
  int grid = (int)std::min<int64_t>((rows + 3) / 4, 8192);
  if (dt == DType::F32) {
    if (log) hipLaunchKernelGGL((softmax_rows<float, true>), dim3(grid), dim3(256), 0, s, (const float*)x, (float*)y, rows, cols);
    else hipLaunchKernelGGL((softmax_rows<float, false>), dim3(grid), dim3(256), 0, s, (const float*)x, (float*)y, rows, cols);
  } else if (dt == DType::F64) {
    if (log) hipLaunchKernelGGL((softmax_rows<double, true>), dim3(grid), dim3(256), 0, s, (const double*)x, (double*)y, rows, cols);
    else hipLaunchKernelGGL((softmax_rows<double, false>), dim3(grid), dim3(256), 0, s, (const double*)x, (double*)y, rows, cols);
  } else {
    TFA_CHECK(false, "softmax: float types only");
  }
  TFA_LAUNCH_CHECK("softmax");
}

void topk(DType dt, const void* x, void* vals, int32_t* idx, int64_t rows, int64_t cols, int kk,
          hipStream_t s) {
  if (rows <= 0 || kk <= 0) return;
  TFA_CHECK(kk <= cols, "topk: k > cols");
  int grid = (int)std::min<int64_t>((rows + 3) / 4, 8192);
  switch (dt) {
    case DType::F32: hipLaunchKernelGGL((topk_rows<float>), dim3(grid), dim3(256), 0, s, (const float*)x, (float*)vals, idx, rows, cols, kk); break;
    case DType::F64: hipLaunchKernelGGL((topk_rows<double>), dim3(grid), dim3(256), 0, s, (const double*)x, (double*)vals, idx, rows, cols, kk); break;
    case DType::I32: hipLaunchKernelGGL((topk_rows<int32_t>), dim3(grid), dim3(256), 0, s, (const int32_t*)x, (int32_t*)vals, idx, rows, cols, kk); break;
    case DType::I64: hipLaunchKernelGGL((topk_rows<int64_t>), dim3(grid), dim3(256), 0, s, (const int64_t*)x, (int64_t*)vals, idx, rows, cols, kk); break;
    default: TFA_CHECK(false, "topk: dtype not supported");
  }
  TFA_LAUNCH_CHECK("topk");
}

// many segments (the LDS-private histograms do not fit): rows are ordered by
// segment with one radix sort (groupby.hip) and reduced per segment
static bool useg_fits_lds(int64_t inner, int64_t nseg) {
  return static_cast<size_t>(nseg * useg_tile(inner) * 8) <= static_cast<size_t>(kUsegLds);
}

static size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

size_t unsorted_segment_workspace_bytes(RedOp, DType, int64_t n, int64_t inner, int64_t nseg) {
  if (useg_fits_lds(inner, nseg)) return static_cast<size_t>(useg_blocks(n, nseg, inner)) * nseg * inner * 8;
  return align256(n * 8) + align256((nseg + 1) * 8) + segment_csr_workspace_bytes(n, nseg);
}

template <typename T>
static void seg_perm_op(RedOp op, const void* x, const int64_t* perm, const int64_t* off, void* y, int64_t nseg,
                        int64_t inner, hipStream_t s) {
  int inner_pad = 1;
  while (inner_pad < inner && inner_pad < 64) inner_pad <<= 1;
  dim3 grid((unsigned)((nseg + 3) / 4));
  switch (op) {
#define TFA_SP(OPV) hipLaunchKernelGGL((seg_perm<T, (int)OPV>), grid, dim3(256), 0, s, (const T*)x, perm, off, (T*)y, nseg, inner, inner_pad); break;
    case RedOp::SUM: TFA_SP(RedOp::SUM)
    case RedOp::PROD: TFA_SP(RedOp::PROD)
    case RedOp::MIN: TFA_SP(RedOp::MIN)
    case RedOp::MAX: TFA_SP(RedOp::MAX)
    case RedOp::MEAN: TFA_SP(RedOp::MEAN)
#undef TFA_SP
    default: TFA_CHECK(false, "segment reduce: unsupported op");
  }
}

void segment_reduce_perm(RedOp op, DType dt, const void* x, const int64_t* perm, const int64_t* offsets, void* y,
                         int64_t nseg, int64_t inner, hipStream_t s) {
  if (nseg * inner <= 0) return;
  TFA_CHECK((nseg + 3) / 4 <= 0x7fffffff, "segment reduce: too many segments");
  switch (dt) {
    case DType::F32: seg_perm_op<float>(op, x, perm, offsets, y, nseg, inner, s); break;
    case DType::F64: seg_perm_op<double>(op, x, perm, offsets, y, nseg, inner, s); break;
    case DType::I32: seg_perm_op<int32_t>(op, x, perm, offsets, y, nseg, inner, s); break;
    case DType::I64: seg_perm_op<int64_t>(op, x, perm, offsets, y, nseg, inner, s); break;
    default: TFA_CHECK(false, "segment reduce: dtype not supported");
  }
  TFA_LAUNCH_CHECK("segment_reduce_perm");
}

// ---- small integer segment reduce (inner == 1): one 1024-thread block folds
// every row into an LDS table with integer atomics (exact, so the order does
// not matter) -- one launch instead of private slabs plus a final pass (the
// per-cluster counts of K-Means)
constexpr int64_t kUsegSmallRows = 1 << 18;
constexpr int64_t kUsegSmallSegs = 4096;
template <typename T, typename I, int OP>
__global__ __launch_bounds__(1024) void useg_small_int(const T* __restrict__ x, const I* __restrict__ ids,
                                                       T* __restrict__ y, int64_t n, int64_t nseg) {
  __shared__ long long acc[kUsegSmallSegs];
  for (int64_t g = threadIdx.x; g < nseg; g += 1024) acc[g] = ident<OP, long long>();
  __syncthreads();
  // 8 rows of ids and values in flight per thread (latency, as above)
  constexpr int U = 8;
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += U * 1024) {
    int64_t g[U];
    long long v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * 1024;
      const bool ok = i < n;
      g[u] = ok ? (int64_t)ids[i] : -1;
      v[u] = ok ? (long long)x[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (g[u] < 0 || g[u] >= nseg) continue;
      if constexpr (OP == (int)RedOp::SUM)
        atomicAdd(reinterpret_cast<unsigned long long*>(&acc[g[u]]), (unsigned long long)v[u]);
      else if constexpr (OP == (int)RedOp::MIN) atomicMin(&acc[g[u]], v[u]);
      else atomicMax(&acc[g[u]], v[u]);
    }
  }
  __syncthreads();
  for (int64_t g = threadIdx.x; g < nseg; g += 1024) {
    long long a = acc[g];
    if constexpr (OP == (int)RedOp::MIN || OP == (int)RedOp::MAX) {
      // TF: empty segments get the type's highest (min) / lowest (max) value
      if (a == ident<OP, long long>())
        a = OP == (int)RedOp::MAX ? (long long)std::numeric_limits<T>::lowest() : (long long)std::numeric_limits<T>::max();
    }
    y[g] = T(a);
  }
}

// ---- very few segments (nseg <= 16, inner == 1, integer data): each thread
// keeps one accumulator per segment in registers (compile-time indexed: a
// compare-select per segment and row, no LDS atomics, no contention), then a
// wave reduction and one LDS slot per wave and segment. Many blocks of 1024
// rows each write one partial row [nseg]; one wave folds the partials in block
// order (integers: exact). The K-Means counts (k = 10 clusters, 25k rows per
// partition) are this shape: a single 1024-thread block took 23.5 us of
// compare-selects on one CU (profiles/r4_kmeans/kernel_stats.csv).
constexpr int kUsegRegSegs = 16;
constexpr int kUsegTinyThreads = 256, kUsegTinyU = 4;
constexpr int64_t kUsegTinyRows = kUsegTinyThreads * kUsegTinyU;  // rows per block
template <typename T, typename I, int OP>
__global__ __launch_bounds__(kUsegTinyThreads) void useg_tiny_int(const T* __restrict__ x, const I* __restrict__ ids,
                                                                  long long* __restrict__ part, int64_t n, int nseg) {
  // per-thread histograms, then transposed through LDS: wave w folds
  // segments w, w+4, ... (4 values per lane, one wave reduction per segment)
  // instead of every wave reducing every segment
  __shared__ long long tab[kUsegRegSegs][kUsegTinyThreads];
  long long acc[kUsegRegSegs];
#pragma unroll
  for (int g = 0; g < kUsegRegSegs; ++g) acc[g] = ident<OP, long long>();
  const int64_t i0 = (int64_t)blockIdx.x * kUsegTinyRows + threadIdx.x;
  int64_t gv[kUsegTinyU];
  long long v[kUsegTinyU];
#pragma unroll
  for (int u = 0; u < kUsegTinyU; ++u) {
    const int64_t i = i0 + u * kUsegTinyThreads;
    const bool ok = i < n;
    gv[u] = ok ? (int64_t)ids[i] : -1;
    v[u] = ok ? (long long)x[i] : 0;
  }
#pragma unroll
  for (int u = 0; u < kUsegTinyU; ++u)
#pragma unroll
    for (int g = 0; g < kUsegRegSegs; ++g)
      if (gv[u] == g) acc[g] = combine<OP, long long>(acc[g], v[u]);
#pragma unroll
  for (int g = 0; g < kUsegRegSegs; ++g)
    if (g < nseg) tab[g][threadIdx.x] = acc[g];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int g = wave; g < nseg; g += kUsegTinyThreads / 64) {
    long long a = tab[g][lane];
#pragma unroll
    for (int q = 1; q < kUsegTinyThreads / 64; ++q) a = combine<OP, long long>(a, tab[g][lane + 64 * q]);
    a = wave_reduce<OP, long long>(a);
    if (lane == 0) part[(int64_t)blockIdx.x * nseg + g] = a;
  }
}

// one wave folds the B partial rows [B][nseg] in block order: the loads of
// 8 rows are in flight together (a dependent load per row took ~6 us)
template <typename T, int OP>
__global__ __launch_bounds__(64) void useg_tiny_final(const long long* __restrict__ part, T* __restrict__ y, int64_t B,
                                                      int nseg) {
  const int g = threadIdx.x;
  if (g >= nseg) return;
  long long a = ident<OP, long long>();
  constexpr int R = 8;
  for (int64_t b0 = 0; b0 < B; b0 += R) {
    long long t[R];
#pragma unroll
    for (int r = 0; r < R; ++r) t[r] = b0 + r < B ? part[(b0 + r) * nseg + g] : ident<OP, long long>();
#pragma unroll
    for (int r = 0; r < R; ++r) a = combine<OP, long long>(a, t[r]);
  }
  if constexpr (OP == (int)RedOp::MIN || OP == (int)RedOp::MAX) {
    // TF: empty segments get the type's highest (min) / lowest (max) value
    if (a == ident<OP, long long>())
      a = OP == (int)RedOp::MAX ? (long long)std::numeric_limits<T>::lowest() : (long long)std::numeric_limits<T>::max();
  }
  y[g] = T(a);
}

template <typename T, typename I, int OP>
static void useg_typed(const void* x, const void* ids, void* y, int64_t n, int64_t inner, int64_t nseg,
                       void* ws, hipStream_t s) {
  using A = typename AccT<T>::type;
  if constexpr (std::is_integral<T>::value && OP != (int)RedOp::PROD) {
    if (inner == 1 && n <= kUsegSmallRows && nseg <= kUsegRegSegs) {
      // partials: B x nseg 8-byte values, within the workspace of the
      // LDS-private pass (B <= n / 1024 <= useg_blocks(n, nseg, 1))
      const int64_t B = (n + kUsegTinyRows - 1) / kUsegTinyRows;
      long long* part = static_cast<long long*>(ws);
      hipLaunchKernelGGL((useg_tiny_int<T, I, OP>), dim3((unsigned)B), dim3(kUsegTinyThreads), 0, s, (const T*)x,
                         (const I*)ids, part, n, (int)nseg);
      hipLaunchKernelGGL((useg_tiny_final<T, OP>), dim3(1), dim3(64), 0, s, (const long long*)part, (T*)y, B,
                         (int)nseg);
      return;
    }
    if (inner == 1 && n <= kUsegSmallRows && nseg <= kUsegSmallSegs) {
      hipLaunchKernelGGL((useg_small_int<T, I, OP>), dim3(1), dim3(1024), 0, s, (const T*)x, (const I*)ids, (T*)y, n,
                         nseg);
      return;
    }
  }
  int64_t tile = useg_tile(inner);
  size_t lds = static_cast<size_t>(nseg * tile * sizeof(A));
  TFA_CHECK(lds <= kUsegLds, "unsorted segment reduce: ", nseg, " segments x ", tile,
            " columns exceed the LDS budget");
  const int64_t rpb = useg_rows_per_block(n, nseg, inner);
  const int64_t B = useg_blocks(n, nseg, inner);
  dim3 grid((unsigned)B, (unsigned)((inner + tile - 1) / tile));
  hipLaunchKernelGGL((useg_private<T, I, OP>), grid, dim3((unsigned)tile), lds, s, (const T*)x, (const I*)ids,
                     (A*)ws, n, inner, nseg, rpb);
  const int64_t m = nseg * inner;
  int G = 1;
  while (G < 64 && G < B) G <<= 1;
  const int64_t groups = (m + 64 / G - 1) / (64 / G);  // waves
  const unsigned fgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((groups + 3) / 4, 65536));
  hipLaunchKernelGGL((useg_final<T, OP>), dim3(fgrid), dim3(256), 0, s, (const A*)ws, (T*)y, m, B, G);
}

template <typename T, typename I>
static void useg_op(RedOp op, const void* x, const void* ids, void* y, int64_t n, int64_t inner,
                    int64_t nseg, void* ws, hipStream_t s) {
  switch (op) {
    case RedOp::SUM: useg_typed<T, I, (int)RedOp::SUM>(x, ids, y, n, inner, nseg, ws, s); break;
    case RedOp::PROD: useg_typed<T, I, (int)RedOp::PROD>(x, ids, y, n, inner, nseg, ws, s); break;
    case RedOp::MIN: useg_typed<T, I, (int)RedOp::MIN>(x, ids, y, n, inner, nseg, ws, s); break;
    case RedOp::MAX: useg_typed<T, I, (int)RedOp::MAX>(x, ids, y, n, inner, nseg, ws, s); break;
    default: TFA_CHECK(false, "unsorted segment reduce: unsupported op");
  }
}

void unsorted_segment_reduce(RedOp op, DType dt, DType idt, const void* x, const void* ids, void* y,
                             int64_t n, int64_t inner, int64_t nseg, void* workspace, hipStream_t s) {
  if (nseg * inner <= 0) return;
  if (n == 0) {
    double v = (op == RedOp::PROD) ? 1.0 : 0.0;
    fill(dt, y, nseg * inner, v, s);
    return;
  }
  TFA_CHECK(workspace != nullptr, "unsorted segment reduce: missing workspace");
  TFA_CHECK(idt == DType::I32 || idt == DType::I64, "segment ids must be int32/int64");
  if (!useg_fits_lds(inner, nseg)) {
    char* p = static_cast<char*>(workspace);
    int64_t* perm = reinterpret_cast<int64_t*>(p);
    int64_t* off = reinterpret_cast<int64_t*>(p + align256(n * 8));
    void* rest = p + align256(n * 8) + align256((nseg + 1) * 8);
    segment_csr(idt, ids, n, nseg, perm, off, rest, segment_csr_workspace_bytes(n, nseg), s);
    segment_reduce_perm(op, dt, x, perm, off, y, nseg, inner, s);
    return;
  }
  bool i64 = idt == DType::I64;
  switch (dt) {
    case DType::F32: i64 ? useg_op<float, int64_t>(op, x, ids, y, n, inner, nseg, workspace, s) : useg_op<float, int32_t>(op, x, ids, y, n, inner, nseg, workspace, s); break;
    case DType::F64: i64 ? useg_op<double, int64_t>(op, x, ids, y, n, inner, nseg, workspace, s) : useg_op<double, int32_t>(op, x, ids, y, n, inner, nseg, workspace, s); break;
    case DType::I32: i64 ? useg_op<int32_t, int64_t>(op, x, ids, y, n, inner, nseg, workspace, s) : useg_op<int32_t, int32_t>(op, x, ids, y, n, inner, nseg, workspace, s); break;
    case DType::I64: i64 ? useg_op<int64_t, int64_t>(op, x, ids, y, n, inner, nseg, workspace, s) : useg_op<int64_t, int32_t>(op, x, ids, y, n, inner, nseg, workspace, s); break;
    default: TFA_CHECK(false, "unsorted segment reduce: dtype not supported");
  }
  TFA_LAUNCH_CHECK("unsorted_segment_reduce");
}

template <typename T>
static void seg_csr_op(RedOp op, const void* x, const int64_t* off, void* y, int64_t nseg, int64_t inner,
                       hipStream_t s) {
  dim3 grid((unsigned)nseg, (unsigned)((inner + 255) / 256));
  unsigned bs = (unsigned)std::min<int64_t>(256, ((inner + 63) / 64) * 64);
  switch (op) {
    case RedOp::SUM: hipLaunchKernelGGL((seg_csr<T, (int)RedOp::SUM>), grid, dim3(bs), 0, s, (const T*)x, off, (T*)y, nseg, inner); break;
    case RedOp::PROD: hipLaunchKernelGGL((seg_csr<T, (int)RedOp::PROD>), grid, dim3(bs), 0, s, (const T*)x, off, (T*)y, nseg, inner); break;
    case RedOp::MIN: hipLaunchKernelGGL((seg_csr<T, (int)RedOp::MIN>), grid, dim3(bs), 0, s, (const T*)x, off, (T*)y, nseg, inner); break;
    case RedOp::MAX: hipLaunchKernelGGL((seg_csr<T, (int)RedOp::MAX>), grid, dim3(bs), 0, s, (const T*)x, off, (T*)y, nseg, inner); break;
    case RedOp::MEAN: hipLaunchKernelGGL((seg_csr<T, (int)RedOp::MEAN>), grid, dim3(bs), 0, s, (const T*)x, off, (T*)y, nseg, inner); break;
    default: TFA_CHECK(false, "segment reduce: unsupported op");
  }
}

void segment_reduce_csr(RedOp op, DType dt, const void* x, const int64_t* offsets, void* y, int64_t nseg,
                        int64_t inner, hipStream_t s) {
  if (nseg * inner <= 0) return;
  TFA_CHECK(nseg <= 0x7fffffff, "segment reduce: too many segments");
  switch (dt) {
    case DType::F32: seg_csr_op<float>(op, x, offsets, y, nseg, inner, s); break;
    case DType::F64: seg_csr_op<double>(op, x, offsets, y, nseg, inner, s); break;
    case DType::I32: seg_csr_op<int32_t>(op, x, offsets, y, nseg, inner, s); break;
    case DType::I64: seg_csr_op<int64_t>(op, x, offsets, y, nseg, inner, s); break;
    default: TFA_CHECK(false, "segment reduce: dtype not supported");
  }
  TFA_LAUNCH_CHECK("segment_reduce_csr");
}

}  // namespace k
}  // namespace tfa

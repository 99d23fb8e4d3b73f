// MFMA GEMM + implicit-GEMM Conv2D + pooling for gfx950 (CDNA4).
//
// f32: v_mfma_f32_32x32x2_f32 (exact f32, no xf32 on gfx950). 128x128x16
//      block tile, 4 waves as 2x2, each wave 64x64 = 2x2 MFMA tiles of 32x32.
// f64: v_mfma_f64_16x16x4_f64. 64x64x16 block tile, 4 waves as 2x2, each
//      wave 32x32 = 2x2 MFMA tiles of 16x16 (f64 has its own C/D layout).
// Both: k-major LDS images (As[k][m], Bs[k][n]) so every MFMA operand read is
// 32 consecutive floats per half-wave (conflict-free ds_read_b32), two LDS
// stages with the next tile's global loads issued before the current tile's
// MFMAs (register-staged pipeline, one barrier per K tile), bias + ReLU fused
// into the epilogue, XCD-aware bijective block->tile remap so that blocks that
// share an A row-panel run on one XCD (shared L2).
// Conv2D (NHWC, filter HWIO) reuses the f32 core with an im2col-on-the-fly A
// loader: A[m = (n,oh,ow)][k = (kh,kw,c)], B = filter viewed as [KH*KW*C, OC].
#include <cmath>

#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  // bijective: blocks with equal b % 8 (same XCD under round-robin dispatch)
  // get a contiguous range of logical tile ids
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

template <typename T>
__device__ __forceinline__ T act_apply(T v, int act) {
  if (act == 1) return v > T(0) ? v : T(0);
  if (act == 2) return v > T(0) ? (v < T(6) ? v : T(6)) : T(0);
  return v;
}

enum ALoad { A_KCONTIG = 0, A_MCONTIG = 1, A_CONV = 2 };

struct ConvGeom {
  int H, W, C, KW, OH, OW, sh, sw, dh, dw, pt, pl;
};

// ============================================================== f32 core
constexpr int F_BM = 128, F_BN = 128, F_BK = 16, F_PAD = 4;
constexpr int F_LDS = F_BM + F_PAD;  // == F_BN + F_PAD

struct F32Regs {
  float a[2][4];
  float b[2][4];
};

template <int AL, bool TB, bool VEC>
__device__ __forceinline__ void f32_load_tile(F32Regs& R, const float* __restrict__ A,
                                              const float* __restrict__ B, int64_t lda, int64_t ldb,
                                              int64_t M, int64_t N, int64_t K, int64_t m0, int64_t n0,
                                              int64_t k0, int tid, const ConvGeom& cg,
                                              const int64_t* conv_base, const int* conv_ih,
                                              const int* conv_iw) {
  // ---- A tile (BM x BK)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int idx = tid + 256 * p;
    if (AL == A_KCONTIG || AL == A_CONV) {
      const int row = idx >> 2, kq = idx & 3;
      const int64_t gm = m0 + row, gk = k0 + 4 * kq;
      if (AL == A_KCONTIG) {
        const float* src = A + gm * lda + gk;
        if (VEC && gm < M && gk < K) {
          float4 v = *reinterpret_cast<const float4*>(src);
          R.a[p][0] = v.x; R.a[p][1] = v.y; R.a[p][2] = v.z; R.a[p][3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) R.a[p][j] = (gm < M && gk + j < K) ? src[j] : 0.f;
        }
      } else {
        // implicit im2col: k = (kh*KW + kw)*C + c
        if (VEC) {  // C % 4 == 0: the 4 k's share (kh, kw)
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (conv_base[p] >= 0 && gk < K) {
            const int c = (int)(gk % cg.C);
            const int t = (int)(gk / cg.C);
            const int kw = t % cg.KW, kh = t / cg.KW;
            const int ih = conv_ih[p] + kh * cg.dh, iw = conv_iw[p] + kw * cg.dw;
            if (ih >= 0 && ih < cg.H && iw >= 0 && iw < cg.W)
              v = *reinterpret_cast<const float4*>(A + conv_base[p] + ((int64_t)ih * cg.W + iw) * cg.C + c);
          }
          R.a[p][0] = v.x; R.a[p][1] = v.y; R.a[p][2] = v.z; R.a[p][3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = 0.f;
            const int64_t kk = gk + j;
            if (conv_base[p] >= 0 && kk < K) {
              const int c = (int)(kk % cg.C);
              const int t = (int)(kk / cg.C);
              const int kw = t % cg.KW, kh = t / cg.KW;
              const int ih = conv_ih[p] + kh * cg.dh, iw = conv_iw[p] + kw * cg.dw;
              if (ih >= 0 && ih < cg.H && iw >= 0 && iw < cg.W)
                v = A[conv_base[p] + ((int64_t)ih * cg.W + iw) * cg.C + c];
            }
            R.a[p][j] = v;
          }
        }
      }
    } else {  // A_MCONTIG: A stored [K][M]
      const int kr = idx >> 5, mq = idx & 31;
      const int64_t gk = k0 + kr, gm = m0 + 4 * mq;
      const float* src = A + gk * lda + gm;
      if (VEC && gk < K && gm + 3 < M) {
        float4 v = *reinterpret_cast<const float4*>(src);
        R.a[p][0] = v.x; R.a[p][1] = v.y; R.a[p][2] = v.z; R.a[p][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) R.a[p][j] = (gk < K && gm + j < M) ? src[j] : 0.f;
      }
    }
  }
  // ---- B tile (BK x BN)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int idx = tid + 256 * p;
    if (!TB) {  // B stored [K][N]
      const int kr = idx >> 5, nq = idx & 31;
      const int64_t gk = k0 + kr, gn = n0 + 4 * nq;
      const float* src = B + gk * ldb + gn;
      if (VEC && gk < K && gn + 3 < N) {
        float4 v = *reinterpret_cast<const float4*>(src);
        R.b[p][0] = v.x; R.b[p][1] = v.y; R.b[p][2] = v.z; R.b[p][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) R.b[p][j] = (gk < K && gn + j < N) ? src[j] : 0.f;
      }
    } else {  // B stored [N][K]
      const int col = idx >> 2, kq = idx & 3;
      const int64_t gn = n0 + col, gk = k0 + 4 * kq;
      const float* src = B + gn * ldb + gk;
      if (VEC && gn < N && gk < K) {
        float4 v = *reinterpret_cast<const float4*>(src);
        R.b[p][0] = v.x; R.b[p][1] = v.y; R.b[p][2] = v.z; R.b[p][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) R.b[p][j] = (gn < N && gk + j < K) ? src[j] : 0.f;
      }
    }
  }
}

template <int AL, bool TB>
__device__ __forceinline__ void f32_store_tile(const F32Regs& R, float (*As)[F_LDS], float (*Bs)[F_LDS],
                                               int tid) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int idx = tid + 256 * p;
    if (AL == A_MCONTIG) {
      const int kr = idx >> 5, mq = idx & 31;
      *reinterpret_cast<float4*>(&As[kr][4 * mq]) = make_float4(R.a[p][0], R.a[p][1], R.a[p][2], R.a[p][3]);
    } else {
      const int row = idx >> 2, kq = idx & 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) As[4 * kq + j][row] = R.a[p][j];
    }
    if (!TB) {
      const int kr = idx >> 5, nq = idx & 31;
      *reinterpret_cast<float4*>(&Bs[kr][4 * nq]) = make_float4(R.b[p][0], R.b[p][1], R.b[p][2], R.b[p][3]);
    } else {
      const int col = idx >> 2, kq = idx & 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) Bs[4 * kq + j][col] = R.b[p][j];
    }
  }
}

template <int AL, bool TB, bool VEC>
__global__ __launch_bounds__(256, 2) void gemm_f32_mfma(GemmArgs g, int tiles_m, int tiles_n,
                                                        ConvGeom cg) {
  __shared__ __attribute__((aligned(16))) float As[2][F_BK][F_LDS];
  __shared__ __attribute__((aligned(16))) float Bs[2][F_BK][F_LDS];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * F_BM;
  const int64_t n0 = (int64_t)(wg % tiles_n) * F_BN;
  const int64_t bz = blockIdx.z;
  const float* A = static_cast<const float*>(g.A) + bz * g.strideA;
  const float* B = static_cast<const float*>(g.B) + bz * g.strideB;
  float* C = static_cast<float*>(g.C) + bz * g.strideC;
  const int64_t M = g.M, N = g.N, K = g.K;

  // conv: per-piece output pixel -> (image base offset, ih0, iw0)
  int64_t conv_base[2] = {-1, -1};
  int conv_ih[2] = {0, 0}, conv_iw[2] = {0, 0};
  if (AL == A_CONV) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int64_t m = m0 + ((tid + 256 * p) >> 2);
      if (m < M) {
        const int64_t ow = m % cg.OW;
        const int64_t t = m / cg.OW;
        const int64_t oh = t % cg.OH;
        const int64_t n = t / cg.OH;
        conv_base[p] = n * (int64_t)cg.H * cg.W * cg.C;
        conv_ih[p] = (int)(oh * cg.sh - cg.pt);
        conv_iw[p] = (int)(ow * cg.sw - cg.pl);
      }
    }
  }

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int64_t ktiles = (K + F_BK - 1) / F_BK;
  F32Regs R;
  f32_load_tile<AL, TB, VEC>(R, A, B, g.lda, g.ldb, M, N, K, m0, n0, 0, tid, cg, conv_base, conv_ih, conv_iw);
  f32_store_tile<AL, TB>(R, As[0], Bs[0], tid);
  __syncthreads();
  int cur = 0;
  for (int64_t kt = 0; kt < ktiles; ++kt) {
    const bool has_next = kt + 1 < ktiles;
    if (has_next)
      f32_load_tile<AL, TB, VEC>(R, A, B, g.lda, g.ldb, M, N, K, m0, n0, (kt + 1) * F_BK, tid, cg,
                                 conv_base, conv_ih, conv_iw);
#pragma unroll
    for (int kk = 0; kk < F_BK; kk += 2) {
      const int kr = kk + (lane >> 5);
      float a0 = As[cur][kr][wm * 64 + (lane & 31)];
      float a1 = As[cur][kr][wm * 64 + 32 + (lane & 31)];
      float b0 = Bs[cur][kr][wn * 64 + (lane & 31)];
      float b1 = Bs[cur][kr][wn * 64 + 32 + (lane & 31)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (has_next) f32_store_tile<AL, TB>(R, As[cur ^ 1], Bs[cur ^ 1], tid);
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const float* bias = static_cast<const float*>(g.bias);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t col = n0 + wn * 64 + j * 32 + (lane & 31);
    const float bv = (bias && col < N) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M && col < N) C[row * g.ldc + col] = act_apply(acc[i][j][r] + bv, g.act);
      }
    }
  }
}

// ============================================================== f64 core
constexpr int D_BM = 64, D_BN = 64, D_BK = 16, D_PAD = 2;
constexpr int D_LDS = D_BM + D_PAD;

template <bool TA, bool TB>
__global__ __launch_bounds__(256, 2) void gemm_f64_mfma(GemmArgs g, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) double As[2][D_BK][D_LDS];
  __shared__ __attribute__((aligned(16))) double Bs[2][D_BK][D_LDS];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * D_BM;
  const int64_t n0 = (int64_t)(wg % tiles_n) * D_BN;
  const int64_t bz = blockIdx.z;
  const double* A = static_cast<const double*>(g.A) + bz * g.strideA;
  const double* B = static_cast<const double*>(g.B) + bz * g.strideB;
  double* C = static_cast<double*>(g.C) + bz * g.strideC;
  const int64_t M = g.M, N = g.N, K = g.K;

  // each thread moves 4 doubles of A and 4 of B per K tile
  double ra[4], rb[4];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int idx = tid + 256 * p;  // 0..1023
      if (!TA) {  // A [M][K]: idx -> (row = idx>>4, k = idx&15)
        const int64_t gm = m0 + (idx >> 4), gk = k0 + (idx & 15);
        ra[p] = (gm < M && gk < K) ? A[gm * g.lda + gk] : 0.0;
      } else {  // A [K][M]: idx -> (k = idx>>6, m = idx&63)
        const int64_t gk = k0 + (idx >> 6), gm = m0 + (idx & 63);
        ra[p] = (gm < M && gk < K) ? A[gk * g.lda + gm] : 0.0;
      }
      if (!TB) {  // B [K][N]
        const int64_t gk = k0 + (idx >> 6), gn = n0 + (idx & 63);
        rb[p] = (gn < N && gk < K) ? B[gk * g.ldb + gn] : 0.0;
      } else {  // B [N][K]
        const int64_t gn = n0 + (idx >> 4), gk = k0 + (idx & 15);
        rb[p] = (gn < N && gk < K) ? B[gn * g.ldb + gk] : 0.0;
      }
    }
  };
  auto store = [&](int st) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int idx = tid + 256 * p;
      if (!TA) As[st][idx & 15][idx >> 4] = ra[p];
      else As[st][idx >> 6][idx & 63] = ra[p];
      if (!TB) Bs[st][idx >> 6][idx & 63] = rb[p];
      else Bs[st][idx & 15][idx >> 4] = rb[p];
    }
  };

  f64x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};

  const int64_t ktiles = (K + D_BK - 1) / D_BK;
  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int64_t kt = 0; kt < ktiles; ++kt) {
    const bool has_next = kt + 1 < ktiles;
    if (has_next) load((kt + 1) * D_BK);
#pragma unroll
    for (int kk = 0; kk < D_BK; kk += 4) {
      const int kr = kk + (lane >> 4);
      double a0 = As[cur][kr][wm * 32 + (lane & 15)];
      double a1 = As[cur][kr][wm * 32 + 16 + (lane & 15)];
      double b0 = Bs[cur][kr][wn * 32 + (lane & 15)];
      double b1 = Bs[cur][kr][wn * 32 + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (has_next) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  // f64 C/D layout: col = lane&15, row = (lane>>4) + 4*r
  const double* bias = static_cast<const double*>(g.bias);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t col = n0 + wn * 32 + j * 16 + (lane & 15);
    const double bv = (bias && col < N) ? bias[col] : 0.0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 32 + i * 16 + (lane >> 4) + 4 * r;
        if (row < M && col < N) C[row * g.ldc + col] = act_apply(acc[i][j][r] + bv, g.act);
      }
    }
  }
}

// ============================================================== integer GEMM (VALU)
template <typename T>
__global__ __launch_bounds__(256) void gemm_int(GemmArgs g) {
  __shared__ T As[16][17];
  __shared__ T Bs[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int64_t row = (int64_t)blockIdx.y * 16 + ty, col = (int64_t)blockIdx.x * 16 + tx;
  const int64_t bz = blockIdx.z;
  const T* A = static_cast<const T*>(g.A) + bz * g.strideA;
  const T* B = static_cast<const T*>(g.B) + bz * g.strideB;
  T* C = static_cast<T*>(g.C) + bz * g.strideC;
  int64_t acc = 0;
  for (int64_t k0 = 0; k0 < g.K; k0 += 16) {
    const int64_t ka = k0 + tx, kb = k0 + ty;
    const int64_t arow = (int64_t)blockIdx.y * 16 + ty;
    const int64_t bcol = (int64_t)blockIdx.x * 16 + tx;
    As[ty][tx] = (arow < g.M && ka < g.K) ? (g.ta ? A[ka * g.lda + arow] : A[arow * g.lda + ka]) : T(0);
    Bs[ty][tx] = (bcol < g.N && kb < g.K) ? (g.tb ? B[bcol * g.ldb + kb] : B[kb * g.ldb + bcol]) : T(0);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) acc += (int64_t)As[ty][kk] * (int64_t)Bs[kk][tx];
    __syncthreads();
  }
  if (row < g.M && col < g.N) {
    T v = T(acc);
    if (g.bias) v += static_cast<const T*>(g.bias)[col];
    C[row * g.ldc + col] = act_apply(v, g.act);
  }
}

// ============================================================== pooling (NHWC)
__global__ __launch_bounds__(256) void pool2d_kernel(PoolArgs a, int64_t n) {
  const float* x = static_cast<const float*>(a.x);
  float* y = static_cast<float*>(a.y);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t c = i % a.C;
    int64_t t = i / a.C;
    int64_t ow = t % a.OW;
    t /= a.OW;
    int64_t oh = t % a.OH;
    int64_t nn = t / a.OH;
    const int64_t h0 = oh * a.sh - a.pad_t, w0 = ow * a.sw - a.pad_l;
    float acc = a.is_max ? -INFINITY : 0.f;
    int cnt = 0;
    for (int64_t kh = 0; kh < a.KH; ++kh) {
      const int64_t ih = h0 + kh;
      if (ih < 0 || ih >= a.H) continue;
      for (int64_t kw = 0; kw < a.KW; ++kw) {
        const int64_t iw = w0 + kw;
        if (iw < 0 || iw >= a.W) continue;
        const float v = x[((nn * a.H + ih) * a.W + iw) * a.C + c];
        if (a.is_max) acc = v > acc ? v : acc;
        else acc += v;
        ++cnt;
      }
    }
    y[i] = a.is_max ? acc : (cnt ? acc / (float)cnt : 0.f);
  }
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <int AL, bool TB>
void launch_f32(const GemmArgs& g, bool vec, const ConvGeom& cg, hipStream_t s) {
  const int64_t tm = (g.M + F_BM - 1) / F_BM, tn = (g.N + F_BN - 1) / F_BN;
  TFA_CHECK(tm * tn < (int64_t(1) << 31), "gemm: grid too large");
  TFA_CHECK(g.batch <= 65535, "gemm: batch too large");
  dim3 grid((unsigned)(tm * tn), 1, (unsigned)g.batch);
  if (vec)
    hipLaunchKernelGGL((gemm_f32_mfma<AL, TB, true>), grid, dim3(256), 0, s, g, (int)tm, (int)tn, cg);
  else
    hipLaunchKernelGGL((gemm_f32_mfma<AL, TB, false>), grid, dim3(256), 0, s, g, (int)tm, (int)tn, cg);
}

}  // namespace

void gemm(DType dt, const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return;
  TFA_CHECK(g.K > 0, "gemm: K must be > 0");
  TFA_CHECK(g.A && g.B && g.C, "gemm: null operand");
  if (dt == DType::F32) {
    // 16-byte vector loads need 4-float aligned rows on the contiguous side
    bool vec = al16(g.A) && al16(g.B) && g.lda % 4 == 0 && g.ldb % 4 == 0 &&
               (g.batch == 1 || (g.strideA % 4 == 0 && g.strideB % 4 == 0));
    if (!g.ta) vec = vec && g.K % 4 == 0;
    if (g.tb) vec = vec && g.K % 4 == 0;
    ConvGeom cg{};
    if (!g.ta && !g.tb) launch_f32<A_KCONTIG, false>(g, vec, cg, s);
    else if (!g.ta && g.tb) launch_f32<A_KCONTIG, true>(g, vec, cg, s);
    else if (g.ta && !g.tb) launch_f32<A_MCONTIG, false>(g, vec, cg, s);
    else launch_f32<A_MCONTIG, true>(g, vec, cg, s);
  } else if (dt == DType::F64) {
    const int64_t tm = (g.M + D_BM - 1) / D_BM, tn = (g.N + D_BN - 1) / D_BN;
    TFA_CHECK(tm * tn < (int64_t(1) << 31), "gemm: grid too large");
    dim3 grid((unsigned)(tm * tn), 1, (unsigned)g.batch);
    if (!g.ta && !g.tb) hipLaunchKernelGGL((gemm_f64_mfma<false, false>), grid, dim3(256), 0, s, g, (int)tm, (int)tn);
    else if (!g.ta && g.tb) hipLaunchKernelGGL((gemm_f64_mfma<false, true>), grid, dim3(256), 0, s, g, (int)tm, (int)tn);
    else if (g.ta && !g.tb) hipLaunchKernelGGL((gemm_f64_mfma<true, false>), grid, dim3(256), 0, s, g, (int)tm, (int)tn);
    else hipLaunchKernelGGL((gemm_f64_mfma<true, true>), grid, dim3(256), 0, s, g, (int)tm, (int)tn);
  } else if (dt == DType::I32 || dt == DType::I64) {
    dim3 grid((unsigned)((g.N + 15) / 16), (unsigned)((g.M + 15) / 16), (unsigned)g.batch);
    TFA_CHECK((g.M + 15) / 16 <= 65535, "int gemm: M too large");
    if (dt == DType::I32) hipLaunchKernelGGL((gemm_int<int32_t>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_int<int64_t>), grid, dim3(256), 0, s, g);
  } else {
    TFA_CHECK(false, "gemm: dtype ", dtype_name(dt), " not supported");
  }
  TFA_LAUNCH_CHECK("gemm");
}

void conv2d_nhwc(DType dt, const ConvArgs& a, hipStream_t s) {
  TFA_CHECK(dt == DType::F32, "conv2d: f32 only");
  TFA_CHECK(a.N > 0 && a.OH > 0 && a.OW > 0 && a.OC > 0, "conv2d: empty output");
  TFA_CHECK(a.H < (1 << 30) && a.W < (1 << 30) && a.C < (1 << 30), "conv2d: dims too large");
  GemmArgs g{};
  g.M = a.N * a.OH * a.OW;
  g.N = a.OC;
  g.K = a.KH * a.KW * a.C;
  g.A = a.x; g.lda = 0; g.strideA = 0;
  g.B = a.w; g.ldb = a.OC; g.strideB = 0;
  g.C = a.y; g.ldc = a.OC; g.strideC = 0;
  g.ta = false; g.tb = false;
  g.bias = a.bias;
  g.act = a.act;
  g.batch = 1;
  ConvGeom cg;
  cg.H = (int)a.H; cg.W = (int)a.W; cg.C = (int)a.C; cg.KW = (int)a.KW;
  cg.OH = (int)a.OH; cg.OW = (int)a.OW;
  cg.sh = (int)a.sh; cg.sw = (int)a.sw; cg.dh = (int)a.dh; cg.dw = (int)a.dw;
  cg.pt = (int)a.pad_t; cg.pl = (int)a.pad_l;
  bool vec = a.C % 4 == 0 && al16(a.x) && al16(a.w) && a.OC % 4 == 0;
  launch_f32<A_CONV, false>(g, vec, cg, s);
  TFA_LAUNCH_CHECK("conv2d");
}

void pool2d_nhwc(DType dt, const PoolArgs& a, hipStream_t s) {
  TFA_CHECK(dt == DType::F32, "pool2d: f32 only");
  int64_t n = a.N * a.OH * a.OW * a.C;
  if (n <= 0) return;
  hipLaunchKernelGGL(pool2d_kernel, dim3(ew_grid(n)), dim3(256), 0, s, a, n);
  TFA_LAUNCH_CHECK("pool2d");
}

}  // namespace k
}  // namespace tfa

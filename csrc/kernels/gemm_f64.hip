// f64 MFMA GEMM, integer GEMM and NHWC pooling kernels for gfx950.
//
// f64: v_mfma_f64_16x16x4_f64. 64x64x16 block tile, 4 waves as 2x2, each
// wave 32x32 = 2x2 MFMA tiles of 16x16 (f64 has its own C/D layout:
// col = lane&15, row = (lane>>4) + 4*reg). k-major LDS images, two stages,
// register-staged prefetch of the next K tile, bias/ReLU epilogue.
#include <cmath>

#include <type_traits>

#include "gemm_internal.h"
#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcd_remap64(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}


constexpr int D_BK = 16, D_PAD = 2;

// sched_group_barrier masks (LLVM AMDGPU): MFMA, VMEM read, DS read, DS write
constexpr int kSchedMfma64 = 0x008, kSchedVmemRead64 = 0x020, kSchedDsRead64 = 0x100, kSchedDsWrite64 = 0x200;

template <int J, int END, int O1, int M1, int M2>
__device__ __forceinline__ void sched_ops64() {
  if constexpr (J < END) {
    __builtin_amdgcn_sched_group_barrier(J < O1 ? M1 : M2, 1, 0);
    sched_ops64<J + 1, END, O1, M1, M2>();
  }
}
// NM MFMAs with O memory ops spread between them (slot I: ops [I*O/NM, (I+1)*O/NM))
template <int I, int NM, int O, int O1, int M1, int M2>
__device__ __forceinline__ void sched_interleave64() {
  if constexpr (I < NM) {
    constexpr int lo = (I * O + NM - 1) / NM, hi = ((I + 1) * O + NM - 1) / NM;
    sched_ops64<lo, hi, O1, M1, M2>();
    __builtin_amdgcn_sched_group_barrier(kSchedMfma64, 1, 0);
    sched_interleave64<I + 1, NM, O, O1, M1, M2>();
  }
}

// Block tile BM x BN (64x64 or 128x128), 4 waves as 2x2, each wave owning
// (BM/2)x(BN/2) as TMxTN 16x16 MFMA tiles. Interior blocks load 2 doubles per
// 16-byte access without bounds checks; edge blocks take the checked path.
template <int BM, int BN, int WM, int WN, bool TA, bool TB>
__global__ __launch_bounds__(256, 2) void gemm_f64_mfma(GemmArgs g, int tiles_m, int tiles_n) {
  constexpr int LDA = BM + D_PAD, LDB = BN + D_PAD;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "4 waves, >= one 16x16 tile each");
  constexpr int AE = BM * D_BK / 256, BE = BN * D_BK / 256;  // doubles per thread per K tile
  static_assert(AE % 2 == 0 && (BE % 2 == 0 || BE == 1), "pairs of doubles (or one B element)");
  __shared__ __attribute__((aligned(16))) double As[2][D_BK][LDA];
  __shared__ __attribute__((aligned(16))) double Bs[2][D_BK][LDB];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap64(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * BM;
  const int64_t n0 = (int64_t)(wg % tiles_n) * BN;
  const int64_t bz = blockIdx.z;
  const double* A = static_cast<const double*>(g.A) + bz * g.strideA;
  const double* B = static_cast<const double*>(g.B) + bz * g.strideB;
  double* C = static_cast<double*>(g.C) + bz * g.strideC;
  const int64_t M = g.M, N = g.N, K = g.K;
  // A and B take the unchecked 16-byte path independently (a skinny N edge
  // tile still streams A unchecked)
  const bool a_rows = m0 + BM <= M && (reinterpret_cast<uintptr_t>(A) & 15) == 0 && g.lda % 2 == 0;
  const bool b_cols = n0 + BN <= N && (reinterpret_cast<uintptr_t>(B) & 15) == 0 && g.ldb % 2 == 0;

  // element e (pairs e, e+1 are adjacent along the contiguous dim) of this
  // thread's share: A [M][K] -> (row, k) with k contiguous; A^T [K][M] -> (k, m)
  double ra[AE], rb[BE];
  auto a_coord = [&](int e, int& r, int& c) {  // r = m, c = k (tile-local)
    const int idx = tid * AE + e;
    if (!TA) { r = idx / D_BK; c = idx % D_BK; }
    else { c = idx / BM; r = idx % BM; }
  };
  auto b_coord = [&](int e, int& r, int& c) {  // r = k, c = n
    const int idx = tid * BE + e;
    if (!TB) { r = idx / BN; c = idx % BN; }
    else { c = idx / D_BK; r = idx % D_BK; }
  };
  // FAST: interior block (A rows and B columns in range, 16-byte aligned,
  // K a multiple of D_BK): unconditional 16-byte loads, no branch in the loop
  auto load = [&](int64_t k0, auto fast_t) __attribute__((always_inline)) {
    constexpr bool FAST = decltype(fast_t)::value;
    const bool kfull = FAST || k0 + D_BK <= K;  // only the K tail tile is checked
    const bool a_fast = FAST || (a_rows && kfull), b_fast = FAST || (b_cols && kfull);
    if (a_fast) {
#pragma unroll
      for (int e = 0; e < AE; e += 2) {
        int r, c;
        a_coord(e, r, c);
        const double* p = !TA ? A + (m0 + r) * g.lda + (k0 + c) : A + (k0 + c) * g.lda + (m0 + r);
        const double2 v = *reinterpret_cast<const double2*>(p);
        ra[e] = v.x;
        ra[e + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int e = 0; e < AE; ++e) {
        int r, c;
        a_coord(e, r, c);
        const int64_t gm = m0 + r, gk = k0 + c;
        ra[e] = (gm < M && gk < K) ? (!TA ? A[gm * g.lda + gk] : A[gk * g.lda + gm]) : 0.0;
      }
    }
    if (b_fast) {
      if constexpr (BE == 1) {
        int r, c;
        b_coord(0, r, c);
        rb[0] = !TB ? B[(k0 + r) * g.ldb + (n0 + c)] : B[(n0 + c) * g.ldb + (k0 + r)];
      } else {
#pragma unroll
        for (int e = 0; e < BE; e += 2) {
          int r, c;
          b_coord(e, r, c);
          const double* p = !TB ? B + (k0 + r) * g.ldb + (n0 + c) : B + (n0 + c) * g.ldb + (k0 + r);
          const double2 v = *reinterpret_cast<const double2*>(p);
          rb[e] = v.x;
          rb[e + 1] = v.y;
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < BE; ++e) {
        int r, c;
        b_coord(e, r, c);
        const int64_t gk = k0 + r, gn = n0 + c;
        rb[e] = (gn < N && gk < K) ? (!TB ? B[gk * g.ldb + gn] : B[gn * g.ldb + gk]) : 0.0;
      }
    }
  };
  auto store = [&](int st) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < AE; ++e) {
      int r, c;
      a_coord(e, r, c);
      As[st][c][r] = ra[e];
    }
#pragma unroll
    for (int e = 0; e < BE; ++e) {
      int r, c;
      b_coord(e, r, c);
      Bs[st][r][c] = rb[e];
    }
  };

  f64x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};

  // per K tile: S k-steps of NM MFMAs; R LDS reads per k-step; L global loads
  // and W LDS writes per tile. Interior blocks use the interleaved schedule of
  // gemm.hip (memory ops spread between the MFMAs with sched_group_barrier,
  // operands read one k-step ahead, last tile peeled: no branch in the loop).
  constexpr int S = D_BK / 4, NM = TM * TN, R = TM + TN;
  constexpr int L = AE / 2 + (BE == 1 ? 1 : BE / 2), W = AE + BE;
  const int64_t ktiles = (K + D_BK - 1) / D_BK;
  auto mainloop = [&](auto fast_t) __attribute__((always_inline)) {
    constexpr bool FAST = decltype(fast_t)::value;
    load(0, fast_t);
    store(0);
    __syncthreads();
    int cur = 0;
    auto tile = [&](int64_t knext, auto more) __attribute__((always_inline)) {
      constexpr bool NEXT = decltype(more)::value;
      double a[2][TM], b[2][TN];
      auto rd = [&](int buf, int kk) __attribute__((always_inline)) {
        const int kr = kk + (lane >> 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) a[buf][i] = As[cur][kr][wm * (BM / WM) + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[buf][j] = Bs[cur][kr][wn * (BN / WN) + j * 16 + (lane & 15)];
      };
      rd(0, 0);
      if constexpr (FAST) __builtin_amdgcn_sched_group_barrier(kSchedDsRead64, R, 0);
      if constexpr (NEXT) load(knext, fast_t);
#pragma unroll
      for (int kk = 0; kk < S; ++kk) {
        if (kk + 1 < S) rd((kk + 1) & 1, 4 * (kk + 1));
        if (NEXT && kk == S - 1) store(cur ^ 1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kk & 1][i], b[kk & 1][j], acc[i][j], 0, 0, 0);
        if constexpr (FAST) {
          if (kk == 0 && NEXT)
            sched_interleave64<0, NM, L + R, L, kSchedVmemRead64, kSchedDsRead64>();
          else if (kk == S - 1 && NEXT)
            sched_interleave64<0, NM, W, W, kSchedDsWrite64, kSchedDsWrite64>();
          else if (kk + 1 < S)
            sched_interleave64<0, NM, R, R, kSchedDsRead64, kSchedDsRead64>();
          else
            __builtin_amdgcn_sched_group_barrier(kSchedMfma64, NM, 0);
        }
      }
      __syncthreads();
      cur ^= 1;
    };
    for (int64_t kt = 0; kt + 1 < ktiles; ++kt) tile((kt + 1) * D_BK, std::true_type{});
    tile(0, std::false_type{});
  };
  if (a_rows && b_cols && K > 0 && K % D_BK == 0)
    mainloop(std::true_type{});
  else
    mainloop(std::false_type{});
  // f64 C/D layout: col = lane&15, row = (lane>>4) + 4*r
  const double* bias = static_cast<const double*>(g.bias);
  // constant acc indices only (see gemm.hip): cheap epilogue while storing,
  // transcendental activations / absorbed chains in a fix-up loop over the
  // elements this thread wrote
  const bool heavy = !(g.act <= ACT_RELU6 && g.epi.n == 0);
  const int cheap_act = heavy ? ACT_NONE : g.act;
  static_for<TN>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int64_t col = n0 + wn * (BN / WN) + j * 16 + (lane & 15);
    const double bv = (bias && col < N) ? bias[col] : 0.0;
    static_for<TM>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const f64x4 v = acc[i][j];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * (BM / WM) + i * 16 + (lane >> 4) + 4 * r;
        if (row < M && col < N) C[row * g.ldc + col] = act_fast(v[r] + bv, cheap_act);
      }
    });
  });
  if (heavy) {
#pragma nounroll
    for (int e = 0; e < TN * TM * 4; ++e) {
      const int j = e / (TM * 4), i = (e / 4) % TM, r = e % 4;
      const int64_t col = n0 + wn * (BN / WN) + j * 16 + (lane & 15);
      const int64_t row = m0 + wm * (BM / WM) + i * 16 + (lane >> 4) + 4 * r;
      if (col >= N || row >= M) continue;
      double* p = C + row * g.ldc + col;
      *p = epi_apply(g.epi, act_apply(*p, g.act), row, col, N, bz * M * N);
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
    C[row * g.ldc + col] = act_fast(v, g.act);
  }
}

// ============================================================== pooling (NHWC)
// One thread per V consecutive channels of one output pixel (V = 4: float4
// loads/stores when C % 4 == 0). Index math is 32-bit when the tensors fit
// (64-bit div/mod costs ~40 VALU ops on CDNA).
template <bool MAX, int V, typename I>
__global__ __launch_bounds__(256) void pool2d_kernel(PoolArgs a, I n_items, FastDivU32 fCV, FastDivU32 fOW,
                                                     FastDivU32 fOH) {
  using vec_t = typename std::conditional<V == 4, float4, float>::type;
  const float* x = static_cast<const float*>(a.x);
  float* y = static_cast<float*>(a.y);
  const I CV = (I)(a.C / V), OW = (I)a.OW, OH = (I)a.OH, H = (I)a.H, W = (I)a.W;
  const I stride = (I)gridDim.x * blockDim.x;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += stride) {
    I cv, t, pix, ow, oh, nn;
    if constexpr (sizeof(I) == 4) {  // 32-bit items: magic-number divides (6 divides per item otherwise)
      t = fdiv(i, fCV);
      cv = i - t * CV;
      pix = t;
      const I t2 = fdiv(t, fOW);
      ow = t - t2 * OW;
      nn = fdiv(t2, fOH);
      oh = t2 - nn * OH;
    } else {
      cv = i % CV;
      t = i / CV;
      pix = t;
      ow = t % OW;
      t /= OW;
      oh = t % OH;
      nn = t / OH;
    }
    const int h0 = (int)(oh * (I)a.sh) - (int)a.pad_t, w0 = (int)(ow * (I)a.sw) - (int)a.pad_l;
    const int hb = h0 < 0 ? 0 : h0, he = min(h0 + (int)a.KH, (int)H);
    const int wb = w0 < 0 ? 0 : w0, we = min(w0 + (int)a.KW, (int)W);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = MAX ? -INFINITY : 0.f;
    const float* base = x + (int64_t)nn * H * W * a.C + (int64_t)cv * V;
    for (int ih = hb; ih < he; ++ih) {
      for (int iw = wb; iw < we; ++iw) {
        vec_t v = *reinterpret_cast<const vec_t*>(base + ((int64_t)ih * W + iw) * a.C);
        const float* f = reinterpret_cast<const float*>(&v);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = MAX ? fmaxf(acc[j], f[j]) : acc[j] + f[j];
      }
    }
    const int cnt = (he - hb) * (we - wb);
    vec_t o;
    float* of = reinterpret_cast<float*>(&o);
#pragma unroll
    for (int j = 0; j < V; ++j) of[j] = MAX ? acc[j] : (cnt > 0 ? acc[j] / (float)cnt : 0.f);
    if (a.bias) {
      const float* b = static_cast<const float*>(a.bias) + (int64_t)cv * V;
#pragma unroll
      for (int j = 0; j < V; ++j) of[j] = act_fast(of[j] + b[j], a.act);
    } else if (a.act) {
#pragma unroll
      for (int j = 0; j < V; ++j) of[j] = act_fast(of[j], a.act);
    }
    float* dst = a.ldc ? y + (int64_t)pix * a.ldc + (int64_t)cv * V : y + (int64_t)i * V;
    *reinterpret_cast<vec_t*>(dst) = o;
  }
}

// 3x3 windows (every pool of Inception-v3), float4 channels, 32-bit indices:
// the nine taps are unrolled with clamped in-bounds addresses, so each lane
// has all nine 16-byte loads in flight before the first max/add (the generic
// kernel's data-dependent window loops issue them one at a time). Taps outside
// the image are masked out of the result; avg divides by the valid-tap count
// (TF semantics). Same epilogue and concat-slice output as pool2d_kernel.
//
// XCD: one block per 256 items, and block b runs the items of block
// xcd_remap64(b): the hardware deals consecutive blocks round-robin over the
// 8 XCDs, so without the remap the output rows that share an input row run on
// different XCDs and each XCD's L2 fetches that row again; with it every XCD
// walks one contiguous range of output rows.
template <bool MAX, bool XCD>
__global__ __launch_bounds__(256) void pool3x3_v4_kernel(PoolArgs a, uint32_t n_items, FastDivU32 fCV,
                                                          FastDivU32 fOW, FastDivU32 fOH) {
  const float* x = static_cast<const float*>(a.x);
  float* y = static_cast<float*>(a.y);
  const uint32_t CV = (uint32_t)(a.C >> 2), OW = (uint32_t)a.OW, OH = (uint32_t)a.OH;
  const int H = (int)a.H, W = (int)a.W, C = (int)a.C;
  const uint32_t stride = XCD ? n_items : gridDim.x * blockDim.x;
  const uint32_t first = XCD ? (uint32_t)xcd_remap64((int)blockIdx.x, (int)gridDim.x) * blockDim.x + threadIdx.x
                             : blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = first; i < n_items; i += stride) {
    const uint32_t pix = fdiv(i, fCV), cv = i - pix * CV;
    const uint32_t t2 = fdiv(pix, fOW), ow = pix - t2 * OW;
    const uint32_t nn = fdiv(t2, fOH), oh = t2 - nn * OH;
    const int h0 = (int)oh * (int)a.sh - (int)a.pad_t, w0 = (int)ow * (int)a.sw - (int)a.pad_l;
    const float* base = x + (uint32_t)((int)nn * H * W * C) + cv * 4;
    float4 v[9];
    bool ok[9];
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {
      const int ih = h0 + dh;
      const int ihc = min(max(ih, 0), H - 1);
#pragma unroll
      for (int dw = 0; dw < 3; ++dw) {
        const int iw = w0 + dw;
        const int iwc = min(max(iw, 0), W - 1);
        ok[dh * 3 + dw] = ih == ihc && iw == iwc;
        v[dh * 3 + dw] = *reinterpret_cast<const float4*>(base + (uint32_t)((ihc * W + iwc) * C));
      }
    }
    const float init = MAX ? -INFINITY : 0.f;
    float4 acc = make_float4(init, init, init, init);
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const float4 u = ok[j] ? v[j] : make_float4(init, init, init, init);
      if (MAX) {
        acc.x = fmaxf(acc.x, u.x); acc.y = fmaxf(acc.y, u.y); acc.z = fmaxf(acc.z, u.z); acc.w = fmaxf(acc.w, u.w);
      } else {
        acc.x += u.x; acc.y += u.y; acc.z += u.z; acc.w += u.w;
      }
    }
    float of[4] = {acc.x, acc.y, acc.z, acc.w};
    if (!MAX) {
      const int cnt = (min(h0 + 3, H) - max(h0, 0)) * (min(w0 + 3, W) - max(w0, 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) of[j] = cnt > 0 ? of[j] / (float)cnt : 0.f;
    }
    if (a.bias) {
      const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(a.bias) + cv * 4);
      of[0] = act_fast(of[0] + b.x, a.act); of[1] = act_fast(of[1] + b.y, a.act);
      of[2] = act_fast(of[2] + b.z, a.act); of[3] = act_fast(of[3] + b.w, a.act);
    } else if (a.act) {
#pragma unroll
      for (int j = 0; j < 4; ++j) of[j] = act_fast(of[j], a.act);
    }
    float* dst = a.ldc ? y + (uint32_t)(pix * (uint32_t)a.ldc) + cv * 4 : y + i * 4;
    *reinterpret_cast<float4*>(dst) = make_float4(of[0], of[1], of[2], of[3]);
  }
}

template <bool MAX>
void pool2d_launch(const PoolArgs& a, hipStream_t s) {
  const bool v4 = a.C % 4 == 0 && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(a.y) & 15) == 0 && a.ldc % 4 == 0;
  const int V = v4 ? 4 : 1;
  const int64_t items = a.N * a.OH * a.OW * (a.C / V);
  const bool small = a.N * a.H * a.W * a.C < (int64_t(1) << 31) && a.N * a.OH * a.OW * a.C < (int64_t(1) << 31);
  const dim3 grid(ew_grid(items)), block(256);
  const FastDivU32 fCV = make_fastdiv((uint32_t)(a.C / V)), fOW = make_fastdiv((uint32_t)a.OW),
                   fOH = make_fastdiv((uint32_t)a.OH);
  static const bool generic = [] {
    const char* e = std::getenv("TFA_POOL_GENERIC");
    return e && e[0] == '1';
  }();
  const int64_t out_span = a.ldc ? a.N * a.OH * a.OW * a.ldc : a.N * a.OH * a.OW * a.C;
  static const bool no_xcd = [] {
    const char* e = std::getenv("TFA_POOL_XCD");
    return e && e[0] == '0';
  }();
  if (v4 && small && a.KH == 3 && a.KW == 3 && out_span < (int64_t(1) << 31) && !generic) {
    const int64_t nblk = (items + 255) / 256;
    if (!no_xcd && nblk < (int64_t(1) << 30))
      hipLaunchKernelGGL((pool3x3_v4_kernel<MAX, true>), dim3((unsigned)nblk), block, 0, s, a, (uint32_t)items, fCV,
                         fOW, fOH);
    else
      hipLaunchKernelGGL((pool3x3_v4_kernel<MAX, false>), grid, block, 0, s, a, (uint32_t)items, fCV, fOW, fOH);
    return;
  }
  if (v4 && small)
    hipLaunchKernelGGL((pool2d_kernel<MAX, 4, uint32_t>), grid, block, 0, s, a, (uint32_t)items, fCV, fOW, fOH);
  else if (v4)
    hipLaunchKernelGGL((pool2d_kernel<MAX, 4, int64_t>), grid, block, 0, s, a, items, fCV, fOW, fOH);
  else if (small)
    hipLaunchKernelGGL((pool2d_kernel<MAX, 1, uint32_t>), grid, block, 0, s, a, (uint32_t)items, fCV, fOW, fOH);
  else
    hipLaunchKernelGGL((pool2d_kernel<MAX, 1, int64_t>), grid, block, 0, s, a, items, fCV, fOW, fOH);
}

}  // namespace

template <int BM, int BN, int WM, int WN>
static void gemm_f64_tile_launch(const GemmArgs& g, hipStream_t s) {
  const int64_t tm = (g.M + BM - 1) / BM, tn = (g.N + BN - 1) / BN;
  TFA_CHECK(tm * tn < (int64_t(1) << 31), "gemm: grid too large");
  TFA_CHECK(g.batch <= 65535, "gemm: batch too large");
  dim3 grid((unsigned)(tm * tn), 1, (unsigned)g.batch);
  if (!g.ta && !g.tb) hipLaunchKernelGGL((gemm_f64_mfma<BM, BN, WM, WN, false, false>), grid, dim3(256), 0, s, g, (int)tm, (int)tn);
  else if (!g.ta && g.tb) hipLaunchKernelGGL((gemm_f64_mfma<BM, BN, WM, WN, false, true>), grid, dim3(256), 0, s, g, (int)tm, (int)tn);
  else if (g.ta && !g.tb) hipLaunchKernelGGL((gemm_f64_mfma<BM, BN, WM, WN, true, false>), grid, dim3(256), 0, s, g, (int)tm, (int)tn);
  else hipLaunchKernelGGL((gemm_f64_mfma<BM, BN, WM, WN, true, true>), grid, dim3(256), 0, s, g, (int)tm, (int)tn);
}

void gemm_f64_launch(const GemmArgs& g, hipStream_t s) {
  // 128x128 tiles halve operand traffic per FLOP; used when they still give
  // >= 2 blocks per CU (256 CUs), else 64x64
  // skinny N (K-Means: points x k centres): 64x16 tiles, A streamed once by
  // many blocks (the shape is HBM-bound)
  const int64_t big = ((g.M + 127) / 128) * ((g.N + 127) / 128) * g.batch;
  if (g.N <= 16) gemm_f64_tile_launch<64, 16, 4, 1>(g, s);
  else if (g.N > 64 && big >= 512) gemm_f64_tile_launch<128, 128, 2, 2>(g, s);
  else gemm_f64_tile_launch<64, 64, 2, 2>(g, s);
}

void gemm_int_launch(DType dt, const GemmArgs& g, hipStream_t s) {
  dim3 grid((unsigned)((g.N + 15) / 16), (unsigned)((g.M + 15) / 16), (unsigned)g.batch);
  TFA_CHECK((g.M + 15) / 16 <= 65535, "int gemm: M too large");
  if (dt == DType::I32) hipLaunchKernelGGL((gemm_int<int32_t>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((gemm_int<int64_t>), grid, dim3(256), 0, s, g);
}

void pool2d_nhwc(DType dt, const PoolArgs& a, hipStream_t s) {
  TFA_CHECK(dt == DType::F32, "pool2d: f32 only");
  if (a.N * a.OH * a.OW * a.C <= 0) return;
  TFA_CHECK(a.KH > 0 && a.KW > 0 && a.sh > 0 && a.sw > 0, "pool2d: bad window");
  if (a.is_max) pool2d_launch<true>(a, s);
  else pool2d_launch<false>(a, s);
  TFA_LAUNCH_CHECK("pool2d");
}

}  // namespace k
}  // namespace tfa

// Reduced-precision f32 GEMM / implicit-GEMM Conv2D on bf16 MFMA (gfx950).
//
// Opt-in compute modes for float32 MatMul / Conv2D (tfa::k::set_f32_precision,
// Python `Config.precision`); the default stays exact f32 (gemm.hip). Operands
// and outputs stay float32 in HBM: the A loader converts each float4 it loads
// to bf16 on the way into LDS, B (the weights / right operand, small) is
// converted once per launch by a prep kernel into [N][Kp] bf16 images.
//
//  * BF16   (mode 1): C = sum bf16(a) * bf16(b)             (8-bit mantissa operands)
//  * BF16X3 (mode 2): a = ah + al, b = bh + bl (bf16 each);
//                     C = sum ah*bh + ah*bl + al*bh        (~16-bit operands, 3 MFMAs)
// Accumulation is f32 in both. v_mfma_f32_32x32x16_bf16 runs 16x the f32 MFMA
// rate, so BF16X3 has 5.3x the f32 core's arithmetic peak.
//
// Layout: LDS images are k-contiguous rows [row][BK + 8] of bf16 (80-byte
// stride: the 16-lane groups of a ds_read_b128 hit 16 distinct 16-byte bank
// slots). MFMA fragment of lane l: row l&31, k = 8*(l>>5) .. +7 of the 16-deep
// step = one ds_read_b128 per operand per step. C/D layout as the f32 form.
#include <array>
#include <cstdlib>
#include <map>
#include <mutex>

#include "gemm_internal.h"
#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kBK = 32;        // k depth of one LDS stage (two 16-deep MFMA steps)
constexpr int kRow = kBK + 8;  // LDS row stride in bf16

// round-to-nearest-even f32 -> bf16: a plain cast, which hipcc lowers to
// v_cvt_pk_bf16_f32 on gfx950 (one instruction per pair; NaN stays NaN)
__device__ __forceinline__ uint32_t bf16_bits_rne(float x) {
  const __bf16 h = static_cast<__bf16>(x);
  return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, h));
}
__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

// hi/lo split of 4 floats, packed as 4 bf16 each (uint2 = 8 bytes)
__device__ __forceinline__ void split4(const float4 v, uint2& hi, uint2& lo) {
  const uint32_t h0 = bf16_bits_rne(v.x), h1 = bf16_bits_rne(v.y), h2 = bf16_bits_rne(v.z),
                 h3 = bf16_bits_rne(v.w);
  hi.x = h0 | (h1 << 16);
  hi.y = h2 | (h3 << 16);
  const uint32_t l0 = bf16_bits_rne(v.x - bf16_to_f32(h0)), l1 = bf16_bits_rne(v.y - bf16_to_f32(h1)),
                 l2 = bf16_bits_rne(v.z - bf16_to_f32(h2)), l3 = bf16_bits_rne(v.w - bf16_to_f32(h3));
  lo.x = l0 | (l1 << 16);
  lo.y = l2 | (l3 << 16);
}

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}


// B f32 ([K][N] or [N][K]) -> hi/lo bf16 images [N][Kp], zero-padded to Kp
__global__ __launch_bounds__(256) void prep_b(const float* __restrict__ B, int64_t ldb, bool tb, int64_t N,
                                              int64_t K, int64_t Kp, uint16_t* __restrict__ hi,
                                              uint16_t* __restrict__ lo) {
  const int64_t total = N * Kp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i / Kp, kk = i % Kp;
    float v = 0.f;
    if (kk < K) v = tb ? B[n * ldb + kk] : B[kk * ldb + n];
    const uint32_t h = bf16_bits_rne(v);
    hi[i] = (uint16_t)h;
    if (lo) lo[i] = (uint16_t)bf16_bits_rne(v - bf16_to_f32(h));
  }
}

enum { A_KCONTIG = 0, A_CONV = 2 };

template <int BM, int BN, int WM, int WN, int AL, bool X3>
__global__ __launch_bounds__(256, 2) void gemm_bf16_tile(GemmArgs g, int tiles_m, int tiles_n, Im2colGeom cg,
                                                         const uint16_t* __restrict__ Bhi,
                                                         const uint16_t* __restrict__ Blo, int64_t Kp) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "4 waves, >= one 32x32 tile each");
  constexpr int NA = X3 ? 2 : 1;                    // A / B images per stage (hi [, lo])
  constexpr int AP = BM * kBK / 4 / 256;            // float4 A pieces per thread per tile
  constexpr int BP = BN * kBK / 8 / 256;            // 16-byte B pieces per thread per image
  static_assert(AP >= 1 && BP >= 1, "tile too small for 256 threads");
  __shared__ __attribute__((aligned(16))) uint16_t As[2][NA][BM * kRow];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][NA][BN * kRow];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * BM;
  const int64_t n0 = (int64_t)(wg % tiles_n) * BN;
  const float* A = static_cast<const float*>(g.A);
  const int64_t M = g.M, N = g.N, K = g.K;

  // A piece p of this thread: row (tid + 256p) / 8, k quad tid % 8 (the same for every p)
  const int kq = tid & 7;
  const float* arow[AP];
  int cih[AP], ciw[AP];
#pragma unroll
  for (int p = 0; p < AP; ++p) {
    const int64_t m = m0 + ((tid + 256 * p) >> 3);
    arow[p] = nullptr;
    cih[p] = ciw[p] = 0;
    if (m < M) {
      if (AL == A_CONV) {
        const int64_t ow = m % cg.OW;
        const int64_t t = m / cg.OW;
        const int64_t oh = t % cg.OH;
        const int64_t n = t / cg.OH;
        arow[p] = A + n * (int64_t)cg.H * cg.W * cg.C;
        cih[p] = (int)(oh * cg.sh - cg.pt);
        ciw[p] = (int)(ow * cg.sw - cg.pl);
      } else {
        arow[p] = A + m * g.lda;
      }
    }
  }
  // conv: k = 4*kq + tile*BK -> (kh, kw, c), advanced incrementally (C % 4 == 0)
  int kc = 0, kkw = 0, kkh = 0;
  if (AL == A_CONV) {
    const int k = 4 * kq;
    kc = k % cg.C;
    const int t = k / cg.C;
    kkw = t % cg.KW;
    kkh = t / cg.KW;
  }

  // register-staged tiles, two sets: the global loads of tile t+2 are in
  // flight while tile t is computed and tile t+1 is written to LDS
  struct Regs {
    float4 ra[AP];
    uint4 rbh[BP], rbl[X3 ? BP : 1];
  };
  auto load = [&](int64_t k0, Regs& R) {
    float4* ra = R.ra;
    uint4* rbh = R.rbh;
    uint4* rbl = R.rbl;
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int64_t k = k0 + 4 * kq;
      const float* src = nullptr;
      if (AL == A_CONV) {
        const int ih = cih[p] + kkh * cg.dh, iw = ciw[p] + kkw * cg.dw;
        if (arow[p] && k < K && ih >= 0 && ih < cg.H && iw >= 0 && iw < cg.W)
          src = arow[p] + ((int64_t)ih * cg.W + iw) * cg.C + kc;
      } else if (arow[p] && k < K) {
        src = arow[p] + k;
      }
      ra[p] = src ? *reinterpret_cast<const float4*>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (AL == A_CONV) {
      kc += kBK;
      while (kc >= cg.C) {
        kc -= cg.C;
        if (++kkw == cg.KW) {
          kkw = 0;
          ++kkh;
        }
      }
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p;
      const int r = idx >> 2, q = idx & 3;  // row of the tile, 8-bf16 chunk
      const int64_t n = n0 + r;
      const bool ok = n < N;  // k beyond K is zero in the padded image
      const int64_t off = n * Kp + k0 + 8 * q;
      rbh[p] = ok ? *reinterpret_cast<const uint4*>(Bhi + off) : make_uint4(0, 0, 0, 0);
      if (X3) rbl[p] = ok ? *reinterpret_cast<const uint4*>(Blo + off) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int st, const Regs& R) {
    const float4* ra = R.ra;
    const uint4* rbh = R.rbh;
    const uint4* rbl = R.rbl;
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int r = (tid + 256 * p) >> 3;
      uint2 hi, lo;
      if (X3) {
        split4(ra[p], hi, lo);
        *reinterpret_cast<uint2*>(&As[st][1][r * kRow + 4 * kq]) = lo;
      } else {
        hi.x = bf16_bits_rne(ra[p].x) | (bf16_bits_rne(ra[p].y) << 16);
        hi.y = bf16_bits_rne(ra[p].z) | (bf16_bits_rne(ra[p].w) << 16);
      }
      *reinterpret_cast<uint2*>(&As[st][0][r * kRow + 4 * kq]) = hi;
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p;
      const int r = idx >> 2, q = idx & 3;
      *reinterpret_cast<uint4*>(&Bs[st][0][r * kRow + 8 * q]) = rbh[p];
      if (X3) *reinterpret_cast<uint4*>(&Bs[st][NA - 1][r * kRow + 8 * q]) = rbl[X3 ? p : 0];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ktiles = (int)((K + kBK - 1) / kBK);
  const int li = lane & 31, lh = lane >> 5;
  // bf16x3 keeps one register set (its 230-VGPR two-set form measured 7% slower);
  // bf16 prefetches two tiles ahead (1.1-1.4x, scripts/gemm_lab.cpp)
  constexpr bool kDeep = !X3;
  Regs r0, r1;
  load(0, r0);
  store(0, r0);
  if (kDeep && ktiles > 1) load(kBK, r0);
  __syncthreads();
  int cur = 0;
  auto compute = [&]() {
#pragma unroll
    for (int s = 0; s < kBK / 16; ++s) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * (BM / WM) + i * 32 + li;
        ah[i] = *reinterpret_cast<const bf16x8*>(&As[cur][0][r * kRow + 16 * s + 8 * lh]);
        if (X3) al[i] = *reinterpret_cast<const bf16x8*>(&As[cur][NA - 1][r * kRow + 16 * s + 8 * lh]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * (BN / WN) + j * 32 + li;
        bh[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][0][r * kRow + 16 * s + 8 * lh]);
        if (X3) bl[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][NA - 1][r * kRow + 16 * s + 8 * lh]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (X3) {
            // small cross terms first, the dominant hi*hi last
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  };
  // iteration kt: `nxt` holds tile kt+1, `far` receives tile kt+2
  auto step = [&](int kt, Regs& nxt, Regs& far) {
    if (kt + 2 < ktiles) load((int64_t)(kt + 2) * kBK, far);
    compute();
    if (kt + 1 < ktiles) store(cur ^ 1, nxt);
    __syncthreads();
    cur ^= 1;
  };
  if constexpr (kDeep) {
    for (int kt = 0; kt < ktiles; kt += 2) {
      step(kt, r0, r1);
      if (kt + 1 < ktiles) step(kt + 1, r1, r0);
    }
  } else {
    for (int kt = 0; kt < ktiles; ++kt) {
      const bool has_next = kt + 1 < ktiles;
      if (has_next) load((int64_t)(kt + 1) * kBK, r0);
      compute();
      if (has_next) store(cur ^ 1, r0);
      __syncthreads();
      cur ^= 1;
    }
  }

  const float* bias = static_cast<const float*>(g.bias);
  // constant acc indices only (see gemm.hip): cheap epilogue while storing,
  // transcendental activations / absorbed chains in a fix-up loop
  const bool heavy = !(g.act <= ACT_RELU6 && g.epi.n == 0);
  const int cheap_act = heavy ? ACT_NONE : g.act;
  float* Cf = static_cast<float*>(g.C);
  static_for<TN>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int64_t col = n0 + wn * (BN / WN) + j * 32 + li;
    if (col >= N) return;
    const float bv = bias ? bias[col] : 0.f;
    static_for<TM>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const auto v = acc[i][j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= M) continue;
        Cf[row * g.ldc + col] = act_fast(v[r] + bv, cheap_act);
      }
    });
  });
  if (heavy) {
#pragma nounroll
    for (int e = 0; e < TN * TM * 16; ++e) {
      const int j = e / (TM * 16), i = (e / 16) % TM, r = e % 16;
      const int64_t col = n0 + wn * (BN / WN) + j * 32 + li;
      const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (col >= N || row >= M) continue;
      float* p = Cf + row * g.ldc + col;
      *p = epi_apply(g.epi, act_apply(*p, g.act), row, col, N, 0);
    }
  }
}

int64_t padded_k(int64_t K) { return (K + kBK - 1) / kBK * kBK; }

constexpr int kBf16Tiles[4][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}};

template <int AL, bool X3>
void launch_tile(int t, const GemmArgs& g, const Im2colGeom& cg, const uint16_t* bh, const uint16_t* bl, int64_t Kp,
                 hipStream_t s) {
  const int bm = kBf16Tiles[t][0], bn = kBf16Tiles[t][1];
  const int64_t tm = (g.M + bm - 1) / bm, tn = (g.N + bn - 1) / bn;
  TFA_CHECK(tm * tn < (int64_t(1) << 31), "gemm bf16: grid too large");
  dim3 grid((unsigned)(tm * tn));
#define TFA_BF16(BM_, BN_)                                                                                \
  hipLaunchKernelGGL((gemm_bf16_tile<BM_, BN_, 2, 2, AL, X3>), grid, dim3(256), 0, s, g, (int)tm, (int)tn, cg, \
                     bh, bl, Kp)
  switch (t) {
    case 0: TFA_BF16(128, 128); break;
    case 1: TFA_BF16(128, 64); break;
    case 2: TFA_BF16(64, 128); break;
    default: TFA_BF16(64, 64); break;
  }
#undef TFA_BF16
}

int heuristic_tile(const GemmArgs& g) {
  auto blocks = [&](int t) {
    return ((g.M + kBf16Tiles[t][0] - 1) / kBf16Tiles[t][0]) * ((g.N + kBf16Tiles[t][1] - 1) / kBf16Tiles[t][1]);
  };
  int t = g.N <= 64 ? 1 : 0;
  if (blocks(t) < 512) t = (t == 0 && blocks(1) >= 512) ? 1 : (g.N > 64 && blocks(2) >= 512 ? 2 : 3);
  return t;
}

// first launch of a (shape, mode, conv geometry) times the four tiles on the
// caller's stream and keeps the fastest (as the f32 core's tuner; never under
// stream capture; TFA_GEMM_AUTOTUNE=0 keeps the heuristic)
template <int AL, bool X3>
void launch(const GemmArgs& g, const Im2colGeom& cg, const uint16_t* bh, const uint16_t* bl, int64_t Kp,
            hipStream_t s) {
  static std::mutex mu;
  static std::map<std::array<int64_t, 16>, int> cache;
  static const bool tune = [] {
    const char* e = std::getenv("TFA_GEMM_AUTOTUNE");
    return !(e && std::atoi(e) == 0);
  }();
  const std::array<int64_t, 16> key{g.M, g.N, g.K, g.ldc == g.N, cg.H, cg.W, cg.C, cg.KW, cg.OH, cg.OW,
                                    cg.sh, cg.sw, cg.dh, cg.dw, cg.pt, cg.pl};
  int t = heuristic_tile(g);
  bool found = false;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) {
      t = it->second;
      found = true;
    }
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (!found && tune && hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone) {
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess) {
      float best = 1e30f;
      for (int round = 0; round < 2; ++round)
        for (int c = 0; c < 4; ++c) {
          if (kBf16Tiles[c][1] >= 2 * g.N && c != t) continue;  // mostly-padding tile
          if (round == 0) launch_tile<AL, X3>(c, g, cg, bh, bl, Kp, s);
          (void)hipEventRecord(e0, s);
          for (int r = 0; r < 3; ++r) launch_tile<AL, X3>(c, g, cg, bh, bl, Kp, s);
          (void)hipEventRecord(e1, s);
          float ms = 0.f;
          if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms < best) {
            best = ms;
            t = c;
          }
        }
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      std::lock_guard<std::mutex> lk(mu);
      cache[key] = t;
    }
  }
  launch_tile<AL, X3>(t, g, cg, bh, bl, Kp, s);
}

}  // namespace

size_t bf16_workspace_bytes(int mode, int64_t N, int64_t K) {
  const int64_t img = N * padded_k(K) * 2;
  const int64_t aligned = (img + 255) / 256 * 256;
  return static_cast<size_t>(mode == 2 ? 2 * aligned : aligned);
}

bool bf16_gemm_eligible(const GemmArgs& g, bool conv, int64_t conv_c) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (g.batch != 1 || g.ta || !al16(g.A) || g.workspace == nullptr) return false;
  if (conv) return conv_c % 4 == 0;
  return g.lda % 4 == 0 && g.K % 4 == 0;
}

void bf16_gemm_launch(int mode, const GemmArgs& g, bool conv, const Im2colGeom& cg, hipStream_t s) {
  TFA_CHECK(mode == 1 || mode == 2, "gemm bf16: bad mode ", mode);
  const int64_t Kp = padded_k(g.K);
  const int64_t img = g.N * Kp * 2;
  const int64_t aligned = (img + 255) / 256 * 256;
  uint16_t* bh = static_cast<uint16_t*>(g.workspace);
  uint16_t* bl = mode == 2 ? reinterpret_cast<uint16_t*>(static_cast<char*>(g.workspace) + aligned) : nullptr;
  hipLaunchKernelGGL(prep_b, dim3(ew_grid(g.N * Kp)), dim3(256), 0, s, static_cast<const float*>(g.B), g.ldb, g.tb,
                     g.N, g.K, Kp, bh, bl);
  if (conv) {
    if (mode == 2) launch<A_CONV, true>(g, cg, bh, bl, Kp, s);
    else launch<A_CONV, false>(g, cg, bh, bl, Kp, s);
  } else {
    if (mode == 2) launch<A_KCONTIG, true>(g, cg, bh, bl, Kp, s);
    else launch<A_KCONTIG, false>(g, cg, bh, bl, Kp, s);
  }
  TFA_LAUNCH_CHECK("gemm bf16");
}

}  // namespace k
}  // namespace tfa

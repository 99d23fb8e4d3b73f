// The f32 MFMA GEMM / implicit-GEMM conv core shared by gemm.hip (plans,
// autotuner, public entry points) and the launcher translation units
// gemm_f32_<loader>.hip, which instantiate the tile kernels of one A loader
// each (five smaller units compile in parallel instead of one ~10-minute one).
// The kernel design notes are at the top of gemm.hip.
#pragma once

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "gemm_internal.h"
#include "hip_common.h"

namespace tfa {
namespace k {
namespace f32core {

enum ALoad { A_KCONTIG = 0, A_MCONTIG = 1, A_CONV = 2 };

struct ConvGeom {
  int H, W, C, KW, OH, OW, sh, sw, dh, dw, pt, pl;
  FastDivU32 fOW, fOH;  // row -> (n, oh, ow) without an integer divide (M < 2^32)
  bool fast = false;
};

constexpr int kBK = 16;          // k depth of one LDS stage
constexpr int kSplitAlign = 32;  // split-K boundaries (multiple of kBK)

struct F32Plan {
  int cfg;      // index into the tile table
  int bm, bn;
  int splits;
  int64_t k_per_split;
};

// one per A loader and B layout (the loader units); vec: 16-byte loads
void launch_conv(const F32Plan& p, const GemmArgs& g, bool vec, const ConvGeom& cg, hipStream_t s);
void launch_kcontig_b(const F32Plan& p, const GemmArgs& g, bool vec, hipStream_t s);   // B [K][N]
void launch_kcontig_bt(const F32Plan& p, const GemmArgs& g, bool vec, hipStream_t s);  // B [N][K]
void launch_mcontig_b(const F32Plan& p, const GemmArgs& g, bool vec, hipStream_t s);
void launch_mcontig_bt(const F32Plan& p, const GemmArgs& g, bool vec, hipStream_t s);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}



// 16 zero bytes in global memory: the source of a conv padding tap
__device__ __attribute__((aligned(16))) float kZeroPage[4] = {0.f, 0.f, 0.f, 0.f};



// bounds-checked 4-float load (edge tiles): vector when all 4 are valid
__device__ __forceinline__ float4 ld4(const float* p, bool vec, bool ok0, bool ok1, bool ok2, bool ok3) {
  if (vec && ok3) return *reinterpret_cast<const float4*>(p);
  return make_float4(ok0 ? p[0] : 0.f, ok1 ? p[1] : 0.f, ok2 ? p[2] : 0.f, ok3 ? p[3] : 0.f);
}

// unchecked 4-float load (interior tiles)
template <bool VEC>
__device__ __forceinline__ float4 ld4_fast(const float* p) {
  if constexpr (VEC) return *reinterpret_cast<const float4*>(p);
  return make_float4(p[0], p[1], p[2], p[3]);
}

// sched_group_barrier masks (LLVM AMDGPU): MFMA, VMEM read, DS read, DS write
constexpr int kSchedMfma = 0x008, kSchedVmemRead = 0x020, kSchedDsRead = 0x100, kSchedDsWrite = 0x200;

// ops [J, END) of a k-step whose first O1 ops have mask M1 and the rest M2
template <int J, int END, int O1, int M1, int M2>
__device__ __forceinline__ void sched_ops() {
  if constexpr (J < END) {
    __builtin_amdgcn_sched_group_barrier(J < O1 ? M1 : M2, 1, 0);
    sched_ops<J + 1, END, O1, M1, M2>();
  }
}
// a k-step of NM MFMAs and O memory ops: slot I gets ops [I*O/NM, (I+1)*O/NM)
// (rounded up), then one MFMA
template <int I, int NM, int O, int O1, int M1, int M2>
__device__ __forceinline__ void sched_interleave() {
  if constexpr (I < NM) {
    constexpr int lo = (I * O + NM - 1) / NM, hi = ((I + 1) * O + NM - 1) / NM;
    sched_ops<lo, hi, O1, M1, M2>();
    __builtin_amdgcn_sched_group_barrier(kSchedMfma, 1, 0);
    sched_interleave<I + 1, NM, O, O1, M1, M2>();
  }
}

// where output column `col` lives: its column base pointer and row stride
// (one output, or one of the sibling-conv segments)
__device__ __forceinline__ void out_col(const GemmArgs& g, float* Cb, int64_t col, float*& base, int64_t& ld,
                                        int& act) {
  if (g.seg.n == 0) {
    base = Cb + col;
    ld = g.ldc;
    act = g.act;
    return;
  }
  int s = 0;
#pragma unroll
  for (int q = 1; q < kMaxOutSegs; ++q)
    if (q < g.seg.n && col >= g.seg.begin[q]) s = q;
  base = static_cast<float*>(g.seg.ptr[s]) + (col - g.seg.begin[s]);
  ld = g.seg.ldc[s];
  act = g.seg.act[s];
}

// NT = 64 * WM * WN threads: 4-wave blocks (one wave per SIMD per block) or
// 8-wave blocks (two waves per SIMD sharing one LDS tile: a 256x128 / 256x192
// block tile at a 64x64 / 64x96 wave tile, half the global traffic per FLOP of
// a 4-wave 256x64 and half the accumulator registers of a 4-wave 256x128)
template <int BM, int BN, int WM, int WN, int AL, bool TB, bool VEC, int BK>
__global__ __launch_bounds__(64 * WM * WN, (WM * WN == 16 ? 4 : (WM * WN == 8 ? 2 : (BM * BN > 128 * 192 ? 1 : 2))))
void gemm_f32_tile(GemmArgs g, int tiles_m, int tiles_n, ConvGeom cg, int64_t k_per_split, int flags) {
  constexpr int NT = 64 * WM * WN;
  // k-major LDS images. One written with scalar stores (a k-contiguous
  // operand, 4 k rows x 8 m per half-wave store) gets a pitch of 2 mod 32
  // banks: kq = 0..3 land on banks 8*kq + m, all 32 distinct (a pitch of 4 mod
  // 32 put kq 0/2 and 1/3 on one bank: 2-way conflicts, ~15 % of the LDS
  // cycles, profiles/r4_pmc/). Float4-stored images keep a 16-byte pitch.
  constexpr int LDA = AL == A_MCONTIG ? BM + 4 : BM + 2;
  constexpr int LDB = TB ? BN + 2 : BN + 4;
  const int vepi = flags & 1;  // bit 0: vector epilogue
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert((WM * WN == 4 || WM * WN == 8 || WM * WN == 16) && TM >= 1 && TN >= 1,
                "4, 8 or 16 waves, >= one 32x32 tile each");
  static_assert(BK % 8 == 0, "k is read in octets (k-step t: k = 8(t/4) + t%4 + 4 * half)");
  constexpr int KQ = BK / 4;  // float4 pieces along k
  constexpr int APIECES = BM * BK / 4, BPIECES = BN * BK / 4;  // float4 pieces per tile
  constexpr int AP = (APIECES + NT - 1) / NT, BP = (BPIECES + NT - 1) / NT;
  // one LDS buffer: the two A/B stages of the main loop, then (vector
  // epilogue) one 32x32 staging tile per wave (pitch 32: the half-wave row
  // stores and the float4 row reads are both conflict-free; 36 put 2 of 16
  // lanes of a ds_read_b128 group on one bank)
  constexpr int kStage = 32 * 32;
  constexpr int kMain = 2 * BK * (LDA + LDB), kEpi = (NT / 64) * kStage;
  __shared__ __attribute__((aligned(16))) float smem[kMain > kEpi ? kMain : kEpi];
  float(&As)[2][BK][LDA] = *reinterpret_cast<float(*)[2][BK][LDA]>(smem);
  float(&Bs)[2][BK][LDB] = *reinterpret_cast<float(*)[2][BK][LDB]>(smem + 2 * BK * LDA);

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * BM;
  const int64_t n0 = (int64_t)(wg % tiles_n) * BN;
  const int64_t bz = blockIdx.y;  // batch
  const float* A = static_cast<const float*>(g.A) + bz * g.strideA;
  const float* B = static_cast<const float*>(g.B) + bz * g.strideB;
  const int64_t M = g.M, N = g.N, K = g.K;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = min(K, kbeg + k_per_split);
  constexpr bool v = VEC;

  // conv: per A piece, output pixel -> (image base, ih0, iw0)
  int64_t cbase[AP];
  int cih[AP], ciw[AP];
  if (AL == A_CONV) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int64_t m = m0 + (tid + NT * p) / KQ;
      cbase[p] = -1;
      cih[p] = ciw[p] = 0;
      if (m < M) {
        int64_t ow, oh, n;
        if (cg.fast) {  // the 64-bit divide sequence is ~100 VALU ops per piece
          const uint32_t m32 = (uint32_t)m, t = fdiv(m32, cg.fOW), q = fdiv(t, cg.fOH);
          ow = m32 - t * (uint32_t)cg.OW;
          oh = t - q * (uint32_t)cg.OH;
          n = q;
        } else {
          ow = m % cg.OW;
          const int64_t t = m / cg.OW;
          oh = t % cg.OH;
          n = t / cg.OH;
        }
        cbase[p] = n * (int64_t)cg.H * cg.W * cg.C;
        cih[p] = (int)(oh * cg.sh - cg.pt);
        ciw[p] = (int)(ow * cg.sw - cg.pl);
      }
    }
  }

  // vec conv: this thread's A k-offset within a tile is fixed (4 * (tid % KQ)), so the
  // k -> (kh, kw, c) split is computed once and advanced by BK per tile (no divides in the loop)
  int kc = 0, kkw = 0, kkh = 0;
  if (AL == A_CONV && VEC) {
    const int k = (int)(kbeg + 4 * (tid % KQ));  // K < 2^31: 32-bit divides
    kc = k % cg.C;
    const int t = k / cg.C;
    kkw = t % cg.KW;
    kkh = t / cg.KW;
  }
  // scalar conv (C % 4 != 0, e.g. RGB input): the same incremental split per
  // element of the thread's 4 k's
  int sc[4] = {0, 0, 0, 0}, skw[4] = {0, 0, 0, 0}, skh[4] = {0, 0, 0, 0};
  if (AL == A_CONV && !VEC) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = (int)(kbeg + 4 * (tid % KQ) + j);
      sc[j] = k % cg.C;
      const int t = k / cg.C;
      skw[j] = t % cg.KW;
      skh[j] = t / cg.KW;
    }
  }

  // loaded tiles stay float4 until the LDS store (no register shuffles, so no
  // early vmcnt wait: the global loads overlap the MFMAs of the current tile)
  float4 ra[AP], rb[BP];
  // CHECK=false: the block's tile lies fully inside M, N and its K range, so
  // loads are unconditional (no exec-mask branches in the hot loop); only
  // edge blocks take the bounds-checked path
  auto load = [&](int64_t k0, auto chk) {
    constexpr bool CHECK = decltype(chk)::value;
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + NT * p;
      if (APIECES % NT != 0 && idx >= APIECES) break;
      if (AL == A_MCONTIG) {
        const int kr = idx / (BM / 4), mq = idx % (BM / 4);
        const int64_t gk = k0 + kr, gm = m0 + 4 * mq;
        if constexpr (CHECK) {
          const bool kk = gk < kend;
          ra[p] = ld4(A + gk * g.lda + gm, v, kk && gm < M, kk && gm + 1 < M, kk && gm + 2 < M, kk && gm + 3 < M);
        } else {
          ra[p] = ld4_fast<VEC>(A + gk * g.lda + gm);
        }
      } else {
        const int row = idx / KQ, kq = idx % KQ;
        const int64_t gm = m0 + row, gk = k0 + 4 * kq;
        if (AL == A_KCONTIG) {
          if constexpr (CHECK) {
            const bool mm = gm < M;
            ra[p] = ld4(A + gm * g.lda + gk, v, mm && gk < kend, mm && gk + 1 < kend, mm && gk + 2 < kend,
                        mm && gk + 3 < kend);
          } else {
            ra[p] = ld4_fast<VEC>(A + gm * g.lda + gk);
          }
        } else if (v) {  // conv, C % 4 == 0: the 4 k's share (kh, kw) = incremental (kc, kkw, kkh)
          const int ih = cih[p] + kkh * cg.dh, iw = ciw[p] + kkw * cg.dw;
          const bool inb = cbase[p] >= 0 && (!CHECK || gk < kend) && ih >= 0 && ih < cg.H && iw >= 0 &&
                           iw < cg.W;
          // padding taps read a zero page instead of being zeroed by selects
          // on the loaded value (no VALU on the data, which also keeps the
          // compiler from waiting for the load before the LDS store);
          // in-image offset in 32 bits (H*W*C < 2^30, conv2d_nhwc): no 64-bit multiplies per piece
          const float* src = inb ? A + cbase[p] + ((ih * cg.W + iw) * cg.C + kc) : kZeroPage;
          ra[p] = *reinterpret_cast<const float4*>(src);
        } else {
          float sv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ih = cih[p] + skh[j] * cg.dh, iw = ciw[p] + skw[j] * cg.dw;
            const bool inb = cbase[p] >= 0 && gk + j < kend && ih >= 0 && ih < cg.H && iw >= 0 && iw < cg.W;
            const float* src = inb ? A + cbase[p] + ((ih * cg.W + iw) * cg.C + sc[j]) : kZeroPage;
            sv[j] = *src;
          }
          ra[p] = make_float4(sv[0], sv[1], sv[2], sv[3]);
        }
      }
    }
    if (AL == A_CONV && VEC) {
      kc += BK;
      while (kc >= cg.C) {
        kc -= cg.C;
        if (++kkw == cg.KW) {
          kkw = 0;
          ++kkh;
        }
      }
    }
    if (AL == A_CONV && !VEC) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sc[j] += BK;
        while (sc[j] >= cg.C) {
          sc[j] -= cg.C;
          if (++skw[j] == cg.KW) {
            skw[j] = 0;
            ++skh[j];
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + NT * p;
      if (BPIECES % NT != 0 && idx >= BPIECES) break;
      if (!TB) {  // B [K][N]
        const int kr = idx / (BN / 4), nq = idx % (BN / 4);
        const int64_t gk = k0 + kr, gn = n0 + 4 * nq;
        if constexpr (CHECK) {
          const bool kk = gk < kend;
          rb[p] = ld4(B + gk * g.ldb + gn, v, kk && gn < N, kk && gn + 1 < N, kk && gn + 2 < N, kk && gn + 3 < N);
        } else {
          rb[p] = ld4_fast<VEC>(B + gk * g.ldb + gn);
        }
      } else {  // B [N][K]
        const int col = idx / KQ, kq = idx % KQ;
        const int64_t gn = n0 + col, gk = k0 + 4 * kq;
        if constexpr (CHECK) {
          const bool nn = gn < N;
          rb[p] = ld4(B + gn * g.ldb + gk, v, nn && gk < kend, nn && gk + 1 < kend, nn && gk + 2 < kend,
                      nn && gk + 3 < kend);
        } else {
          rb[p] = ld4_fast<VEC>(B + gn * g.ldb + gk);
        }
      }
    }
  };
  auto store = [&](int st) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + NT * p;
      if (APIECES % NT != 0 && idx >= APIECES) break;
      if (AL == A_MCONTIG) {
        const int kr = idx / (BM / 4), mq = idx % (BM / 4);
        *reinterpret_cast<float4*>(&As[st][kr][4 * mq]) = ra[p];
      } else {
        const int row = idx / KQ, kq = idx % KQ;
        As[st][4 * kq + 0][row] = ra[p].x;
        As[st][4 * kq + 1][row] = ra[p].y;
        As[st][4 * kq + 2][row] = ra[p].z;
        As[st][4 * kq + 3][row] = ra[p].w;
      }
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + NT * p;
      if (BPIECES % NT != 0 && idx >= BPIECES) break;
      if (!TB) {
        const int kr = idx / (BN / 4), nq = idx % (BN / 4);
        *reinterpret_cast<float4*>(&Bs[st][kr][4 * nq]) = rb[p];
      } else {
        const int col = idx / KQ, kq = idx % KQ;
        Bs[st][4 * kq + 0][col] = rb[p].x;
        Bs[st][4 * kq + 1][col] = rb[p].y;
        Bs[st][4 * kq + 2][col] = rb[p].z;
        Bs[st][4 * kq + 3][col] = rb[p].w;
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ktiles = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;
  // instructions per tile, for the interleaved schedule: global loads (a
  // non-vector piece is 4 scalar loads), LDS writes (a k-major image of a
  // k-contiguous operand is 4 scalar stores per piece), LDS reads per k-step
  constexpr int S = BK / 2, NM = TM * TN, R = TM + TN;
  constexpr int L = (VEC ? 1 : 4) * (AP + BP);
  constexpr int W = AP * (AL == A_MCONTIG ? 1 : 4) + BP * (TB ? 4 : 1);
  auto mainloop = [&](auto chk) __attribute__((always_inline)) {
    if (ktiles > 0) {
      load(kbeg, chk);
      store(0);
    }
    __syncthreads();
    int cur = 0;
    // One k tile. The next tile's global loads (first k-step), the next
    // k-step's LDS operand reads (every k-step) and the next stage's LDS
    // writes (last k-step) are spread between the MFMAs with
    // sched_group_barrier instead of being issued as a block: each wave keeps
    // the MFMA pipe fed while its memory ops are in flight (measured +5% on
    // 128x128, and what makes the 256x128 tile pay; scripts/bigtile_lab.hip).
    // The last tile is peeled off so the loop body has no branch.
    auto tile = [&](int64_t knext, auto more) {
      constexpr bool NEXT = decltype(more)::value;
      float a[2][TM], b[2][TN];
      // k-step t pairs k = 8(t/4) + t%4 (lanes 0-31) with the same k + 4
      // (lanes 32-63): the order of the g2 core's quad fragments
      // (gemm_g2_core.h), so every f32 tile sums identically
      auto rd = [&](int buf, int t) {
        const int kr = 8 * (t >> 2) + (t & 3) + 4 * (lane >> 5);
#pragma unroll
        for (int i = 0; i < TM; ++i) a[buf][i] = As[cur][kr][wm * (BM / WM) + i * 32 + (lane & 31)];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[buf][j] = Bs[cur][kr][wn * (BN / WN) + j * 32 + (lane & 31)];
      };
      rd(0, 0);
      __builtin_amdgcn_sched_group_barrier(kSchedDsRead, R, 0);
      if constexpr (NEXT) load(knext, chk);
#pragma unroll
      for (int kk = 0; kk < S; ++kk) {
        if (kk + 1 < S) rd((kk + 1) & 1, kk + 1);
        if (NEXT && kk == S - 1) store(cur ^ 1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk & 1][i], b[kk & 1][j], acc[i][j], 0, 0, 0);
        if (kk == 0 && NEXT)
          sched_interleave<0, NM, L + R, L, kSchedVmemRead, kSchedDsRead>();
        else if (kk == S - 1 && NEXT)
          sched_interleave<0, NM, W, W, kSchedDsWrite, kSchedDsWrite>();
        else if (kk + 1 < S)
          sched_interleave<0, NM, R, R, kSchedDsRead, kSchedDsRead>();
        else
          __builtin_amdgcn_sched_group_barrier(kSchedMfma, NM, 0);
      }
      __syncthreads();
      cur ^= 1;
    };
    for (int kt = 0; kt + 1 < ktiles; ++kt) tile(kbeg + (int64_t)(kt + 1) * BK, std::true_type{});
    if (ktiles > 0) tile(0, std::false_type{});
  };
  const bool interior = m0 + BM <= M && n0 + BN <= N && (kend - kbeg) % BK == 0;
  if (interior)
    mainloop(std::false_type{});
  else
    mainloop(std::true_type{});

  // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float* ws = static_cast<float*>(g.workspace);
  const float* bias = static_cast<const float*>(g.bias);
  // Accumulators are only ever indexed with constants (static_for), so they stay
  // in registers. The cheap epilogue (bias + none/ReLU/ReLU6) is applied while
  // storing; a transcendental activation or an absorbed elementwise chain is
  // applied afterwards by a runtime loop over the elements this thread just
  // wrote (re-read from its own stores: small code, no dynamic acc index).
  const bool heavy = !ws && !(g.act <= ACT_RELU6 && g.epi.n == 0);
  float* Cb = static_cast<float*>(g.C) + bz * g.strideC;
  if (vepi) {
    // Vector epilogue (single pass, cheap activation, 16-byte aligned rows):
    // each 32x32 accumulator tile goes through a wave-private LDS tile and
    // leaves as float4 rows, 4 global_store_dwordx4 per lane instead of 16
    // scalar stores (the scalar stores cost up to 15 % of a conv layer;
    // profiles/r3_epilogue/). LDS is free: the main loop ended on a barrier,
    // and each wave only touches its own staging tile (in-order LDS per wave).
    float* st = smem + wave * kStage;
    static_for<TN>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      static_for<TM>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        const f32x16 v = acc[i][j];
#pragma unroll
        for (int r = 0; r < 16; ++r) st[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = v[r];
        const int64_t col = n0 + wn * (BN / WN) + j * 32 + 4 * (lane & 7);
        if (col < N) {
          float* cbase;
          int64_t cld;
          int cact;
          out_col(g, Cb, col, cbase, cld, cact);
          float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (bias) bv = make_float4(bias[col], bias[col + 1], bias[col + 2], bias[col + 3]);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int rr = 8 * q + (lane >> 3);
            const int64_t row = m0 + wm * (BM / WM) + i * 32 + rr;
            float4 o = *reinterpret_cast<const float4*>(&st[rr * 32 + 4 * (lane & 7)]);
            o.x = act_fast(o.x + bv.x, cact);
            o.y = act_fast(o.y + bv.y, cact);
            o.z = act_fast(o.z + bv.z, cact);
            o.w = act_fast(o.w + bv.w, cact);
            if (row < M) *reinterpret_cast<float4*>(cbase + row * cld) = o;
          }
        }
      });
    });
    return;
  }
  static_for<TN>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int64_t col = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
    if (col >= N) return;
    const float bv = (!ws && bias) ? bias[col] : 0.f;
    float* cbase;
    int64_t cld;
    int cact;
    out_col(g, Cb, col, cbase, cld, cact);
    if (heavy) cact = ACT_NONE;
    static_for<TM>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const f32x16 v = acc[i][j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= M) continue;
        if (ws)  // split-K partial slab [split][batch][M][N]
          ws[(((int64_t)blockIdx.z * gridDim.y + bz) * M + row) * N + col] = v[r];
        else
          cbase[row * cld] = act_fast(v[r] + bv, cact);
      }
    });
  });
  if (heavy) {
#pragma nounroll
    for (int e = 0; e < TN * TM * 16; ++e) {
      const int j = e / (TM * 16), i = (e / 16) % TM, r = e % 16;
      const int64_t col = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
      const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (col >= N || row >= M) continue;
      float* cbase;
      int64_t cld;
      int cact;
      out_col(g, Cb, col, cbase, cld, cact);
      float* p = cbase + row * cld;
      *p = epi_apply(g.epi, act_apply(*p, cact), row, col, N, bz * M * N);
    }
  }
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// the vector epilogue applies: single pass, bias + none/ReLU/ReLU6 only, and
// every output row segment of 4 columns is 16-byte aligned in one output
int vector_epilogue(const GemmArgs& g) {
  static const bool off = [] {
    const char* e = std::getenv("TFA_GEMM_VEC_EPILOGUE");
    return e && std::atoi(e) == 0;
  }();
  if (off || g.workspace || g.act > ACT_RELU6 || g.epi.n != 0 || g.N % 4 != 0) return 0;
  if (g.seg.n == 0) {
    if (!al16(g.C) || g.ldc % 4 != 0 || (g.batch > 1 && g.strideC % 4 != 0)) return 0;
  } else {
    for (int q = 0; q < g.seg.n; ++q)
      if (g.seg.begin[q] % 4 != 0 || g.seg.ldc[q] % 4 != 0 || !al16(g.seg.ptr[q]) || g.seg.act[q] > ACT_RELU6)
        return 0;
    if (g.seg.begin[g.seg.n] % 4 != 0) return 0;
  }
  return 1;
}

template <int AL, bool TB, bool VEC>
void launch_cfg(const F32Plan& p, const GemmArgs& g, const ConvGeom& cg, hipStream_t s) {
  const int vepi = p.splits == 1 ? vector_epilogue(g) : 0;
  const int64_t tm = (g.M + p.bm - 1) / p.bm, tn = (g.N + p.bn - 1) / p.bn;
  TFA_CHECK(tm * tn < (int64_t(1) << 31), "gemm: grid too large");
  TFA_CHECK(g.batch <= 65535 && p.splits <= 65535, "gemm: batch/splits too large");
  dim3 grid((unsigned)(tm * tn), (unsigned)g.batch, (unsigned)p.splits);
#define TFA_LAUNCH_TILE_BK(BM_, BN_, WM_, WN_, BK_)                                                         \
  hipLaunchKernelGGL((gemm_f32_tile<BM_, BN_, WM_, WN_, AL, TB, VEC, BK_>), grid, dim3(64 * WM_ * WN_), 0, s, g, \
                     (int)tm, (int)tn, cg, p.k_per_split, vepi)
#define TFA_LAUNCH_TILE(BM_, BN_, WM_, WN_) TFA_LAUNCH_TILE_BK(BM_, BN_, WM_, WN_, kBK)
  switch (p.cfg) {
    case 0: TFA_LAUNCH_TILE(128, 128, 2, 2); break;
    case 1: TFA_LAUNCH_TILE(128, 64, 2, 2); break;
    case 2: TFA_LAUNCH_TILE(64, 128, 2, 2); break;
    case 3: TFA_LAUNCH_TILE(64, 64, 2, 2); break;
    case 4: TFA_LAUNCH_TILE(128, 32, 4, 1); break;
    case 5: TFA_LAUNCH_TILE(128, 96, 4, 1); break;
    case 6: TFA_LAUNCH_TILE(128, 192, 2, 2); break;
    case 7: TFA_LAUNCH_TILE(128, 160, 4, 1); break;
    case 8: TFA_LAUNCH_TILE(64, 192, 2, 2); break;
    case 9: TFA_LAUNCH_TILE(256, 128, 2, 2); break;
    // tall tiles for narrow-N convs: 4 waves stacked along M, so each wave
    // runs 2 x TN MFMAs per k-step instead of 1 x TN (128x32 / 128x64 / 128x96)
    case 10: TFA_LAUNCH_TILE(256, 64, 4, 1); break;
    case 11: TFA_LAUNCH_TILE(256, 32, 4, 1); break;
    case 12: TFA_LAUNCH_TILE(256, 96, 4, 1); break;
    // 8-wave blocks: two waves per SIMD share the block's LDS tile
    case 13: TFA_LAUNCH_TILE(256, 128, 4, 2); break;
    case 14: TFA_LAUNCH_TILE(256, 96, 8, 1); break;
    case 15: TFA_LAUNCH_TILE(128, 128, 2, 4); break;
    case 16: TFA_LAUNCH_TILE(128, 192, 4, 2); break;
    case 17: TFA_LAUNCH_TILE(256, 64, 8, 1); break;
    case 18: TFA_LAUNCH_TILE(128, 64, 4, 2); break;
    case 19: TFA_LAUNCH_TILE(128, 256, 4, 2); break;
    case 20: TFA_LAUNCH_TILE(256, 256, 4, 2); break;
    default: TFA_LAUNCH_TILE(256, 256, 4, 4); break;
  }
#undef TFA_LAUNCH_TILE
#undef TFA_LAUNCH_TILE_BK
}

}  // namespace
}  // namespace f32core
}  // namespace k
}  // namespace tfa

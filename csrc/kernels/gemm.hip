// f32 MFMA GEMM + implicit-GEMM Conv2D for gfx950 (CDNA4).
//
// v_mfma_f32_32x32x2_f32 (exact f32: gfx950 has no xf32). One kernel
// template over the block tile BMxBN (4 waves arranged WMxWN, each wave
// owning (BM/WM)x(BN/WN) as 32x32 MFMA tiles) so the tile can follow the
// problem: 128x128 for the big tall-skinny GEMMs, 128x64 / 64x64 / 128x32
// for narrow conv layers, split-K for grids that cannot fill 256 CUs.
//
//  * k-major LDS images (As[k][m], Bs[k][n]): every MFMA operand read is 32
//    consecutive floats per half-wave (conflict-free ds_read_b32);
//  * two LDS stages; the next K tile's global loads are issued during the
//    current tile's MFMAs (register-staged pipeline, one barrier per tile),
//    with every memory op interleaved between MFMAs (sched_group_barrier);
//  * bias + ReLU/ReLU6 fused into the epilogue (or into the split-K reducer);
//  * XCD-aware bijective block->tile remap: blocks sharing an A row panel
//    run on one XCD and share its L2.
// Conv2D (NHWC, filter HWIO) uses the same core with an im2col-on-the-fly A
// loader: A[m = (n,oh,ow)][k = (kh,kw,c)], B = filter viewed as [KH*KW*C, OC];
// 1x1 stride-1 convs are plain GEMMs over x viewed as [N*H*W, C].
#include <array>
#include <atomic>
#include <cmath>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "gemm_internal.h"
#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}


enum ALoad { A_KCONTIG = 0, A_MCONTIG = 1, A_CONV = 2 };

// 16 zero bytes in global memory: the source of a conv padding tap
__device__ __attribute__((aligned(16))) float kZeroPage[4] = {0.f, 0.f, 0.f, 0.f};

struct ConvGeom {
  int H, W, C, KW, OH, OW, sh, sw, dh, dw, pt, pl;
  FastDivU32 fOW, fOH;  // row -> (n, oh, ow) without an integer divide (M < 2^32)
  bool fast = false;
};

constexpr int kBK = 16;          // k depth of one LDS stage
constexpr int kSplitAlign = 32;  // split-K boundaries (multiple of kBK)

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
__global__ __launch_bounds__(64 * WM * WN, (WM * WN == 8 ? 2 : (BM * BN > 128 * 192 ? 1 : 2)))
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
  static_assert((WM * WN == 4 || WM * WN == 8) && TM >= 1 && TN >= 1, "4 or 8 waves, >= one 32x32 tile each");
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
      auto rd = [&](int buf, int kk) {
        const int kr = kk + (lane >> 5);
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
        if (kk + 1 < S) rd((kk + 1) & 1, 2 * (kk + 1));
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

// split-K combine: fixed summation order over the splits (deterministic)
__global__ __launch_bounds__(256) void splitk_reduce(const float* __restrict__ ws, GemmArgs g, int splits) {
  const int64_t M = g.M, N = g.N;
  const int64_t total = g.batch * M * N;
  const float* bias = static_cast<const float*>(g.bias);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += ws[z * total + i];
    const int64_t col = i % N;
    const int64_t row = (i / N) % M;
    const int64_t b = i / (M * N);
    if (bias) s += bias[col];
    float* cbase;
    int64_t cld;
    int cact;
    out_col(g, static_cast<float*>(g.C) + b * g.strideC, col, cbase, cld, cact);
    cbase[row * cld] = epi_apply(g.epi, act_apply(s, cact), row, col, N, b * M * N);
  }
}

// ------------------------------------------------------------------ tile choice
struct F32Plan {
  int cfg;      // index into the tile table
  int bm, bn;
  int splits;
  int64_t k_per_split;
};

// measured (scripts/gemm_bench.py, scripts/bigtile_lab.hip): 128x256 and BK=32 variants were slower on every
// shape; 256x128 (wave tile 128x64) pays only with the interleaved schedule (+8-12% on big GEMMs) and
// loses on grids of a few hundred blocks
// {BM, BN}; the N-widths 96/160/192 fit Inception-style channel counts without
// padding a 128-wide tile (a 128 tile on N=96 computes 25% zeros)
// 13-15 are 8-wave blocks (512 threads). Measured (scripts/tile_ab.sh,
// profiles/r3_tiles/): the 8-wave 256x128 wins 4096^3 (137.5 TF vs 133.6 for
// 128x128) and ties the headline 2.5Mx512x512; 256x96 (8x1) and 128x128 (2x4)
// win some Inception convs. 256x192, a BK=32 256x128 and BK=32 128x64 /
// 128x32 (one whole C=32 filter tap per k tile) never won.
// 16-18 are 8-wave versions of narrow conv tiles: 128x192 as 4x2 waves
// (each 32x96, the wave tile of 64x192), 256x64 as 8x1 (each 32x64) and
// 128x64 as 4x2 (each 32x32, the wave tile of 64x64): the block's A and B
// tiles are shared by twice the waves (less global and LDS traffic per FLOP)
// at the same wave tile. 256x160 as 8x1 never won (profiles/r4_tiles/).
constexpr int kNumTiles = 19;
constexpr int kTiles[kNumTiles][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}, {128, 32},
                                      {128, 96}, {128, 192}, {128, 160}, {64, 192}, {256, 128},
                                      {256, 64}, {256, 32}, {256, 96}, {256, 128}, {256, 96},
                                      {128, 128}, {128, 192}, {256, 64}, {128, 64}};

int64_t tile_blocks(int c, int64_t M, int64_t N, int64_t batch) {
  return ((M + kTiles[c][0] - 1) / kTiles[c][0]) * ((N + kTiles[c][1] - 1) / kTiles[c][1]) * batch;
}

// the launch plan of tile `cfg`: split K when the grid is under one block per CU
F32Plan plan_for(int cfg, int64_t M, int64_t N, int64_t K, int64_t batch) {
  F32Plan p{cfg, kTiles[cfg][0], kTiles[cfg][1], 1, K};
  const int64_t nb = tile_blocks(cfg, M, N, batch);
  if (nb < 256 && K >= 256) {  // each split >= 128 deep
    int64_t s = std::min<int64_t>((512 + nb - 1) / nb, K / 128);
    s = std::max<int64_t>(1, std::min<int64_t>(s, 16));
    int64_t kps = ((K + s - 1) / s + kSplitAlign - 1) / kSplitAlign * kSplitAlign;
    p.splits = (int)((K + kps - 1) / kps);
    p.k_per_split = kps;
  }
  return p;
}

// forced f32 tile (-1 = heuristic + autotuner): TFA_GEMM_TILE or set_gemm_tile()
std::atomic<int>& forced_tile() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_GEMM_TILE");
    const int t = e ? std::atoi(e) : -1;
    return t >= 0 && t < kNumTiles ? t : -1;
  }());
  return v;
}
int tile_env() { return forced_tile().load(); }

// Heuristic plan (also the fallback of the autotuner and what sizes the split-K workspace)
F32Plan plan_f32(int64_t M, int64_t N, int64_t K, int64_t batch) {
  // narrow N picks a narrow tile (a 128-wide tile on N=32 wastes 3/4 of the MFMAs)
  int cfg = N <= 32 ? 4 : (N <= 64 ? 1 : 0);
  // big GEMMs: 256x64 with the 4 waves stacked along M (each 64x64, B fragments shared);
  // measured best on 2.5Mx512x512, 262kx512x512, 4096^3 and 8192x1024^2 (scripts/bigtile_lab.hip)
  if (cfg == 0 && tile_blocks(10, M, N, batch) >= 512) cfg = 10;
  // too few blocks to fill 256 CUs twice: shrink the tile
  if (tile_blocks(cfg, M, N, batch) < 512) {
    if (cfg == 0) cfg = N > 96 ? 2 : 3;
    else if (cfg == 1) cfg = 3;
  }
  if (tile_env() >= 0) cfg = tile_env();  // tuning override
  return plan_for(cfg, M, N, K, batch);
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
    default: TFA_LAUNCH_TILE(128, 64, 4, 2); break;
  }
#undef TFA_LAUNCH_TILE
#undef TFA_LAUNCH_TILE_BK
}

void launch_plan(const F32Plan& p, const GemmArgs& g, int al, bool vec, const ConvGeom& cg, hipStream_t s) {
#define TFA_VEC(AL_, TB_) \
  (vec ? launch_cfg<AL_, TB_, true>(p, g, cg, s) : launch_cfg<AL_, TB_, false>(p, g, cg, s))
  if (al == A_CONV) TFA_VEC(A_CONV, false);
  else if (al == A_KCONTIG && !g.tb) TFA_VEC(A_KCONTIG, false);
  else if (al == A_KCONTIG) TFA_VEC(A_KCONTIG, true);
  else if (!g.tb) TFA_VEC(A_MCONTIG, false);
  else TFA_VEC(A_MCONTIG, true);
#undef TFA_VEC
}

// ---- tile autotuner. The best tile depends on the grid the shape makes (an
// Inception 12x12 conv runs 35% faster on 64x64 tiles than on 128x128, the
// 10M-row headline GEMM is fastest on 128x128), so the first launch of a new
// (shape, loader) times the single-pass tiles on the caller's stream and keeps
// the fastest. Split-K shapes keep the heuristic plan (the summation order, and
// so the result bits, never depend on a timing). Never during stream capture.
// TFA_GEMM_AUTOTUNE=0 disables it; TFA_GEMM_TILE=<cfg> forces a tile.
using TuneKey = std::array<int64_t, 20>;
std::mutex& tune_mu() {
  static std::mutex m;
  return m;
}
std::map<TuneKey, int>& tune_cache() {
  static std::map<TuneKey, int> c;
  return c;
}
bool autotune_on() {
  static const bool v = [] {
    const char* e = std::getenv("TFA_GEMM_AUTOTUNE");
    return !(e && std::atoi(e) == 0);
  }();
  return v && tile_env() < 0;
}

F32Plan tuned_plan(const F32Plan& heur, const GemmArgs& g0, int al, bool vec, const ConvGeom& cg, hipStream_t s) {
  GemmArgs g = g0;
  g.workspace = nullptr;  // single-pass candidates only (a workspace would select the split-K epilogue)
  const TuneKey key{g.M, g.N, g.K, g.batch, al, g.tb, vec, cg.H, cg.W, cg.C, cg.KW, cg.OH, cg.OW,
                    cg.sh, cg.sw, cg.dh, cg.dw, cg.pt, cg.pl, (g.ldc == g.N) + 2 * g.seg.n};
  {
    std::lock_guard<std::mutex> lk(tune_mu());
    auto it = tune_cache().find(key);
    if (it != tune_cache().end()) return plan_for(it->second, g.M, g.N, g.K, g.batch);
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return heur;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return heur;
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return heur;
  }
  // Three rounds over the candidates (interleaved, so clock drift hits every
  // tile alike); a candidate's time is its best round, each round >= ~1 ms of
  // launches (a 3-launch round of a 0.3 ms conv was noisy enough to keep a
  // tile 3-5 % off the best; profiles/r3_tiles/)
  int reps = 3;
  {
    launch_plan(heur, g, al, vec, cg, s);  // warm
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < 3; ++r) launch_plan(heur, g, al, vec, cg, s);
    (void)hipEventRecord(e1, s);
    float ms = 0.f;
    if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms > 0.f)
      reps = std::max(3, std::min(16, (int)std::ceil(1.0f / (ms / 3))));
  }
  float cand_ms[kNumTiles];
  for (int c = 0; c < kNumTiles; ++c) cand_ms[c] = 1e30f;
  for (int round = 0; round < 3; ++round) {
    for (int c = 0; c < kNumTiles; ++c) {
      const F32Plan q = plan_for(c, g.M, g.N, g.K, g.batch);
      if (q.splits != 1) continue;
      if (c != heur.cfg && kTiles[c][1] >= 2 * g.N && kTiles[c][1] > 32) continue;  // mostly-padding tile
      if (round == 0) launch_plan(q, g, al, vec, cg, s);  // warm
      (void)hipEventRecord(e0, s);
      for (int r = 0; r < reps; ++r) launch_plan(q, g, al, vec, cg, s);
      (void)hipEventRecord(e1, s);
      float ms = 0.f;
      if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) continue;
      cand_ms[c] = std::min(cand_ms[c], ms / reps);
    }
  }
  int best = heur.cfg;
  for (int c = 0; c < kNumTiles; ++c)
    if (cand_ms[c] < cand_ms[best]) best = c;
  static const bool log = std::getenv("TFA_GEMM_TUNE_LOG") != nullptr;
  if (log) {
    std::fprintf(stderr, "[gemm tune] M=%lld N=%lld K=%lld al=%d conv=%dx%dx%d heur=%d best=%d |",
                 (long long)g.M, (long long)g.N, (long long)g.K, al, cg.H, cg.W, cg.C, heur.cfg, best);
    for (int c = 0; c < kNumTiles; ++c)
      if (cand_ms[c] < 1e29f) std::fprintf(stderr, " %d:%.4f", c, cand_ms[c]);
    std::fprintf(stderr, "\n");
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  TFA_LAUNCH_CHECK("gemm autotune");
  {
    std::lock_guard<std::mutex> lk(tune_mu());
    tune_cache()[key] = best;
  }
  return plan_for(best, g.M, g.N, g.K, g.batch);
}

void run_f32(const GemmArgs& g0, int al, bool vec, const ConvGeom& cg, hipStream_t s) {
  F32Plan p = plan_f32(g0.M, g0.N, g0.K, g0.batch);
  if (p.splits == 1 && autotune_on()) p = tuned_plan(p, g0, al, vec, cg, s);
  GemmArgs g = g0;
  if (p.splits > 1) {
    TFA_CHECK(g0.workspace != nullptr, "gemm: split-K needs a workspace (gemm_workspace_bytes)");
  } else {
    g.workspace = nullptr;
  }
  launch_plan(p, g, al, vec, cg, s);
  if (p.splits > 1) {
    int64_t total = g.batch * g.M * g.N;
    hipLaunchKernelGGL(splitk_reduce, dim3(ew_grid(total)), dim3(256), 0, s, static_cast<const float*>(g.workspace), g,
                       p.splits);
  }
}

size_t f32_ws_bytes(int64_t M, int64_t N, int64_t K, int64_t batch) {
  F32Plan p = plan_f32(M, N, K, batch);
  return p.splits > 1 ? static_cast<size_t>(p.splits) * batch * M * N * sizeof(float) : 0;
}

bool conv_is_pointwise(const ConvArgs& a) {
  return a.KH == 1 && a.KW == 1 && a.sh == 1 && a.sw == 1 && a.pad_t == 0 && a.pad_l == 0 &&
         a.OH == a.H && a.OW == a.W;
}

std::atomic<int>& precision_state() {
  static std::atomic<int> mode([] {
    const char* e = std::getenv("TFA_PRECISION");
    if (!e) return 0;
    if (!std::strcmp(e, "bf16")) return 1;
    if (!std::strcmp(e, "bf16x3")) return 2;
    return 0;
  }());
  return mode;
}

// bf16 paths: batch 1, 16-byte A rows (K % 4 / C % 4), no transposed A
bool bf16_candidate(const GemmArgs& g) {
  return f32_precision() != 0 && g.batch == 1 && !g.ta && g.lda % 4 == 0 && g.K % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(g.A) & 15) == 0;
}

GemmArgs conv_as_gemm(const ConvArgs& a) {
  GemmArgs g{};
  g.M = a.N * a.OH * a.OW;
  g.N = a.OC;
  g.K = a.KH * a.KW * a.C;
  g.A = a.x; g.lda = a.C; g.strideA = 0;
  g.B = a.w; g.ldb = a.OC; g.strideB = 0;
  g.C = a.y; g.ldc = a.ldc > 0 ? a.ldc : a.OC; g.strideC = 0;
  g.ta = false; g.tb = false;
  g.bias = a.bias;
  g.act = a.act;
  g.batch = 1;
  g.workspace = a.workspace;
  g.epi = a.epi;
  g.seg = a.seg;
  return g;
}

}  // namespace

void set_gemm_tile(int cfg) {
  TFA_CHECK(cfg >= -1 && cfg < kNumTiles, "gemm tile must be -1 (auto) or 0..", kNumTiles - 1);
  forced_tile().store(cfg);
}
int gemm_tile_count() { return kNumTiles; }

void set_f32_precision(int mode) {
  TFA_CHECK(mode >= 0 && mode <= 2, "precision mode must be 0 (f32), 1 (bf16) or 2 (bf16x3)");
  precision_state().store(mode);
}
int f32_precision() { return precision_state().load(); }

size_t gemm_workspace_bytes(DType dt, const GemmArgs& g) {
  if (dt != DType::F32 || g.M <= 0 || g.N <= 0) return 0;
  if (bf16_candidate(g)) return bf16_workspace_bytes(f32_precision(), g.N, g.K);
  return f32_ws_bytes(g.M, g.N, g.K, g.batch);
}

size_t conv2d_workspace_bytes(DType dt, const ConvArgs& a) {
  if (dt != DType::F32) return 0;
  const GemmArgs g = conv_as_gemm(a);
  if (a.seg.n == 0 && bf16_candidate(g)) return bf16_workspace_bytes(f32_precision(), g.N, g.K);
  return f32_ws_bytes(g.M, g.N, g.K, 1);
}

void gemm(DType dt, const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return;
  TFA_CHECK(g.K > 0, "gemm: K must be > 0");
  TFA_CHECK(g.A && g.B && g.C, "gemm: null operand");
  if (dt == DType::F32 && bf16_candidate(g) && bf16_gemm_eligible(g, false, 0)) {
    bf16_gemm_launch(f32_precision(), g, false, Im2colGeom{}, s);
    return;
  }
  if (dt == DType::F32) {
    // 16-byte vector loads need 4-float aligned rows on the contiguous side
    bool vec = al16(g.A) && al16(g.B) && g.lda % 4 == 0 && g.ldb % 4 == 0 &&
               (g.batch == 1 || (g.strideA % 4 == 0 && g.strideB % 4 == 0));
    if (!g.ta || g.tb) vec = vec && g.K % 4 == 0;
    run_f32(g, g.ta ? A_MCONTIG : A_KCONTIG, vec, ConvGeom{}, s);
  } else if (dt == DType::F64) {
    gemm_f64_launch(g, s);
  } else if (dt == DType::I32 || dt == DType::I64) {
    gemm_int_launch(dt, g, s);
  } else {
    TFA_CHECK(false, "gemm: dtype ", dtype_name(dt), " not supported");
  }
  TFA_LAUNCH_CHECK("gemm");
}

void conv2d_nhwc(DType dt, const ConvArgs& a, hipStream_t s) {
  TFA_CHECK(dt == DType::F32, "conv2d: f32 only");
  TFA_CHECK(a.N > 0 && a.OH > 0 && a.OW > 0 && a.OC > 0, "conv2d: empty output");
  TFA_CHECK(a.H < (1 << 30) && a.W < (1 << 30) && a.C < (1 << 30), "conv2d: dims too large");
  TFA_CHECK(a.H * a.W * a.C < (int64_t(1) << 31), "conv2d: one input image must hold < 2^31 elements");
  GemmArgs g = conv_as_gemm(a);
  // the bf16 modes have no segmented epilogue: fused sibling convs stay exact f32
  if (a.seg.n == 0 && bf16_candidate(g) && bf16_gemm_eligible(g, true, a.C)) {
    Im2colGeom cg;
    cg.H = (int)a.H; cg.W = (int)a.W; cg.C = (int)a.C; cg.KW = (int)a.KW;
    cg.OH = (int)a.OH; cg.OW = (int)a.OW;
    cg.sh = (int)a.sh; cg.sw = (int)a.sw; cg.dh = (int)a.dh; cg.dw = (int)a.dw;
    cg.pt = (int)a.pad_t; cg.pl = (int)a.pad_l;
    bf16_gemm_launch(f32_precision(), g, !conv_is_pointwise(a), cg, s);
    return;
  }
  if (!conv_is_pointwise(a) && conv_smallc_eligible(a)) {  // RGB stems: filter in registers, no LDS
    conv_smallc_launch(a, s);
    return;
  }
  if (conv_direct_eligible(a)) {  // narrow stem convs: filter in LDS, A to registers
    conv_direct_launch(a, s);
    return;
  }
  if (conv_is_pointwise(a)) {  // 1x1/s1: x is already the [N*H*W, C] A matrix
    bool vec = al16(a.x) && al16(a.w) && a.C % 4 == 0 && a.OC % 4 == 0;
    run_f32(g, A_KCONTIG, vec, ConvGeom{}, s);
  } else {
    ConvGeom cg;
    cg.H = (int)a.H; cg.W = (int)a.W; cg.C = (int)a.C; cg.KW = (int)a.KW;
    cg.OH = (int)a.OH; cg.OW = (int)a.OW;
    cg.sh = (int)a.sh; cg.sw = (int)a.sw; cg.dh = (int)a.dh; cg.dw = (int)a.dw;
    cg.pt = (int)a.pad_t; cg.pl = (int)a.pad_l;
    cg.fast = g.M < (int64_t(1) << 32);
    cg.fOW = make_fastdiv((uint32_t)a.OW);
    cg.fOH = make_fastdiv((uint32_t)a.OH);
    bool vec = a.C % 4 == 0 && al16(a.x) && al16(a.w) && a.OC % 4 == 0;
    run_f32(g, A_CONV, vec, cg, s);
  }
  TFA_LAUNCH_CHECK("conv2d");
}

}  // namespace k
}  // namespace tfa

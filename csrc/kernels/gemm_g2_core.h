// The "g2" f32 MFMA core: one wave per SIMD, LDS-DMA staging (gfx950).
//
// The round-4 core (gemm_f32_core.h) stages tiles through registers and
// ds_write, reads one k-step of fragments per ds_read_b32, and keeps 2-4
// waves per SIMD; its MFMA pipe sat ~13 % idle on the big shapes. This core
// is the structure measured in scripts/g2_lab.hip (4096^3 144 TF, 8192^3 145
// TF, 2.56M x 512 x 512 135 TF against 139.7 / 142.5 / 131.9 for the round-4
// core on the same box):
//
//   * a block of 4 waves (one per SIMD) over BM x BN, each wave a
//     (BM/WM) x (BN/WN) tile of 32x32 accumulators: up to 256 accumulator
//     registers per lane, which the compiler keeps in AGPRs;
//   * operands go global -> LDS with global_load_lds_dwordx4 (no VGPR
//     staging, no ds_write). The DMA image of an instruction is lane-linear,
//     so the layout is chosen through the per-lane SOURCE addresses:
//       - k-contiguous operands (A [M][K], conv im2col rows, B^T [N][K]):
//         one instruction = 16 rows x 64 B (whole row segments: coalesced),
//         image [row][4 k-quad slots] with slot c holding k quad
//         c ^ ((row >> 2) & 3), which makes the fragment reads conflict-free;
//       - row-contiguous B ([K][N] weights): image [k][n], one instruction =
//         256 consecutive floats of it;
//   * fragments: a lane reads its row's k quad with one ds_read_b128 and
//     feeds it to 4 MFMA k-steps (a [k][n] image: one ds_read_b32 per step);
//     the two wave halves carry the two quads of a k-octet (k = 8j + s and
//     8j + 4 + s in step s), the order the round-4 core reads k in too, so
//     every tile of both cores gives bit-identical results;
//   * a ring of STAGES LDS stages of BK = 16 with one stage in flight beyond
//     the next: counted vmcnt (never 0 in the steady loop), one raw s_barrier
//     per stage; the next fragments (and the next stage's first ones) are
//     read in the shadow of the current MFMAs, and the stage's LDS-DMA
//     instructions are spread over its k quads and between the MFMAs
//     (sched_group_barrier: each costs ~60 issue cycles back to back);
//   * out-of-range rows, padding taps and the K tail read a 16-byte zero page
//     (the DMA source is per lane), so interior and edge blocks run one path;
//   * epilogue as the round-4 core: bias + none/ReLU/ReLU6 through a
//     wave-private LDS tile and float4 stores, the sibling-conv segments, the
//     heavy (transcendental / chained) epilogue, split-K partial slabs.
#pragma once

#include "gemm_f32_core.h"

namespace tfa {
namespace k {
namespace g2 {

using f32core::A_CONV;
using f32core::A_KCONTIG;
using f32core::ConvGeom;
using f32core::F32Plan;

enum BLoad { B_RC = 0, B_KC = 1 };  // B [K][N] (row-contiguous) or B^T [N][K]
// the conv loader when C % 16 == 0: a stage's 16 k then lie in one filter tap,
// so the tap (kh, kw) and its input offset are block-uniform scalars (no
// per-lane carry chain) and a piece costs two bounds adds, the compares and
// one select
constexpr int A_CONV16 = 100;

// the launcher translation units (cfg indexes kG2Tiles): k-contiguous A with
// B [K][N] or B^T [N][K] (g.tb), and the implicit-GEMM conv (filter [K][N])
void launch_kc(const F32Plan& p, const GemmArgs& g, hipStream_t s);
void launch_conv(const F32Plan& p, const GemmArgs& g, const ConvGeom& cg, hipStream_t s);

// {BM, BN, WM, WN, STAGES, OCC}: OCC blocks per CU. (192x192: the 12x12
// Inception layers, M = 2048 * 144, make exactly 3 waves of two-block CUs.) The big tiles hold 192-256
// accumulators per lane and one block per CU; the smaller ones are sized
// (<= 256 registers, <= 80 KB of LDS) for two, so one block's prologue and
// epilogue overlap the other's main loop (K = 512 GEMMs, the convs)
// 128x224 (7 column tiles per wave, two blocks per CU): the fused sibling 1x1
// convs whose OC sum is 208-224 (Inception Mixed_5b: 64 + 48 + 64 + 32) or 448
// (= 2 x 224), which 64- / 96- / 128-wide tiles pad by 14-23 %. (A 256x224
// one-block tile needs 472 bytes of scratch per lane: not shipped.)
constexpr int kNumG2Tiles = 11;
constexpr int kG2Tiles[kNumG2Tiles][6] = {
    {256, 256, 2, 2, 4, 1}, {256, 192, 2, 2, 4, 1}, {256, 128, 2, 2, 3, 2}, {256, 64, 4, 1, 4, 2},
    {128, 128, 2, 2, 4, 2}, {128, 64, 2, 2, 5, 2},  {128, 192, 2, 2, 4, 2}, {256, 96, 4, 1, 3, 2},
    {128, 160, 4, 1, 4, 2}, {192, 192, 2, 2, 3, 2}, {128, 224, 4, 1, 3, 2}};

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// global -> LDS, 16 bytes per lane: lane i lands at lds + 16 * i
__device__ __forceinline__ void glds16(const void* gp, void* lds) {
  __builtin_amdgcn_global_load_lds(gp, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt at their maxima; gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int BM, int BN, int WM, int WN, int STAGES, int OCC, int AL, int BL>
__global__ __launch_bounds__(64 * WM * WN, OCC) void g2_tile(GemmArgs g, int tiles_m, int tiles_n, ConvGeom cg,
                                                             int64_t k_per_split, int flags) {
  constexpr int NW = WM * WN, NT = 64 * NW, BK = 16, KQ = BK / 4;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int AI = BM / 16 / NW;        // A: 16 rows per LDS-DMA instruction
  constexpr int BREAL = BN / 16;          // B: 16 rows ([N][K]) or 256 floats ([K][N]) per instruction
  constexpr int BI = (BREAL + NW - 1) / NW;
  // a B width that does not split evenly over the waves (96): the last
  // waves issue dummy pieces into a pad area, so every wave issues the same
  // G instructions per stage and the counted vmcnt waits stay uniform
  constexpr int BPAD = BI * NW - BREAL;
  constexpr int A_BYTES = BM * BK * 4, B_BYTES = BN * BK * 4, STAGE = A_BYTES + B_BYTES + BPAD * 1024;
  constexpr int G = AI + BI;              // LDS-DMA instructions per wave per stage
  constexpr int kEpi = NW * 32 * 32 * 4;
  static_assert(NW == 4 && TM >= 1 && TN >= 1 && AI >= 1 && BI >= 1 && BM % (16 * NW) == 0 && BN % 16 == 0,
                "4 waves, >= one 32x32 tile each, whole DMA instructions per wave");
  static_assert(STAGES >= 3 && STAGES * STAGE <= 160 * 1024 / OCC && STAGES * STAGE >= kEpi, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE];

  // wave index in an SGPR: every LDS-DMA destination (M0) and stage base is
  // then scalar arithmetic, not a VGPR sum + v_readfirstlane per piece
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, r32 = lane & 31;
  const int nwg = tiles_m * tiles_n;
  const int wg = f32core::xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * BM;
  const int64_t n0 = (int64_t)(wg % tiles_n) * BN;
  const int64_t bz = blockIdx.y;
  const float* A = static_cast<const float*>(g.A) + bz * g.strideA;
  const float* B = static_cast<const float*>(g.B) + bz * g.strideB;
  const int64_t M = g.M, N = g.N, K = g.K;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = min(K, kbeg + k_per_split);
  const float* zero = f32core::kZeroPage;

  // ---- operand sources. k-contiguous A, and B either way: a block-uniform
  // stage base (SGPRs, advanced by one stage per issue) plus a per-lane
  // 32-bit byte offset fixed for the whole loop (global_load_lds saddr +
  // voffset), so an unchecked piece costs no VALU at all. Checked pieces
  // (edge blocks, the K tail) select the 16-byte zero page per lane. Every
  // choice is a select: a branch here makes the compiler drain the DMA
  // queue (vmcnt(0)) at the join, which serialises the ring.
  // A instruction q = wave*AI + i covers rows 16q .. 16q+15, lane -> row
  // 16q + lane/4, k quad koff/4 of the stage (swizzled slot).
  constexpr bool CONV = AL == A_CONV || AL == A_CONV16, TAPU = AL == A_CONV16;
  const int koff = 4 * ((lane & 3) ^ ((lane >> 4) & 3));
  const char* abase = reinterpret_cast<const char*>(AL == A_KCONTIG ? A + m0 * g.lda + kbeg : A);
  uint32_t aoff[AI];    // k-contiguous: byte offset of the lane's row piece from abase
  const float* ap[AI];  // conv: the lane's image base
  bool aok[AI];         // row in range
  int cih[AI], ciw[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = (wave * AI + i) * 16 + lane / 4;
    const int64_t m = m0 + r;
    aok[i] = m < M;
    const int64_t mc = aok[i] ? m : 0;
    aoff[i] = 0;
    ap[i] = A;
    cih[i] = ciw[i] = 0;
    if constexpr (AL == A_KCONTIG) {
      aoff[i] = (uint32_t)(((int64_t)r * g.lda + koff) * 4);
    } else {
      int64_t ow, oh, n;
      if (cg.fast) {
        const uint32_t m32 = (uint32_t)mc, t = fdiv(m32, cg.fOW), q = fdiv(t, cg.fOH);
        ow = m32 - t * (uint32_t)cg.OW;
        oh = t - q * (uint32_t)cg.OH;
        n = q;
      } else {
        ow = mc % cg.OW;
        const int64_t t = mc / cg.OW;
        oh = t % cg.OH;
        n = t / cg.OH;
      }
      ap[i] = A + n * (int64_t)cg.H * cg.W * cg.C;
      cih[i] = (int)(oh * cg.sh - cg.pt);
      ciw[i] = (int)(ow * cg.sw - cg.pl);
      // TAPU: the lane's channel quad at the tap (0, 0) of its output pixel
      // (only dereferenced once a tap's bounds check passed)
      if constexpr (TAPU) ap[i] += ((int64_t)cih[i] * cg.W + ciw[i]) * cg.C + koff;
    }
  }
  // conv: this lane's k -> (kh, kw, c), advanced by BK per stage
  int kc = 0, kkw = 0, kkh = 0;
  if constexpr (CONV) {
    const int k = (int)(kbeg + (TAPU ? 0 : koff));  // TAPU: the stage's (uniform) first k
    kc = k % cg.C;
    const int t = k / cg.C;
    kkw = t % cg.KW;
    kkh = t / cg.KW;
  }
  // TAPU: the stage's tap displacement and input offset (block-uniform)
  int tdh = kkh * cg.dh, tdw = kkw * cg.dw;
  int64_t toff = ((int64_t)tdh * cg.W + tdw) * cg.C + kc;
  const char* bbase = reinterpret_cast<const char*>(BL == B_KC ? B + n0 * g.ldb + kbeg : B + kbeg * g.ldb + n0);
  uint32_t boff[BI];
  bool bok[BI];
  int bk_[BI];  // the piece's k within the stage
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int q = wave * BI + i;
    if (q >= BREAL) {  // a pad piece: any valid source (B's first row), or the zero page when checked
      bok[i] = false;
      boff[i] = 0;
      bk_[i] = 0;
    } else if constexpr (BL == B_KC) {
      const int r = q * 16 + lane / 4;
      bok[i] = n0 + r < N;
      boff[i] = (uint32_t)(((int64_t)r * g.ldb + koff) * 4);
      bk_[i] = koff;
    } else {
      const int e = q * 256 + 4 * lane;
      const int kb = e / BN, nb = e % BN;
      bok[i] = n0 + nb < N;
      boff[i] = (uint32_t)(((int64_t)kb * g.ldb + nb) * 4);
      bk_[i] = kb;
    }
  }
  constexpr int64_t astep = BK * 4;                                                  // bytes per stage
  const int64_t bstep = BL == B_KC ? (int64_t)BK * 4 : (int64_t)BK * g.ldb * 4;
  int64_t kpos = kbeg;  // k0 of the next stage to issue

  // The LDS-DMA of one stage, piece by piece (A pieces 0..AI-1, then B
  // pieces), so the main loop can place each between two MFMAs. CHECK: the
  // block's rows / columns or the stage's k may fall outside the operands.
  auto issue_piece = [&](int slot, int p, auto chk) __attribute__((always_inline)) {
    constexpr bool CHECK = decltype(chk)::value;
    char* base = smem + slot * STAGE;
    const bool kok = !CHECK || kpos + koff < kend;
    if (p < AI) {
      const int i = p;
      const float* src;
      if constexpr (AL == A_KCONTIG) {
        src = reinterpret_cast<const float*>(abase + aoff[i]);
        if constexpr (CHECK) src = (aok[i] & kok) ? src : zero;
      } else if constexpr (TAPU) {
        const int ih = cih[i] + tdh, iw = ciw[i] + tdw;
        const bool ok = aok[i] & kok & ((unsigned)ih < (unsigned)cg.H) & ((unsigned)iw < (unsigned)cg.W);
        // an arithmetic select: written as `ok ? p : zero` the compiler sinks
        // the address math into an exec-masked branch per piece
        const uint64_t msk = 0ull - (uint64_t)ok;
        src = reinterpret_cast<const float*>((reinterpret_cast<uint64_t>(ap[i] + toff) & msk) |
                                             (reinterpret_cast<uint64_t>(zero) & ~msk));
      } else {
        const int ih = cih[i] + kkh * cg.dh, iw = ciw[i] + kkw * cg.dw;
        const bool ok = aok[i] & kok & (ih >= 0) & (ih < cg.H) & (iw >= 0) & (iw < cg.W);
        src = ok ? ap[i] + ((ih * cg.W + iw) * cg.C + kc) : zero;
      }
      glds16(src, base + (wave * AI + i) * 1024);
      if (TAPU && i == AI - 1) {
        // the next stage's tap: one step of the uniform (c0, kw, kh) counter
        const bool wrap = kc + BK >= cg.C;
        kc = wrap ? 0 : kc + BK;
        const int w1 = kkw + (wrap ? 1 : 0);
        const bool wrap2 = w1 == cg.KW;
        kkw = wrap2 ? 0 : w1;
        kkh = kkh + (wrap2 ? 1 : 0);
        tdh = kkh * cg.dh;
        tdw = kkw * cg.dw;
        toff = ((int64_t)tdh * cg.W + tdw) * cg.C + kc;
      } else if (CONV && i == AI - 1) {
        // advance (kc, kkw, kkh) by BK; C >= 4, so at most BK / 4 carries:
        // a fixed, select-only sequence (no data-dependent loop)
        kc += BK;
#pragma unroll
        for (int r = 0; r < BK / 4; ++r) {
          const bool carry = kc >= cg.C;
          kc = carry ? kc - cg.C : kc;
          const int w1 = kkw + (carry ? 1 : 0);
          const bool wrap = w1 == cg.KW;
          kkw = wrap ? 0 : w1;
          kkh = kkh + (wrap ? 1 : 0);
        }
      }
    } else {
      const int i = p - AI;
      const float* src = reinterpret_cast<const float*>(bbase + boff[i]);
      if constexpr (CHECK) src = (bok[i] & (kpos + bk_[i] < kend)) ? src : zero;
      glds16(src, base + A_BYTES + (wave * BI + i) * 1024);
      if (i == BI - 1) {
        kpos += BK;
        abase += astep;
        bbase += bstep;
      }
    }
  };
  auto issue = [&](int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < G; ++p) issue_piece(slot, p, std::true_type{});
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){};

  // Fragments. MFMA k-step s of k-quad pair j takes k = 8j + s from lanes
  // 0-31 and k = 8j + 4 + s from lanes 32-63, steps in increasing (j, s): a
  // lane reads ITS row's k quad 2j + h once (ds_read_b128) and feeds its 4
  // components to 4 steps, no per-step select. The round-4 core
  // (gemm_f32_core.h) reads k in the same order, so every f32 tile gives
  // bit-identical results (the autotuner's pick never changes a result).
  // A [k][n] image (B row-contiguous) is read per step (ds_read_b32).
  struct Frag {
    f32x4 a[TM];
    f32x4 b[TN];
  };
  const int slot_sw = (r32 >> 2) & 3;  // the rows a lane reads differ by multiples of 32: one swizzle
  // fragment r of k-quad pair j of stage kt: r < TM an A fragment, else B fragment r - TM
  auto read_frag = [&](int kt, int j, int r, Frag& f) __attribute__((always_inline)) {
    const char* st = smem + (kt % STAGES) * STAGE;
    const int q = 2 * j + h;
    const int slot = q ^ slot_sw;
    if (r < TM) {
      const int i = r;
      f.a[i] = *reinterpret_cast<const f32x4*>(st + (wm * (BM / WM) + i * 32 + r32) * 64 + slot * 16);
    } else {
      const int jn = r - TM;
      const int n = wn * (BN / WN) + jn * 32 + r32;
      if constexpr (BL == B_KC) {
        f.b[jn] = *reinterpret_cast<const f32x4*>(st + A_BYTES + n * 64 + slot * 16);
      } else {
        const float* bs = reinterpret_cast<const float*>(st + A_BYTES) + 4 * q * BN + n;
        f.b[jn] = (f32x4){bs[0], bs[BN], bs[2 * BN], bs[3 * BN]};
      }
    }
  };
  auto read = [&](int kt, int j, Frag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < TM + TN; ++r) read_frag(kt, j, r, f);
  };
  constexpr int KP = KQ / 2;                            // k-quad pairs per stage
  constexpr int NM = 4 * TM * TN;                       // MFMAs per pair
  constexpr int NR = TM + TN * (BL == B_KC ? 1 : 4);    // LDS read instructions per pair
  static_assert(KQ % 2 == 0, "whole k-quad pairs per stage");

  const int KT = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;
  // prologue: stages 0 .. S-2 (a stage past KT reads only zero pages)
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) issue(s);
  wait_vm<G * (STAGES - 2)>();  // stage 0 landed
  __builtin_amdgcn_s_barrier();
  Frag cur, nxt;
  read(0, 0, cur);
  // One stage: stage kt+1 retired for every wave (counted wait + barrier),
  // which also frees the slot of stage kt-1 for the DMA of stage kt+S-1;
  // then KP pairs of NM MFMAs, each with the next pair's fragment reads (the
  // next stage's first pair after the last) in its shadow. The stage's G DMA
  // pieces are spread over the pairs (each costs ~60 issue cycles when
  // issued back to back) and, inside a pair, alternate with the MFMAs
  // (sched_group_barrier), as do the fragment reads. A stage past KT reads a
  // slot with no live data: those values feed no MFMA.
  auto stage = [&](int kt, auto do_issue, auto do_check) __attribute__((always_inline)) {
    constexpr bool ISSUE = decltype(do_issue)::value;
    // a stage that issues stage kt+S-1 < KT has stage kt+S-2 in flight too
    if (ISSUE || kt + STAGES - 2 < KT) wait_vm<G * (STAGES - 3)>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    const int slot_next = (kt + STAGES - 1) % STAGES;
    static_for<KP>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      // the stage's DMA pieces all go with pair 0 (measured: spreading them
      // over the pairs leaves the last pair's pieces clustered at the loop
      // end, where no MFMA hides them)
      constexpr int p0 = 0, p1 = (ISSUE && j == 0) ? G : 0;
      constexpr int NP = p1 - p0;
      if constexpr (j + 1 < KP) read(kt, j + 1, nxt);
      else read(kt + 1, 0, nxt);
      static_for<NP>([&](auto pc) __attribute__((always_inline)) {
        issue_piece(slot_next, p0 + decltype(pc)::value, do_check);
      });
#pragma unroll
      for (int sk = 0; sk < 4; ++sk)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int jn = 0; jn < TN; ++jn)
            acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.a[i][sk], cur.b[jn][sk], acc[i][jn], 0, 0, 0);
      // MFMA, DMA piece, MFMA, DMA piece, ..., then MFMA, read, MFMA, read, ...
      static_for<NM>([&](auto xc) __attribute__((always_inline)) {
        constexpr int x = decltype(xc)::value;
        __builtin_amdgcn_sched_group_barrier(f32core::kSchedMfma, 1, 0);
        if constexpr (x < NP) __builtin_amdgcn_sched_group_barrier(f32core::kSchedVmemRead, 1, 0);
        else if constexpr (x < NP + NR) __builtin_amdgcn_sched_group_barrier(f32core::kSchedDsRead, 1, 0);
      });
      cur = nxt;
    });
  };
  // stages whose DMA stays inside the operands (interior block, a stage
  // entirely inside [kbeg, kend)) issue unchecked; the rest select per lane
  int kt = 0;
  const int KTF = kend > kbeg ? (int)((kend - kbeg) / BK) : 0;
  if (m0 + BM <= M && n0 + BN <= N)
    for (; kt + STAGES - 1 < KTF; ++kt) stage(kt, std::true_type{}, std::false_type{});
  for (; kt + STAGES - 1 < KT; ++kt) stage(kt, std::true_type{}, std::true_type{});
  for (; kt < KT; ++kt) stage(kt, std::false_type{}, std::true_type{});
  __syncthreads();  // every wave is done with the ring: its LDS becomes the epilogue staging

  // ---- epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int vepi = flags & 1;
  float* ws = static_cast<float*>(g.workspace);
  const float* bias = static_cast<const float*>(g.bias);
  const bool heavy = !ws && !(g.act <= ACT_RELU6 && g.epi.n == 0);
  float* Cb = static_cast<float*>(g.C) + bz * g.strideC;
  if (vepi) {
    float* stg = reinterpret_cast<float*>(smem) + wave * 1024;
    static_for<TN>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      static_for<TM>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        const f32x16 v = acc[i][j];
#pragma unroll
        for (int r = 0; r < 16; ++r) stg[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + r32] = v[r];
        const int64_t col = n0 + wn * (BN / WN) + j * 32 + 4 * (lane & 7);
        if (col < N) {
          float* cbase;
          int64_t cld;
          int cact;
          f32core::out_col(g, Cb, col, cbase, cld, cact);
          float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (bias) bv = make_float4(bias[col], bias[col + 1], bias[col + 2], bias[col + 3]);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int rr = 8 * q + (lane >> 3);
            const int64_t row = m0 + wm * (BM / WM) + i * 32 + rr;
            float4 o = *reinterpret_cast<const float4*>(&stg[rr * 32 + 4 * (lane & 7)]);
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
    const int64_t col = n0 + wn * (BN / WN) + j * 32 + r32;
    if (col >= N) return;
    const float bv = (!ws && bias) ? bias[col] : 0.f;
    float* cbase;
    int64_t cld;
    int cact;
    f32core::out_col(g, Cb, col, cbase, cld, cact);
    if (heavy) cact = ACT_NONE;
    static_for<TM>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const f32x16 v = acc[i][j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
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
      const int64_t col = n0 + wn * (BN / WN) + j * 32 + r32;
      const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (col >= N || row >= M) continue;
      float* cbase;
      int64_t cld;
      int cact;
      f32core::out_col(g, Cb, col, cbase, cld, cact);
      float* p = cbase + row * cld;
      *p = epi_apply(g.epi, act_apply(*p, cact), row, col, N, bz * M * N);
    }
  }
}

template <int AL, int BL>
void launch_cfg(const F32Plan& p, const GemmArgs& g, const ConvGeom& cg, hipStream_t s) {
  const int vepi = p.splits == 1 ? f32core::vector_epilogue(g) : 0;
  const int bm = kG2Tiles[p.cfg][0], bn = kG2Tiles[p.cfg][1];
  const int64_t tm = (g.M + bm - 1) / bm, tn = (g.N + bn - 1) / bn;
  TFA_CHECK(tm * tn < (int64_t(1) << 31), "gemm: grid too large");
  TFA_CHECK(g.batch <= 65535 && p.splits <= 65535, "gemm: batch/splits too large");
  dim3 grid((unsigned)(tm * tn), (unsigned)g.batch, (unsigned)p.splits);
#define TFA_G2(C_)                                                                                             \
  hipLaunchKernelGGL((g2_tile<kG2Tiles[C_][0], kG2Tiles[C_][1], kG2Tiles[C_][2], kG2Tiles[C_][3], kG2Tiles[C_][4], \
                              kG2Tiles[C_][5], AL, BL>),                                                         \
                     grid, dim3(64 * kG2Tiles[C_][2] * kG2Tiles[C_][3]), 0, s, g, (int)tm, (int)tn, cg,          \
                     p.k_per_split, vepi)
  switch (p.cfg) {
    case 0: TFA_G2(0); break;
    case 1: TFA_G2(1); break;
    case 2: TFA_G2(2); break;
    case 3: TFA_G2(3); break;
    case 4: TFA_G2(4); break;
    case 5: TFA_G2(5); break;
    case 6: TFA_G2(6); break;
    case 7: TFA_G2(7); break;
    case 8: TFA_G2(8); break;
    case 9: TFA_G2(9); break;
    default: TFA_G2(10); break;
  }
#undef TFA_G2
}

}  // namespace
}  // namespace g2
}  // namespace k
}  // namespace tfa

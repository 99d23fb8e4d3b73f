// Winograd F(2x2, 3x3) Conv2D on the f32 MFMA pipe (gfx950), fully fused.
//
// Why: on gfx950 exact f32 runs at 64 FLOP/clk/SIMD on MFMA and VALU alike
// (157 TF/s), and the implicit-GEMM core sits at 77-83 % of that on the 3x3
// stride-1 convs of Inception-v3 and VGG-16 (profiles/r5_layers/). F(2x2,3x3)
// computes a 2x2 output tile from a 4x4 input patch with 16 products per
// (tile, in-channel, out-channel) instead of 36: 2.25x fewer MFMA FLOPs for the
// same result (Lavin & Gray 2016). Reference workload: BASELINE config 5 and
// src/main/python/tensorframes_snippets/read_image.py:62-71 (VGG-16 scoring).
//
// Math (cross-correlation, as TF's Conv2D): per tile with input patch d (4x4)
// and filter g (3x3) of one (c, oc) pair,
//   V = B^T d B,  U = G g G^T,  M = sum_c V (.) U,  Y = A^T M A   (2x2)
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
//   G   = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]
//   A^T = [1 1 1 0; 0 1 -1 -1]
// U is computed once per plan on the host in fp64 (executor planner pass,
// conv_wino_filter) and kept in HBM as [C/4][16 xi][OCP][4 c] (OCP = OC
// rounded up to 64, zero filled) so one 16-byte DMA piece holds 4 channels of
// one (xi, oc).
//
// Kernel structure (one block of 4 waves = one wave per SIMD, T tiles x BN
// output channels, all 16 xi):
//   * wave w owns the xi row xi_y = w: its accumulators are M[w][xi_x][T][BN]
//     (4 * T * BN / 64 = 256 registers per lane), so the input transform for
//     its A operands needs only the two patch rows B^T row w combines (rows
//     {0,2}, {1,2}, {2,1}, {1,3}) and no V tile ever goes through LDS;
//   * per k-step of 4 channels one LDS stage holds the block's input patches
//     [16 px][T][4 c] and the transformed filter [16 xi][BN][4 c], both filled
//     by global_load_lds_dwordx4 (padding taps / tiles past the end read a
//     16-byte zero page), in a ring of S stages with counted vmcnt waits and
//     one raw s_barrier per stage (the g2 core's pipeline, gemm_g2_core.h);
//   * v_mfma_f32_16x16x4_f32: lane (q = l>>4, i = l&15) feeds A[tile i][c q]
//     and B[c q][oc i]: every fragment is one conflict-free ds_read_b32, and
//     the A value is (row-combine, then column-transform) of 8 patch reads:
//     8 VALU ops per 16 MFMAs that use it;
//   * epilogue: A^T along x in registers (M[w][.] -> 2 values per wave), the
//     4 waves' partial rows through LDS (pitch BN+4: conflict-free writes), A^T
//     along y, bias + none/ReLU/ReLU6, float4 stores into the NHWC output (or
//     its concat channel slice, or the sibling-conv segments).
// Summation order is fixed (no atomics): a given conv always gives the same
// bits. Numerics: tests/test_gpu_wino.py gates the error against fp64.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "gemm_f32_core.h"

namespace tfa {
namespace k {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct WinoGeom {
  int H, W, C, OH, OW, pt, pl, TH, TW, OCP, KT;
  int64_t ntiles;
  int64_t img_floats;    // H * W * C
  int64_t u_bytes;       // the whole transformed filter
  int dbg;               // timing experiments (TFA_WINO_DEBUG): 1 no filter traffic, 2 no input traffic, 4 no stores
  // F(2,7) (1x7 / 7x1): tile t -> (n, i0, i1) over (D0, D1); the conv axis
  // is W (axis 0: tile = 2 outputs along W) or H (axis 1)
  int axis, D0, D1;
  FastDivU32 fD0, fD1;
  // F(4,5) x 5 rows (5x5): k-stage kt = kh * KTC + (8-channel block)
  int KTC;
  FastDivU32 fKTC;
  FastDivU32 fTW, fTH;
};

template <int N>
__device__ __forceinline__ void wwait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// a raw buffer descriptor (gfx9 dword 3); bases and sizes must be provably
// uniform (readfirstlane) or every buffer op becomes a waterfall loop
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wrsrc(const void* base, uint32_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// 16 bytes per lane global -> LDS (lane i lands at lds + 16 i); a lane whose
// offset is past the descriptor's size reads zeros (padding taps, tiles past
// the end): no per-lane select, no branch between DMA issues
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ float act3(float v, int a) {  // none / ReLU / ReLU6 as selects
  float r = (a != 0 && !(v > 0.f)) ? 0.f : v;
  return (a == ACT_RELU6 && r > 6.f) ? 6.f : r;
}

constexpr uint32_t kOOB = 0x80000000u;  // an offset past every input descriptor

// epilogue stores of rows past the end (tiles past the last, odd output
// edges, oc past OC) land here, so every lane issues the same stores (the
// next item's first wait counts them: no branch around a store)
__device__ __attribute__((aligned(16))) float4 kWinoTrash[64];

// Persistent: one block of 8 waves (two per SIMD) per CU, each taking work
// items (T tiles x BN oc) b', b' + G, ... (b' = XCD remap of its index, so
// the 32 blocks of one XCD hold 32 consecutive items: the oc blocks of a tile
// block, and neighbouring tile blocks, share L2). The DMA of the next item's
// first stage is issued before this item's epilogue, which hides its latency.
// BN = 64 (T = 64): wave w owns the xi row xr = w & 3 of tiles
// [32 (w >> 2), +32) x 64 oc. BN = 32 (T = 128, OC <= 32 layers such as
// Inception's Conv2d_2a: no padded oc half): tiles [64 (w >> 2), +64) x 32 oc.
// Either way acc[xi_x][2] = 4 x 2 32x32 accumulators = 128 registers per lane.
template <int BN, bool POOL>
__global__ __launch_bounds__(512, 1) void wino23_kernel(GemmArgs g, WinoGeom q, int nbn, int nwork) {
  constexpr int T = 4096 / BN, TWV = 32;
  constexpr int NG = T / 32;                   // 32-tile groups per block
  constexpr int MT = T / 64, NT = BN / 32;     // a wave's tile groups and 32-oc halves (MT * NT = 2)
  static_assert(MT * NT == 2, "two 32x32 accumulators per xi column");
  constexpr int IN_BYTES = 16 * 2 * T * 16, U_BYTES = 16 * 2 * BN * 16, STAGE = IN_BYTES + U_BYTES;
  constexpr int GI = 2 * NG, GU = BN / 16;     // DMA pieces per wave per stage
  constexpr int EP = BN + 4;                   // exchange row pitch (floats): conflict-free ds_write_b32
  constexpr int EH_BYTES = 4 * T * EP * 4;     // one px plane of the exchange
  constexpr int SMEM = (2 * STAGE > STAGE + EH_BYTES) ? 2 * STAGE : STAGE + EH_BYTES;  // slot 0 | slot 1 (+ exchange)
  constexpr int LPT = BN / 4, TPP = 64 / LPT;  // epilogue: lanes per tile (float4 of oc), tiles per pass
  constexpr int NPASS = T / 8 / TPP;           // passes over the wave's T/8 tiles
  // stores per lane per item (unconditional): one per (pass, px, py), or with
  // the fused 2x2 max pool one per pass (the pooled pixel of the 2x2 tile)
  constexpr int NST = POOL ? NPASS : NPASS * 2 * 2;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int xr = wave & 3, tp = wave >> 2;  // xi row, tile part
  const int h = lane >> 5, r32 = lane & 31;
  const int G = gridDim.x;
  const int KT = q.KT;
  const float* x = static_cast<const float*>(g.A);
  const __amdgpu_buffer_rsrc_t ru = wrsrc(g.B, (q.dbg & 1) ? 0u : (uint32_t)q.u_bytes);
  const __amdgpu_buffer_rsrc_t rnil = wrsrc(g.B, 0u);
  // filter piece p = wave * GU + i covers (xi, quad) rows p * (64 / BN) + lane / BN,
  // oc n0 + lane % BN (global layout [C/8][16 xi][2 quads][OCP][4 c])
  uint32_t uoff[GU];
#pragma unroll
  for (int i = 0; i < GU; ++i)
    uoff[i] = (uint32_t)((((wave * GU + i) * (64 / BN) + lane / BN) * q.OCP + lane % BN) * 16);
  const uint32_t ustep = (uint32_t)(32 * q.OCP * 16);  // filter bytes per 8-channel stage

  // ---- one work item's DMA state. Input: the descriptor starts at the
  // item's first image (every valid tap lies within 2^31 bytes of it:
  // conv_wino_eligible); piece p = wave * GI + i: patch position p / NG
  // (= 4 py + px), tile group p % NG, lane L: tile 32 (p % NG) + (L & 31),
  // channel quad L >> 5 (a pixel's two quads are one 32-byte access). A
  // padding tap or a tile past the end has an out-of-range offset (zeros).
  // An item past the end (the prefetch after a block's last item) reads
  // through the empty descriptor.
  struct Item {
    int64_t t0;
    int n0;
    __amdgpu_buffer_rsrc_t rin, rf;
    uint32_t ioff[GI];
  };
  auto setup = [&](int item, bool live, Item& it) __attribute__((always_inline)) {
    const int itc = live ? item : 0;
    it.t0 = (int64_t)(itc / nbn) * T;
    it.n0 = (itc % nbn) * BN;
    const uint32_t nb0 = (uint32_t)(it.t0 / ((int64_t)q.TH * q.TW));
    const __amdgpu_buffer_rsrc_t r = wrsrc(x + (int64_t)nb0 * q.img_floats, (q.dbg & 2) ? 0u : kOOB);
    it.rin = live ? r : rnil;
    it.rf = live ? ru : rnil;
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int p = wave * GI + i, pos = p / NG, py = pos >> 2, px = pos & 3;
      const int64_t t = it.t0 + (p % NG) * 32 + r32;
      const bool tl = t < q.ntiles;
      const uint32_t tc = tl ? (uint32_t)t : 0u;
      const uint32_t qa = fdiv(tc, q.fTW), tx = tc - qa * (uint32_t)q.TW;
      const uint32_t n = fdiv(qa, q.fTH), ty = qa - n * (uint32_t)q.TH;
      const int ih = 2 * (int)ty - q.pt + py, iw = 2 * (int)tx - q.pl + px;
      const bool ok = tl & ((unsigned)ih < (unsigned)q.H) & ((unsigned)iw < (unsigned)q.W);
      it.ioff[i] = ok ? (uint32_t)((((int64_t)(n - nb0) * q.H + ih) * q.W + iw) * q.C * 4 + h * 16) : kOOB;
    }
  };
  // stage kt -> slot kt & 1: input [pos][group][quad][32 tiles][16 B], filter [xi][quad][oc][16 B]
  auto issue = [&](const Item& it, int kt) __attribute__((always_inline)) {
    char* base = smem + (kt & 1) * STAGE;
    const uint32_t is = (uint32_t)kt * 32u, us = (uint32_t)(it.n0 * 16) + (uint32_t)kt * ustep;
#pragma unroll
    for (int i = 0; i < GI; ++i) bdma16(it.rin, it.ioff[i], is, base + (wave * GI + i) * 1024);
#pragma unroll
    for (int i = 0; i < GU; ++i) bdma16(it.rf, uoff[i], us, base + IN_BYTES + (wave * GU + i) * 1024);
  };

  // ---- fragments: lane (h, r32) holds tile r32 of a 32-tile group and oc
  // r32 of a 32-oc half, channel quad h; MFMA step s takes channel 4h + s.
  // B^T row xr: t = d[ra] + sgn * d[rb]
  const int ra = xr == 0 ? 0 : (xr == 2 ? 2 : 1);
  const int rb = xr == 0 ? 2 : (xr == 1 ? 2 : (xr == 2 ? 1 : 3));
  const float sgn = xr == 1 ? 1.f : -1.f;
  f32x4 av[4][MT], bv[4][NT];
  // reads in the order the xi_x columns need them (V_0 = t0 - t2, then t1,
  // then t3), so the first MFMAs wait for part of the reads only
  auto read = [&](int kt) __attribute__((always_inline)) {
    const char* st = smem + (kt & 1) * STAGE;
    auto inp = [&](int r, int px, int m) __attribute__((always_inline)) {
      return *reinterpret_cast<const f32x4*>(st + (((r * 4 + px) * NG + tp * MT + m) * 2 + h) * 512 + r32 * 16);
    };
    auto filt = [&](int j) __attribute__((always_inline)) {
#pragma unroll
      for (int nh = 0; nh < NT; ++nh)
        bv[j][nh] = *reinterpret_cast<const f32x4*>(st + IN_BYTES + (((4 * xr + j) * 2 + h) * BN + nh * 32 + r32) * 16);
    };
    auto tr = [&](f32x4 a, f32x4 b) __attribute__((always_inline)) {
      f32x4 t;
#pragma unroll
      for (int c = 0; c < 4; ++c) t[c] = __builtin_fmaf(sgn, b[c], a[c]);  // exact a +- b
      return t;
    };
    f32x4 t1v[MT], t2v[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const f32x4 t0v = tr(inp(ra, 0, m), inp(rb, 0, m));
      t2v[m] = tr(inp(ra, 2, m), inp(rb, 2, m));
      av[0][m] = t0v - t2v[m];
    }
    filt(0);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      t1v[m] = tr(inp(ra, 1, m), inp(rb, 1, m));
      av[1][m] = t1v[m] + t2v[m];
      av[2][m] = t2v[m] - t1v[m];
    }
    filt(1);
    filt(2);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const f32x4 t3v = tr(inp(ra, 3, m), inp(rb, 3, m));
      av[3][m] = t1v[m] - t3v;
    }
    filt(3);
  };

  f32x16 acc[4][2];  // [xi_x][m * NT + nh]
  auto mfma_cols = [&](int j0, int j1, const f32x4 (&a)[4][MT], const f32x4 (&b)[4][NT]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = j0; j < j1; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int nh = 0; nh < NT; ++nh)
            acc[j][m * NT + nh] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j][m][s], b[j][nh][s], acc[j][m * NT + nh], 0, 0, 0);
  };
  f32x4 pa[4][MT], pb[4][NT];  // the deferred xi_x = 3 column (only [3] is live)
  float* E = reinterpret_cast<float*>(smem + STAGE);

  int item = f32core::xcd_remap(blockIdx.x, G);
  if (item >= nwork) return;
  Item cur;
  setup(item, true, cur);
  issue(cur, 0);
  for (bool first = true;; first = false) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) acc[j][k2] = (f32x16){};
    // The xi_x = 3 column's MFMAs of stage kt run right after stage kt+1's
    // barrier: they keep the matrix pipe busy while that stage's fragment
    // reads and input transform are in flight.
    for (int kt = 0; kt < KT; ++kt) {
      if (kt == 0 && !first) wwait_vm<NST>();  // the previous epilogue's stores may still fly
      else wwait_vm<0>();
      __builtin_amdgcn_s_barrier();
      if (kt + 1 < KT) issue(cur, kt + 1);
      if (kt > 0) mfma_cols(3, 4, pa, pb);
      read(kt);
      mfma_cols(0, 3, av, bv);
#pragma unroll
      for (int m = 0; m < MT; ++m) pa[3][m] = av[3][m];
#pragma unroll
      for (int nh = 0; nh < NT; ++nh) pb[3][nh] = bv[3][nh];
    }
    mfma_cols(3, 4, pa, pb);
    // the epilogue's per-lane column, its activation and bias (loaded before
    // the barrier, whose vmcnt(0) it then costs nothing)
    const int cq = lane % LPT, trr = lane / LPT;
    const int64_t col = cur.n0 + 4 * cq;
    const bool colok = col < g.N;
    float* cbase;
    int64_t cld;
    int cact;
    f32core::out_col(g, static_cast<float*>(g.C), colok ? col : 0, cbase, cld, cact);
    const float* bias = static_cast<const float*>(g.bias);
    const float4 bvv = (bias && colok) ? *reinterpret_cast<const float4*>(bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();  // the ring is free: slot 0 takes the next item's first stage, slot 1 the exchange
    const int next = item + G;
    const bool live = next < nwork;
    Item nx;
    setup(next, live, nx);
    issue(nx, 0);
    // ---- epilogue, one output column px at a time. A^T along x in
    // registers: m'[xr][px] (C/D layout of 32x32x2: oc = 32 nh + (l & 31),
    // tile = (r & 3) + 8 (r >> 2) + 4 h of a 32-tile group); the 4 xi rows
    // through LDS; A^T along y; bias + activation; float4 stores (POOL: the
    // max of the tile's 4 activated outputs, one store at the pooled pixel).
    float4 pmax[NPASS];
#pragma unroll
    for (int px = 0; px < 2; ++px) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int nh = 0; nh < NT; ++nh)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int k2 = m * NT + nh;
            const float mv = px == 0 ? (acc[0][k2][r] + acc[1][k2][r]) + acc[2][k2][r]
                                     : (acc[1][k2][r] - acc[2][k2][r]) - acc[3][k2][r];
            const int tile = (tp * MT + m) * TWV + (r & 3) + 8 * (r >> 2) + 4 * h;
            E[(xr * T + tile) * EP + 32 * nh + r32] = mv;
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) {
        const int tile = wave * (T / 8) + ps * TPP + trr;
        const int64_t t = cur.t0 + tile;
        const bool tl = t < q.ntiles;
        const uint32_t tc = tl ? (uint32_t)t : 0u, qa = fdiv(tc, q.fTW), tx = tc - qa * (uint32_t)q.TW;
        const uint32_t n = fdiv(qa, q.fTH), ty = qa - n * (uint32_t)q.TH;
        f32x4 e[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) e[w] = *reinterpret_cast<const f32x4*>(&E[(w * T + tile) * EP + 4 * cq]);
        const f32x4 y0 = (e[0] + e[1]) + e[2];
        const f32x4 y1 = (e[1] - e[2]) - e[3];
        const int ow = 2 * (int)tx + px;
        float4 ov[2];
#pragma unroll
        for (int py = 0; py < 2; ++py) {
          const f32x4 v = py ? y1 : y0;
          ov[py].x = act3(v[0] + bvv.x, cact);
          ov[py].y = act3(v[1] + bvv.y, cact);
          ov[py].z = act3(v[2] + bvv.z, cact);
          ov[py].w = act3(v[3] + bvv.w, cact);
        }
        if constexpr (POOL) {  // OH, OW even: a tile is one whole pooling window
          const float4 m = make_float4(fmaxf(ov[0].x, ov[1].x), fmaxf(ov[0].y, ov[1].y), fmaxf(ov[0].z, ov[1].z),
                                       fmaxf(ov[0].w, ov[1].w));
          if (px == 0) {
            pmax[ps] = m;
          } else {
            const float4 o = make_float4(fmaxf(pmax[ps].x, m.x), fmaxf(pmax[ps].y, m.y), fmaxf(pmax[ps].z, m.z),
                                         fmaxf(pmax[ps].w, m.w));
            const bool ok = tl && colok && !(q.dbg & 4);
            const int64_t row = ((int64_t)n * (q.OH / 2) + ty) * (q.OW / 2) + tx;
            float4* dst = ok ? reinterpret_cast<float4*>(cbase + (ok ? row : 0) * cld) : &kWinoTrash[lane];
            *dst = o;
          }
        } else {
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            const int oh = 2 * (int)ty + py;
            const bool ok = tl && colok && ow < q.OW && oh < q.OH && !(q.dbg & 4);
            const int64_t row = ((int64_t)n * q.OH + oh) * q.OW + ow;
            float4* dst = ok ? reinterpret_cast<float4*>(cbase + (ok ? row : 0) * cld) : &kWinoTrash[lane];
            *dst = ov[py];
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // the plane is read: the next one may overwrite it
    }
    if (!live) break;
    item = next;
    cur = nx;
  }
}

// ---------------------------------------------------------------- F(2,7)
// 1x7 / 7x1 convs (Inception-v3 Mixed_6x: ~25 % of its conv time): a tile is
// 2 outputs along the conv axis, its patch 8 inputs; 8 transform points
// {0, +-1, +-2, +-1/2, inf} (tests/test_wino.py derives and checks the
// matrices):
//   V = B^T d: V0 = (d6 - d0) + 21/4 (d2 - d4), V7 = (d7 - d1) + 21/4 (d3 - d5),
//     V1,2 = E1 +- O1 (E1 = d2 - 17/4 d4 + d6, O1 = d1 - 17/4 d3 + d5),
//     V3,4 = E3 +- O3 (E3 = d2/4 - 5/4 d4 + d6, O3 = d1/2 - 5/2 d3 + 2 d5),
//     V5,6 = E5 +- O5 (E5 = 4 d2 - 5 d4 + d6, O5 = 2 d1 - 5/2 d3 + d5/2)
//   Y0 = M0 + ... + M6,  Y1 = (M1 - M2) + 2 (M3 - M4) + (M5 - M6) / 2 + M7
// 8 products per 2 outputs instead of 14 (1.75x fewer MFMA FLOPs); f32 error
// ~1.7x the direct path's (the gate in tests/test_gpu_wino.py).
//
// With 8 transform points a wave holds ALL of them for a 32-tile x 32-oc
// quadrant (8 accumulators of 32x32 = 128 registers per lane, two waves per
// SIMD), so the output transform is in registers: no LDS exchange, no
// epilogue barrier. Block: 8 waves = 4 tile quarters x 2 oc halves = 128
// tiles x 64 oc; 8-channel stages of 48 KB (input [8 pos][4 tq][2 quads][32
// tiles][16 B], filter [8 xi][2 quads][64 oc][16 B]) in a ring of 3, DMA two
// stages ahead; persistent blocks prefetch the next item's first stage under
// the epilogue (as wino23_kernel). BN = 32 (OC = 160 layers: 5 blocks of 32
// instead of 3 of 64 with the last half empty): 8 waves = 8 tile groups x one
// 32-oc half = 256 tiles x 32 oc, 72 KB stages in a ring of 2, DMA one stage
// ahead (as the F(2x2,3x3) kernel).
// ---------------------------------------------------------------- F(4,5)
// 5x5 convs (Inception-v3 Mixed_5b/c/d branch 1): the same 8 transform points
// (so the same input transform B^T) give F(4,5) along W: a tile is 4 outputs,
// its patch 8 inputs, U = G5 g with G5[i][k] = c_i p_i^k (G7's row scales)
// and A^T = [p_i^j] (j < 4, the inf point in row 3):
//   Y0 = M0 + ... + M6,  Y1 = (M1 - M2) + 2 (M3 - M4) + (M5 - M6) / 2,
//   Y2 = (M1 + M2) + 4 (M3 + M4) + (M5 + M6) / 4,
//   Y3 = (M1 - M2) + 8 (M3 - M4) + (M5 - M6) / 8 + M7.
// The 5 filter rows are 5 more k blocks of the same accumulation (stage kt =
// kh * C/8 + channel block reads input row oh - pt + kh): 8 products per 4
// outputs per filter row instead of 20 (2.5x fewer MFMA FLOPs). tests/test_wino.py
// checks the matrices exactly; the f32 error gate is tests/test_gpu_wino.py's.
template <int BN, bool F45 = false>
__global__ __launch_bounds__(512, 1) void wino27_kernel(GemmArgs g, WinoGeom q, int nbn, int nwork) {
  constexpr int T = 8192 / BN, NQ = T / 32;   // tiles per item, 32-tile groups
  constexpr int IN_BYTES = 8 * 2 * T * 16, U_BYTES = 8 * 2 * BN * 16, STAGE = IN_BYTES + U_BYTES;
  constexpr int S = BN == 64 ? 3 : 2;         // ring depth (DMA S - 1 stages ahead)
  constexpr int GI = NQ, GU = BN / 32, G = GI + GU;  // DMA pieces per wave per stage
  constexpr int NST = F45 ? 64 : 32;          // stores per lane per item (unconditional)
  // vmcnt saturates at 63: a smaller count only waits longer (in-order counter)
  constexpr int WFIRST = NST + G < 63 ? NST + G : 63, WST = NST < 63 ? NST : 63;
  static_assert(S * STAGE <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[S * STAGE];

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int tq = BN == 64 ? (wave & 3) : wave, nh = BN == 64 ? (wave >> 2) : 0;
  const int h = lane >> 5, r32 = lane & 31;
  const int Gd = gridDim.x;
  const int KT = q.KT;
  const int dh = F45 ? 0 : q.axis, dw = 1 - dh;  // the conv axis: H (7x1) or W (1x7, 5x5)
  const uint32_t rowb = (uint32_t)(q.W * q.C * 4);  // F(4,5): bytes per input row
  const float* x = static_cast<const float*>(g.A);
  const __amdgpu_buffer_rsrc_t ru = wrsrc(g.B, (q.dbg & 1) ? 0u : (uint32_t)q.u_bytes);
  const __amdgpu_buffer_rsrc_t rnil = wrsrc(g.B, 0u);
  // filter piece p = wave * GU + i covers (xi, quad) rows p * (64 / BN) + lane / BN, oc n0 + lane % BN
  uint32_t uoff[GU];
#pragma unroll
  for (int i = 0; i < GU; ++i)
    uoff[i] = (uint32_t)((((wave * GU + i) * (64 / BN) + lane / BN) * q.OCP + lane % BN) * 16);
  const uint32_t ustep = (uint32_t)(16 * q.OCP * 16);  // filter bytes per 8-channel stage

  auto tile_of = [&](uint32_t tc, uint32_t& n, int& o_h, int& o_w) __attribute__((always_inline)) {
    const uint32_t qa = fdiv(tc, q.fD1), i1 = tc - qa * (uint32_t)q.D1;
    n = fdiv(qa, q.fD0);
    const uint32_t i0 = qa - n * (uint32_t)q.D0;
    o_h = dh ? 2 * (int)i0 : (int)i0;   // the tile's first output pixel
    o_w = dh ? (int)i1 : (F45 ? 4 : 2) * (int)i1;
  };
  // input piece p = wave * GI + i: patch position p / NQ, tile group p % NQ;
  // lane L: tile 32 (p % NQ) + (L & 31), channel quad L >> 5
  struct Item {
    int64_t t0;
    int n0;
    __amdgpu_buffer_rsrc_t rin, rf;
    uint32_t ioff[GI];
    int ihw[F45 ? GI : 1];  // F(4,5): the patch's row at kh = 0 (tile / column out of range: far negative)
  };
  auto setup = [&](int item, bool live, Item& it) __attribute__((always_inline)) {
    const int itc = live ? item : 0;
    it.t0 = (int64_t)(itc / nbn) * T;
    it.n0 = (itc % nbn) * BN;
    const uint32_t nb0 = (uint32_t)(it.t0 / ((int64_t)q.D0 * q.D1));
    const __amdgpu_buffer_rsrc_t r = wrsrc(x + (int64_t)nb0 * q.img_floats, (q.dbg & 2) ? 0u : kOOB);
    it.rin = live ? r : rnil;
    it.rf = live ? ru : rnil;
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int p = wave * GI + i, pos = p / NQ;
      const int64_t t = it.t0 + (p % NQ) * 32 + r32;
      const bool tl = t < q.ntiles;
      uint32_t n;
      int oh, ow;
      tile_of(tl ? (uint32_t)t : 0u, n, oh, ow);
      const int ih = oh - q.pt + pos * dh, iw = ow - q.pl + pos * dw;
      if constexpr (F45) {
        // row kh is in range iff 0 <= ih + kh < H; the offset at kh = 0 may be
        // negative (top padding): kept as its 32-bit pattern, + kh rows at issue
        const bool okw = tl & ((unsigned)iw < (unsigned)q.W);
        it.ihw[i] = okw ? ih : -(1 << 20);
        it.ioff[i] = (uint32_t)(int)((((int64_t)(n - nb0) * q.H + ih) * q.W + iw) * q.C * 4 + h * 16);
      } else {
        const bool ok = tl & ((unsigned)ih < (unsigned)q.H) & ((unsigned)iw < (unsigned)q.W);
        it.ioff[i] = ok ? (uint32_t)((((int64_t)(n - nb0) * q.H + ih) * q.W + iw) * q.C * 4 + h * 16) : kOOB;
      }
    }
  };
  auto issue = [&](const Item& it, int kt) __attribute__((always_inline)) {
    char* base = smem + (kt % S) * STAGE;
    const uint32_t us = (uint32_t)(it.n0 * 16) + (uint32_t)kt * ustep;
    if constexpr (F45) {
      const uint32_t kh = fdiv((uint32_t)kt, q.fKTC), is = ((uint32_t)kt - kh * (uint32_t)q.KTC) * 32u;
#pragma unroll
      for (int i = 0; i < GI; ++i) {
        const uint32_t off = (unsigned)(it.ihw[i] + (int)kh) < (unsigned)q.H ? it.ioff[i] + kh * rowb : kOOB;
        bdma16(it.rin, off, is, base + (wave * GI + i) * 1024);
      }
    } else {
      const uint32_t is = (uint32_t)kt * 32u;
#pragma unroll
      for (int i = 0; i < GI; ++i) bdma16(it.rin, it.ioff[i], is, base + (wave * GI + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < GU; ++i) bdma16(it.rf, uoff[i], us, base + IN_BYTES + (wave * GU + i) * 1024);
  };

  // ---- fragments: lane (h, r32): tile r32 of the wave's 32, oc r32 of its
  // half, channel quad h; MFMA step s takes channel 4h + s
  f32x4 av[8], bv[8];
  auto read = [&](int kt) __attribute__((always_inline)) {
    const char* st = smem + (kt % S) * STAGE;
    f32x4 d[8];
#pragma unroll
    for (int p = 0; p < 8; ++p)
      d[p] = *reinterpret_cast<const f32x4*>(st + (((p * NQ + tq) * 2 + h) * 512) + r32 * 16);
#pragma unroll
    for (int xi = 0; xi < 8; ++xi)
      bv[xi] = *reinterpret_cast<const f32x4*>(st + IN_BYTES + ((xi * 2 + h) * BN + nh * 32 + r32) * 16);
    const f32x4 c21 = 5.25f, c17 = 4.25f, c5q = 1.25f, c5h = 2.5f, c5 = 5.f;
    av[0] = (d[6] - d[0]) + c21 * (d[2] - d[4]);
    av[7] = (d[7] - d[1]) + c21 * (d[3] - d[5]);
    const f32x4 e1 = (d[2] + d[6]) - c17 * d[4], o1 = (d[1] + d[5]) - c17 * d[3];
    av[1] = e1 + o1;
    av[2] = e1 - o1;
    const f32x4 e3 = (0.25f * d[2] + d[6]) - c5q * d[4], o3 = (0.5f * d[1] + 2.f * d[5]) - c5h * d[3];
    av[3] = e3 + o3;
    av[4] = e3 - o3;
    const f32x4 e5 = (4.f * d[2] + d[6]) - c5 * d[4], o5 = (2.f * d[1] + 0.5f * d[5]) - c5h * d[3];
    av[5] = e5 + o5;
    av[6] = e5 - o5;
  };

  f32x16 acc[8];
  auto mfma_pts = [&](int x0, int x1, const f32x4 (&a)[8], const f32x4 (&b)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int xi = x0; xi < x1; ++xi)
#pragma unroll
      for (int st = 0; st < 4; ++st) acc[xi] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[xi][st], b[xi][st], acc[xi], 0, 0, 0);
  };
  f32x4 pa[8], pb[8];  // the deferred points 6, 7 of the previous stage (only [6], [7] are live)
  int item = f32core::xcd_remap(blockIdx.x, Gd);
  if (item >= nwork) return;
  Item cur;
  setup(item, true, cur);
  issue(cur, 0);
  for (bool first = true;; first = false) {
#pragma unroll
    for (int xi = 0; xi < 8; ++xi) acc[xi] = (f32x16){};
    if (S == 3 && KT > 1) issue(cur, 1);
    for (int kt = 0; kt < KT; ++kt) {
      // stage kt landed: newer ops that may fly are (ring of 3) stage kt+1's
      // DMA and, in an item's first stage, the previous item's epilogue
      // stores (older than stage 1's DMA, newer than stage 0's)
      const bool more = S == 3 && kt + 1 < KT;
      if (kt == 0 && !first) {
        if (more) wwait_vm<WFIRST>();
        else wwait_vm<WST>();
      } else if (more) {
        wwait_vm<G>();
      } else {
        wwait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      // into the slot of stage kt-1 (ring of 3: kt+2; ring of 2: kt+1), read before this barrier
      if (kt + S - 1 < KT) issue(cur, kt + S - 1);
      // the last two transform points' MFMAs of stage kt-1 run here, in the
      // shadow of this stage's fragment reads and input transform
      if (kt > 0) mfma_pts(6, 8, pa, pb);
      read(kt);
      mfma_pts(0, 6, av, bv);
#pragma unroll
      for (int xi = 6; xi < 8; ++xi) {
        pa[xi] = av[xi];
        pb[xi] = bv[xi];
      }
    }
    mfma_pts(6, 8, pa, pb);
    const int64_t col = cur.n0 + nh * 32 + r32;
    const bool colok = col < g.N;
    float* cbase;
    int64_t cld;
    int cact;
    f32core::out_col(g, static_cast<float*>(g.C), colok ? col : 0, cbase, cld, cact);
    const float bias = (g.bias && colok) ? static_cast<const float*>(g.bias)[col] : 0.f;
    __syncthreads();  // the ring is free: slot 0 takes the next item's first stage
    const int next = item + Gd;
    const bool live = next < nwork;
    Item nx;
    setup(next, live, nx);
    issue(nx, 0);
    // ---- epilogue in registers: C/D row r -> tile 32 tq + (r & 3) + 8 (r >> 2) + 4 h
#pragma unroll
    for (int r = 0; r < 16 && F45; ++r) {
      const float s12 = acc[1][r] - acc[2][r], s34 = acc[3][r] - acc[4][r], s56 = acc[5][r] - acc[6][r];
      const float a12 = acc[1][r] + acc[2][r], a34 = acc[3][r] + acc[4][r], a56 = acc[5][r] + acc[6][r];
      float y[4];
      y[0] = ((acc[0][r] + a12) + a34) + a56;
      y[1] = (s12 + 2.f * s34) + 0.5f * s56;
      y[2] = (a12 + 4.f * a34) + 0.25f * a56;
      y[3] = ((s12 + 8.f * s34) + 0.125f * s56) + acc[7][r];
      const int64_t t = cur.t0 + tq * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const bool tl = t < q.ntiles;
      uint32_t n;
      int oh, ow;
      tile_of(tl ? (uint32_t)t : 0u, n, oh, ow);
      const int64_t row0 = ((int64_t)n * q.OH + oh) * q.OW + ow;
      const bool ok0 = tl && colok && !(q.dbg & 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool okj = ok0 && ow + j < q.OW;
        float* pj = okj ? cbase + (okj ? row0 + j : 0) * cld : reinterpret_cast<float*>(&kWinoTrash[lane]) + j;
        *pj = act3(y[j] + bias, cact);
      }
    }
#pragma unroll
    for (int r = 0; r < 16 && !F45; ++r) {
      const float y0 = ((((acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r])) + (acc[4][r] + acc[5][r])) + acc[6][r]);
      const float y1 = (((acc[1][r] - acc[2][r]) + 2.f * (acc[3][r] - acc[4][r])) + 0.5f * (acc[5][r] - acc[6][r])) +
                       acc[7][r];
      const int64_t t = cur.t0 + tq * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const bool tl = t < q.ntiles;
      uint32_t n;
      int oh, ow;
      tile_of(tl ? (uint32_t)t : 0u, n, oh, ow);
      const int64_t row0 = ((int64_t)n * q.OH + oh) * q.OW + ow, step = dh ? q.OW : 1;
      const bool ok0 = tl && colok && !(q.dbg & 4);
      const bool ok1 = ok0 && (dh ? oh + 1 < q.OH : ow + 1 < q.OW);
      float* p0 = ok0 ? cbase + (ok0 ? row0 : 0) * cld : reinterpret_cast<float*>(&kWinoTrash[lane]);
      float* p1 = ok1 ? cbase + (ok1 ? row0 + step : 0) * cld : reinterpret_cast<float*>(&kWinoTrash[lane]) + 1;
      *p0 = act3(y0 + bias, cact);
      *p1 = act3(y1 + bias, cact);
    }
    if (!live) break;
    item = next;
    cur = nx;
  }
}

std::atomic<int>& wino_state() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_CONV_ALGO");
    return (e && !std::strcmp(e, "direct")) ? 0 : 1;
  }());
  return v;
}

// forced variant (-1 auto: persistent blocks, 3: one work item per block, for A/B)
std::atomic<int>& wino_variant() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_WINO_TILE");
    return e ? std::atoi(e) : -1;
  }());
  return v;
}

bool al16p(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// F(2x2,3x3) oc block: 32 (128 tiles per item) when a 64-wide block would
// leave at least half of the last block empty (OC <= 32, OC = 96, 160, ...),
// else 64 (64 tiles). Measured per layer (profiles/r6_wino/layers_bn32.json):
// Conv2d_2a (OC 32) 4.33 ms direct -> 3.42 ms, Mixed_5x 3x3 OC 96 1.006 ->
// 0.905 and 1.436 -> 1.284 ms; OC 64 / 192 / 384 lose with 32 (5.51 -> 6.69,
// 7.26 -> 8.93, 0.92 -> 1.07 ms). TFA_WINO_BN=32/64 (or set_wino_bn) forces one.
std::atomic<int>& wino_bn_forced() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_WINO_BN");
    const int b = e ? std::atoi(e) : 0;
    return (b == 32 || b == 64) ? b : 0;
  }());
  return v;
}
int wino23_bn(int64_t OC) {
  const int forced = wino_bn_forced().load();
  return forced ? forced : ((OC % 64 != 0 && OC % 64 <= 32) ? 32 : 64);
}

}  // namespace

void set_conv_wino(int on) { wino_state().store(on ? 1 : 0); }
bool conv_wino_enabled() { return wino_state().load() != 0; }
void set_wino_tile(int v) { wino_variant().store(v); }
void set_wino_bn(int bn) {
  TFA_CHECK(bn == 0 || bn == 32 || bn == 64, "set_wino_bn: 0 (auto), 32 or 64");
  wino_bn_forced().store(bn);
}

int64_t conv_wino_ocp(int64_t OC) { return (OC + 63) / 64 * 64; }

// F(4,5) for 5x5 convs: opt-in (TFA_WINO_5X5=1, config.wino_5x5). Its f32
// error is 5.6e-7 of sum|a*b| on Inception's Mixed_5x b1_5x5, 5.0x the
// implicit-GEMM path's, above the 4x gate the default-on kernels pass
// (tests/test_gpu_wino.py). Read by the planner when it makes the filters.
std::atomic<int>& wino_5x5_state() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_WINO_5X5");
    return (e && e[0] == '1') ? 1 : 0;
  }());
  return v;
}
static bool wino_5x5_enabled() { return wino_5x5_state().load() != 0; }
void set_wino_5x5(int on) { wino_5x5_state().store(on ? 1 : 0); }

int conv_wino_kind(int64_t KH, int64_t KW, int64_t sh, int64_t sw, int64_t dh, int64_t dw, int64_t C, int64_t OC) {
  if (sh != 1 || sw != 1 || dh != 1 || dw != 1 || C <= 0 || OC <= 0 || C % 8 != 0 || OC % 4 != 0) return 0;
  if (KH == 3 && KW == 3) return 1;
  if (KH == 1 && KW == 7) return 2;
  if (KH == 7 && KW == 1) return 3;
  if (KH == 5 && KW == 5 && wino_5x5_enabled()) return 4;
  return 0;
}

int64_t conv_wino_filter_elems(int kind, int64_t C, int64_t OC) {
  return (kind == 1 ? 16 : kind == 4 ? 40 : 8) * C * conv_wino_ocp(OC);
}

// kind 1: U = G g G^T per (c, oc) into [C/8][16 xi][2][OCP][4 c];
// kinds 2/3: U = G7 g into [C/8][8 xi][2][OCP][4 c]; kind 4 (5x5): U = G5 g
// per filter row into [5 kh][C/8][8 xi][2][OCP][4 c]. fp64, rounded once to f32.
void conv_wino_filter(int kind, const float* w, int64_t C, int64_t OC, float* u) {
  static const double G[4][3] = {{1, 0, 0}, {.5, .5, .5}, {.5, -.5, .5}, {0, 0, 1}};
  // F(2,7), points {0, 1, -1, 2, -2, 1/2, -1/2, inf} (rows of G7: tests/test_wino.py)
  static const double G7[8][7] = {
      {-1, 0, 0, 0, 0, 0, 0},
      {-2. / 9, -2. / 9, -2. / 9, -2. / 9, -2. / 9, -2. / 9, -2. / 9},
      {-2. / 9, 2. / 9, -2. / 9, 2. / 9, -2. / 9, 2. / 9, -2. / 9},
      {1. / 90, 1. / 45, 2. / 45, 4. / 45, 8. / 45, 16. / 45, 32. / 45},
      {1. / 90, -1. / 45, 2. / 45, -4. / 45, 8. / 45, -16. / 45, 32. / 45},
      {32. / 45, 16. / 45, 8. / 45, 4. / 45, 2. / 45, 1. / 45, 1. / 90},
      {32. / 45, -16. / 45, 8. / 45, -4. / 45, 2. / 45, -1. / 45, 1. / 90},
      {0, 0, 0, 0, 0, 0, 1}};
  const int64_t OCP = conv_wino_ocp(OC);
  std::memset(u, 0, sizeof(float) * conv_wino_filter_elems(kind, C, OC));
  for (int64_t c = 0; c < C; ++c)
    for (int64_t o = 0; o < OC; ++o) {
      if (kind == 1) {
        double gg[3][3], t[4][3];
        for (int a = 0; a < 3; ++a)
          for (int b = 0; b < 3; ++b) gg[a][b] = w[((a * 3 + b) * C + c) * OC + o];
        for (int i = 0; i < 4; ++i)
          for (int b = 0; b < 3; ++b) t[i][b] = G[i][0] * gg[0][b] + G[i][1] * gg[1][b] + G[i][2] * gg[2][b];
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j) {
            const double v = t[i][0] * G[j][0] + t[i][1] * G[j][1] + t[i][2] * G[j][2];
            u[((((c / 8) * 16 + i * 4 + j) * 2 + (c / 4) % 2) * OCP + o) * 4 + c % 4] = static_cast<float>(v);
          }
      } else if (kind == 4) {
        // G5[i][k] = c_i p_i^k = G7[i][k] for the finite points (k < 5); the
        // inf point takes the last tap
        for (int kh = 0; kh < 5; ++kh)
          for (int i = 0; i < 8; ++i) {
            double v = 0;
            for (int k = 0; k < 5; ++k) {
              const double g5 = i == 7 ? (k == 4 ? 1.0 : 0.0) : G7[i][k];
              v += g5 * w[((kh * 5 + k) * C + c) * OC + o];
            }
            u[(((((int64_t)kh * (C / 8) + c / 8) * 8 + i) * 2 + (c / 4) % 2) * OCP + o) * 4 + c % 4] = static_cast<float>(v);
          }
      } else {
        // HWIO [1][7] or [7][1]: tap k at w[(k * C + c) * OC + o] either way
        for (int i = 0; i < 8; ++i) {
          double v = 0;
          for (int k = 0; k < 7; ++k) v += G7[i][k] * w[(k * C + c) * OC + o];
          u[((((c / 8) * 8 + i) * 2 + (c / 4) % 2) * OCP + o) * 4 + c % 4] = static_cast<float>(v);
        }
      }
    }
}

bool conv_wino_eligible(const ConvArgs& a) {
  if (!a.wino || !conv_wino_enabled()) return false;
  const int kind = conv_wino_kind(a.KH, a.KW, a.sh, a.sw, a.dh, a.dw, a.C, a.OC);
  if (kind == 0) return false;
  if (a.epi.n != 0 || a.act > ACT_RELU6) return false;
  if (!al16p(a.x) || !al16p(a.wino) || (a.bias && !al16p(a.bias))) return false;
  const int64_t tpi = kind == 1   ? ((a.OH + 1) / 2) * ((a.OW + 1) / 2)
                      : kind == 2 ? a.OH * ((a.OW + 1) / 2)
                      : kind == 4 ? a.OH * ((a.OW + 3) / 4)
                                  : ((a.OH + 1) / 2) * a.OW;
  const int64_t T = (kind == 1 ? 4096 : 8192) / wino23_bn(a.OC), ntiles = a.N * tpi;
  if (ntiles >= (int64_t(1) << 31)) return false;
  // a block's taps lie within (images a block spans + 1) images of its first
  // image: under 2^31 bytes for the input descriptor's 32-bit offsets
  if ((T / tpi + 2) * a.H * a.W * a.C * 4 >= (int64_t(1) << 31)) return false;
  if (conv_wino_filter_elems(kind, a.C, a.OC) * 4 >= (int64_t(1) << 31)) return false;
  if (kind != 1) {  // scalar stores
    for (int s = 0; s < a.seg.n; ++s)
      if (a.seg.act[s] > ACT_RELU6) return false;
    return true;
  }
  if (a.seg.n == 0) return al16p(a.y) && (a.ldc > 0 ? a.ldc : a.OC) % 4 == 0;
  for (int s = 0; s < a.seg.n; ++s) {
    if (a.seg.begin[s] % 4 != 0 || a.seg.ldc[s] % 4 != 0 || !al16p(a.seg.ptr[s])) return false;
    if (a.seg.act[s] > ACT_RELU6) return false;
  }
  return true;
}

void conv_wino_launch(const ConvArgs& a, hipStream_t s) {
  WinoGeom q;
  q.H = (int)a.H; q.W = (int)a.W; q.C = (int)a.C; q.OH = (int)a.OH; q.OW = (int)a.OW;
  q.pt = (int)a.pad_t; q.pl = (int)a.pad_l;
  q.TH = (int)((a.OH + 1) / 2); q.TW = (int)((a.OW + 1) / 2);
  q.OCP = (int)conv_wino_ocp(a.OC);
  const int kind = conv_wino_kind(a.KH, a.KW, a.sh, a.sw, a.dh, a.dw, a.C, a.OC);
  q.KTC = (int)(a.C / 8);
  q.KT = kind == 4 ? 5 * q.KTC : q.KTC;
  q.fKTC = make_fastdiv((uint32_t)q.KTC);
  q.axis = kind == 3 ? 1 : 0;
  // F(2,7) / F(4,5): tiles (n, i0, i1) over (D0, D1)
  q.D0 = (kind == 2 || kind == 4) ? (int)a.OH : q.TH;
  q.D1 = kind == 3 ? (int)a.OW : kind == 4 ? (int)((a.OW + 3) / 4) : q.TW;
  q.fD0 = make_fastdiv((uint32_t)q.D0);
  q.fD1 = make_fastdiv((uint32_t)q.D1);
  q.ntiles = kind == 1 ? a.N * q.TH * q.TW : a.N * (int64_t)q.D0 * q.D1;
  q.img_floats = a.H * a.W * a.C;
  q.u_bytes = conv_wino_filter_elems(kind, a.C, a.OC) * 4;
  static const int dbg = [] {
    const char* e = std::getenv("TFA_WINO_DEBUG");
    return e ? std::atoi(e) : 0;
  }();
  q.dbg = dbg;
  q.fTW = make_fastdiv((uint32_t)q.TW);
  q.fTH = make_fastdiv((uint32_t)q.TH);
  GemmArgs g{};
  g.M = a.N * a.OH * a.OW;
  g.N = a.OC;
  g.K = a.KH * a.KW * a.C;
  g.A = a.x;
  g.B = a.wino;
  g.C = a.y;
  g.ldc = a.ldc > 0 ? a.ldc : a.OC;
  g.bias = a.bias;
  g.act = a.act;
  g.batch = 1;
  g.seg = a.seg;
  const int bn = wino23_bn(a.OC);
  const int64_t TB = kind == 1 ? 4096 / bn : 8192 / bn;
  const int64_t nbt = (q.ntiles + TB - 1) / TB, nbn = (a.OC + bn - 1) / bn;
  TFA_CHECK(nbt * nbn < (int64_t(1) << 31), "conv_wino: grid too large");
  const int nwork = (int)(nbt * nbn);
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    (void)hipGetLastError();
    return n > 0 ? n : 256;
  }();
  const int per_cu = wino_variant().load() == 3 ? 0 : 1;  // 3: one item per block (no persistence), for A/B
  const int grid = per_cu ? std::min(nwork, ncu) : nwork;
  TFA_CHECK(!a.pool2 || kind == 1, "conv_wino: pooled epilogue on F(2x2,3x3) only");
  if (kind == 1) {
    TFA_CHECK(!a.pool2 || (a.OH % 2 == 0 && a.OW % 2 == 0 && a.seg.n == 0), "conv_wino: pooled epilogue geometry");
    auto k23 = bn == 32 ? (a.pool2 ? wino23_kernel<32, true> : wino23_kernel<32, false>)
                        : (a.pool2 ? wino23_kernel<64, true> : wino23_kernel<64, false>);
    hipLaunchKernelGGL(k23, dim3((unsigned)grid), dim3(512), 0, s, g, q, (int)nbn, nwork);
  }
  else if (kind == 4 && bn == 32)
    hipLaunchKernelGGL((wino27_kernel<32, true>), dim3((unsigned)grid), dim3(512), 0, s, g, q, (int)nbn, nwork);
  else if (kind == 4)
    hipLaunchKernelGGL((wino27_kernel<64, true>), dim3((unsigned)grid), dim3(512), 0, s, g, q, (int)nbn, nwork);
  else if (bn == 32)
    hipLaunchKernelGGL(wino27_kernel<32>, dim3((unsigned)grid), dim3(512), 0, s, g, q, (int)nbn, nwork);
  else
    hipLaunchKernelGGL(wino27_kernel<64>, dim3((unsigned)grid), dim3(512), 0, s, g, q, (int)nbn, nwork);
  TFA_LAUNCH_CHECK("conv_wino");
}

}  // namespace k
}  // namespace tfa

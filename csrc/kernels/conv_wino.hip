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
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "gemm_f32_core.h"

namespace tfa {
namespace k {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct WinoGeom {
  int H, W, C, OH, OW, pt, pl, TH, TW, OCP, KT;
  int64_t ntiles;
  int64_t img_floats;    // H * W * C
  int64_t u_bytes;       // the whole transformed filter
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

// NW = 4: one wave per SIMD, 4 * T * BN / 64 accumulators per lane; NW = 8:
// two waves per SIMD splitting the tiles (half the accumulators each, so one
// wave's LDS waits and barrier skew are covered by its partner's MFMAs)
template <int T, int BN, int S, int NW>
__global__ __launch_bounds__(64 * NW, 1) void wino23_kernel(GemmArgs g, WinoGeom q, int nbn) {
  constexpr int NTP = NW / 4;                                  // tile parts (waves per xi row)
  constexpr int TWV = T / NTP;                                 // tiles per wave
  constexpr int TG = TWV / 16, CG = BN / 16;                   // 16x16 MFMA tiles per wave
  constexpr int IN_BYTES = 16 * T * 16, U_BYTES = 16 * BN * 16, STAGE = IN_BYTES + U_BYTES;
  constexpr int GI = 16 * (T / 64) / NW, GU = 16 * (BN / 64) / NW, G = GI + GU;  // DMA pieces per wave
  constexpr int EP = BN + 4;                                   // epilogue row pitch (floats)
  constexpr int E_BYTES = 4 * 2 * T * EP * 4;
  constexpr int SMEM = S * STAGE > E_BYTES ? S * STAGE : E_BYTES;
  static_assert(T % 64 == 0 && BN % 64 == 0 && S >= 3 && (NW == 4 || NW == 8), "tile shape");
  static_assert(GI >= 1 && GU >= 1 && GI * NW == 16 * (T / 64) && GU * NW == 16 * (BN / 64), "whole DMA pieces");
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(4 * TG * CG * 4 * NTP <= 256, "accumulators");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int xr = wave & 3, tp = wave >> 2;  // xi row, tile part
  const int li = lane & 15, lq = lane >> 4;
  const int nwg = gridDim.x;
  const int wg = f32core::xcd_remap(blockIdx.x, nwg);
  const int64_t t0 = (int64_t)(wg / nbn) * T;
  const int n0 = (wg % nbn) * BN;
  const int KT = q.KT;

  // ---- descriptors: the input from the block's first image on (every valid
  // tap of the block lies within 2^31 bytes of it: conv_wino_eligible), the
  // whole filter, and an empty one (stages past the end)
  const uint32_t nb0 = (uint32_t)(t0 / ((int64_t)q.TH * q.TW));
  const __amdgpu_buffer_rsrc_t rin = wrsrc(static_cast<const float*>(g.A) + (int64_t)nb0 * q.img_floats, kOOB);
  const __amdgpu_buffer_rsrc_t ru = wrsrc(g.B, (uint32_t)q.u_bytes);
  const __amdgpu_buffer_rsrc_t rnil = wrsrc(g.B, 0u);
  // input piece p = wave * GI + i: patch position p / (T/64) (= 4 py + px),
  // tiles (p % (T/64)) * 64 + lane; byte offset per lane fixed for the loop
  uint32_t ioff[GI];
#pragma unroll
  for (int i = 0; i < GI; ++i) {
    const int p = wave * GI + i, pos = p / (T / 64), sub = p % (T / 64);
    const int py = pos >> 2, px = pos & 3;
    const int64_t t = t0 + sub * 64 + lane;
    const bool live = t < q.ntiles;
    const uint32_t tc = live ? (uint32_t)t : 0u;
    const uint32_t qa = fdiv(tc, q.fTW), tx = tc - qa * (uint32_t)q.TW;
    const uint32_t n = fdiv(qa, q.fTH), ty = qa - n * (uint32_t)q.TH;
    const int ih = 2 * (int)ty - q.pt + py, iw = 2 * (int)tx - q.pl + px;
    const bool ok = live & ((unsigned)ih < (unsigned)q.H) & ((unsigned)iw < (unsigned)q.W);
    ioff[i] = ok ? (uint32_t)((((int64_t)(n - nb0) * q.H + ih) * q.W + iw) * q.C * 4) : kOOB;
  }
  // filter piece p = wave * GU + i: elements p * 64 + lane of [16 xi][BN]
  uint32_t uoff[GU];
#pragma unroll
  for (int i = 0; i < GU; ++i) {
    const int e = (wave * GU + i) * 64 + lane, xi = e / BN, oc = e % BN;
    uoff[i] = (uint32_t)((xi * q.OCP + n0 + oc) * 16);
  }
  const uint32_t ustep = (uint32_t)(16 * q.OCP * 16);  // bytes per channel quad
  int kiss = 0;                                        // index of the next stage to issue

  auto issue = [&](int slot) __attribute__((always_inline)) {
    char* base = smem + slot * STAGE;
    const bool live = kiss < KT;
    const __amdgpu_buffer_rsrc_t ri = live ? rin : rnil, rf = live ? ru : rnil;
    const uint32_t is = (uint32_t)kiss * 16u, us = (uint32_t)kiss * ustep;
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int p = wave * GI + i, pos = p / (T / 64), sub = p % (T / 64);
      bdma16(ri, ioff[i], is, base + (pos * T + sub * 64) * 16);
    }
#pragma unroll
    for (int i = 0; i < GU; ++i) bdma16(rf, uoff[i], us, base + IN_BYTES + (wave * GU + i) * 1024);
    ++kiss;
  };

  // ---- fragments of one stage: A[xi_x][tile group], B[xi_x][oc group]
  struct Frag {
    float a[4][TG];
    float b[4][CG];
  };
  // B^T row xr: t = d[ra] + sgn * d[rb]
  const int ra = xr == 0 ? 0 : (xr == 2 ? 2 : 1);
  const int rb = xr == 0 ? 2 : (xr == 1 ? 2 : (xr == 2 ? 1 : 3));
  const float sgn = xr == 1 ? 1.f : -1.f;
  auto read = [&](int kt, Frag& f) __attribute__((always_inline)) {
    const char* st = smem + (kt % S) * STAGE;
    const float* in = reinterpret_cast<const float*>(st);
    const float* us = reinterpret_cast<const float*>(st + IN_BYTES);
#pragma unroll
    for (int gi = 0; gi < TG; ++gi) {
      const int tile = tp * TWV + 16 * gi + li;
      float t[4];
#pragma unroll
      for (int px = 0; px < 4; ++px) {
        const float a = in[((ra * 4 + px) * T + tile) * 4 + lq];
        const float b = in[((rb * 4 + px) * T + tile) * 4 + lq];
        t[px] = __builtin_fmaf(sgn, b, a);  // exact a +- b, one rounding
      }
      f.a[0][gi] = t[0] - t[2];
      f.a[1][gi] = t[1] + t[2];
      f.a[2][gi] = t[2] - t[1];
      f.a[3][gi] = t[1] - t[3];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int cg = 0; cg < CG; ++cg) f.b[j][cg] = us[((4 * xr + j) * BN + 16 * cg + li) * 4 + lq];
  };

  f32x4 acc[4][TG][CG];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int gi = 0; gi < TG; ++gi)
#pragma unroll
      for (int cg = 0; cg < CG; ++cg) acc[j][gi][cg] = (f32x4){0.f, 0.f, 0.f, 0.f};

  constexpr int NM = 4 * TG * CG;          // MFMAs per stage
  constexpr int NR = 8 * TG + 4 * CG;      // LDS reads per stage
  auto compute = [&](const Frag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int gi = 0; gi < TG; ++gi)
#pragma unroll
        for (int cg = 0; cg < CG; ++cg)
          acc[j][gi][cg] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[j][gi], f.b[j][cg], acc[j][gi][cg], 0, 0, 0);
  };

  // prologue: stages 0 .. S-2 (stages past KT read through the empty descriptor)
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);
  wwait_vm<G * (S - 2)>();  // stage 0 landed
  __builtin_amdgcn_s_barrier();
  Frag cur;
  read(0, cur);
  int kt = 0;
  // One stage: stage kt+1 retired for every wave (counted wait + barrier),
  // which also frees the slot of stage kt-1 for the DMA of stage kt+S-1;
  // then the stage's MFMAs with the next stage's fragment reads (and its
  // input transform) in their shadow.
  for (; kt + S - 1 < KT; ++kt) {
    wwait_vm<G * (S - 3)>();  // stage kt+1 landed (kt+2 .. kt+S-2 may fly)
    __builtin_amdgcn_s_barrier();
    issue((kt + S - 1) % S);
    Frag nxt;
    read(kt + 1, nxt);
    compute(cur);
    // MFMA, DMA piece, MFMA, ..., then MFMA, LDS read, MFMA, LDS read, ...
    f32core::sched_interleave<0, NM, G + NR, G, f32core::kSchedVmemRead, f32core::kSchedDsRead>();
    cur = nxt;
  }
  for (; kt + 1 < KT; ++kt) {
    wwait_vm<0>();
    __builtin_amdgcn_s_barrier();
    Frag nxt;
    read(kt + 1, nxt);
    compute(cur);
    f32core::sched_interleave<0, NM, NR, 0, f32core::kSchedVmemRead, f32core::kSchedDsRead>();
    cur = nxt;
  }
  compute(cur);
  __syncthreads();  // every wave is done with the ring: it becomes the epilogue exchange

  // ---- epilogue. A^T along x: this wave's rows m'[xr][px] (C/D layout of
  // 16x16x4: oc = 16 cg + (l & 15), tile = 16 gi + 4 (l >> 4) + r)
  float* E = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int gi = 0; gi < TG; ++gi)
#pragma unroll
    for (int cg = 0; cg < CG; ++cg)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float m0 = (acc[0][gi][cg][r] + acc[1][gi][cg][r]) + acc[2][gi][cg][r];
        const float m1 = (acc[1][gi][cg][r] - acc[2][gi][cg][r]) - acc[3][gi][cg][r];
        const int tile = tp * TWV + 16 * gi + 4 * lq + r, oc = 16 * cg + li;
        E[((xr * 2 + 0) * T + tile) * EP + oc] = m0;
        E[((xr * 2 + 1) * T + tile) * EP + oc] = m1;
      }
  __syncthreads();
  // A^T along y over the 4 xi rows; wave w writes tiles [w T/NW, (w+1) T/NW)
  constexpr int LPT = BN / 4, TPP = 64 / LPT;  // lanes per tile (float4 of oc), tiles per pass
  const int cq = lane % LPT, tr = lane / LPT;
  const int64_t col = n0 + 4 * cq;
  if (col >= g.N) return;
  float* cbase;
  int64_t cld;
  int cact;
  f32core::out_col(g, static_cast<float*>(g.C), col, cbase, cld, cact);
  const float* bias = static_cast<const float*>(g.bias);
  const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int ps = 0; ps < T / NW / TPP; ++ps) {
    const int tile = wave * (T / NW) + ps * TPP + tr;
    const int64_t t = t0 + tile;
    if (t >= q.ntiles) continue;
    const uint32_t tc = (uint32_t)t, qa = fdiv(tc, q.fTW), tx = tc - qa * (uint32_t)q.TW;
    const uint32_t n = fdiv(qa, q.fTH), ty = qa - n * (uint32_t)q.TH;
#pragma unroll
    for (int px = 0; px < 2; ++px) {
      const int ow = 2 * (int)tx + px;
      f32x4 e[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) e[w] = *reinterpret_cast<const f32x4*>(&E[((w * 2 + px) * T + tile) * EP + 4 * cq]);
      const f32x4 y0 = (e[0] + e[1]) + e[2];
      const f32x4 y1 = (e[1] - e[2]) - e[3];
#pragma unroll
      for (int py = 0; py < 2; ++py) {
        const int oh = 2 * (int)ty + py;
        const f32x4 v = py ? y1 : y0;
        float4 o;
        o.x = act3(v[0] + bv.x, cact);
        o.y = act3(v[1] + bv.y, cact);
        o.z = act3(v[2] + bv.z, cact);
        o.w = act3(v[3] + bv.w, cact);
        const int64_t row = ((int64_t)n * q.OH + oh) * q.OW + ow;
        if (ow < q.OW && oh < q.OH) *reinterpret_cast<float4*>(cbase + row * cld) = o;
      }
    }
  }
}

std::atomic<int>& wino_state() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_CONV_ALGO");
    return (e && !std::strcmp(e, "direct")) ? 0 : 1;
  }());
  return v;
}

// forced variant (-1 auto, 0: 4 waves (one per SIMD), 1: 8 waves; both 64 tiles x 64 oc)
std::atomic<int>& wino_variant() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_WINO_TILE");
    return e ? std::atoi(e) : -1;
  }());
  return v;
}

bool al16p(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

void set_conv_wino(int on) { wino_state().store(on ? 1 : 0); }
bool conv_wino_enabled() { return wino_state().load() != 0; }
void set_wino_tile(int v) { wino_variant().store(v); }

int64_t conv_wino_ocp(int64_t OC) { return (OC + 63) / 64 * 64; }

// U = G g G^T per (c, oc) in fp64, rounded once to f32, into [C/4][16 xi][OCP][4 c]
void conv_wino_filter(const float* w, int64_t C, int64_t OC, float* u) {
  static const double G[4][3] = {{1, 0, 0}, {.5, .5, .5}, {.5, -.5, .5}, {0, 0, 1}};
  const int64_t OCP = conv_wino_ocp(OC);
  std::memset(u, 0, sizeof(float) * 16 * C * OCP);
  for (int64_t c = 0; c < C; ++c)
    for (int64_t o = 0; o < OC; ++o) {
      double gg[3][3], t[4][3];
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) gg[a][b] = w[((a * 3 + b) * C + c) * OC + o];
      for (int i = 0; i < 4; ++i)
        for (int b = 0; b < 3; ++b) t[i][b] = G[i][0] * gg[0][b] + G[i][1] * gg[1][b] + G[i][2] * gg[2][b];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          const double v = t[i][0] * G[j][0] + t[i][1] * G[j][1] + t[i][2] * G[j][2];
          u[(((c / 4) * 16 + i * 4 + j) * OCP + o) * 4 + c % 4] = static_cast<float>(v);
        }
    }
}

bool conv_wino_shape_ok(int64_t KH, int64_t KW, int64_t sh, int64_t sw, int64_t dh, int64_t dw, int64_t C, int64_t OC) {
  return KH == 3 && KW == 3 && sh == 1 && sw == 1 && dh == 1 && dw == 1 && C % 4 == 0 && OC % 4 == 0 && C > 0 &&
         OC > 0;
}

bool conv_wino_eligible(const ConvArgs& a) {
  if (!a.wino || !conv_wino_enabled()) return false;
  if (!conv_wino_shape_ok(a.KH, a.KW, a.sh, a.sw, a.dh, a.dw, a.C, a.OC)) return false;
  if (a.epi.n != 0 || a.act > ACT_RELU6) return false;
  if (!al16p(a.x) || !al16p(a.wino) || (a.bias && !al16p(a.bias))) return false;
  const int64_t tpi = ((a.OH + 1) / 2) * ((a.OW + 1) / 2), ntiles = a.N * tpi;
  if (ntiles >= (int64_t(1) << 31)) return false;
  // a block's taps lie within (images a block spans + 1) images of its first
  // image: under 2^31 bytes for the input descriptor's 32-bit offsets
  if ((128 / tpi + 2) * a.H * a.W * a.C * 4 >= (int64_t(1) << 31)) return false;
  if (16 * a.C * conv_wino_ocp(a.OC) * 4 >= (int64_t(1) << 31)) return false;
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
  q.KT = (int)(a.C / 4);
  q.ntiles = a.N * q.TH * q.TW;
  q.img_floats = a.H * a.W * a.C;
  q.u_bytes = 16 * a.C * q.OCP * 4;
  q.fTW = make_fastdiv((uint32_t)q.TW);
  q.fTH = make_fastdiv((uint32_t)q.TH);
  GemmArgs g{};
  g.M = a.N * a.OH * a.OW;
  g.N = a.OC;
  g.K = 9 * a.C;
  g.A = a.x;
  g.B = a.wino;
  g.C = a.y;
  g.ldc = a.ldc > 0 ? a.ldc : a.OC;
  g.bias = a.bias;
  g.act = a.act;
  g.batch = 1;
  g.seg = a.seg;
  int v = wino_variant().load();
  if (v < 0) v = 1;
  const int T = 64, BN = 64;
  const int64_t nbt = (q.ntiles + T - 1) / T, nbn = (a.OC + BN - 1) / BN;
  TFA_CHECK(nbt * nbn < (int64_t(1) << 31), "conv_wino: grid too large");
  const dim3 grid((unsigned)(nbt * nbn));
  if (v == 0)
    hipLaunchKernelGGL((wino23_kernel<64, 64, 4, 4>), grid, dim3(256), 0, s, g, q, (int)nbn);
  else
    hipLaunchKernelGGL((wino23_kernel<64, 64, 4, 8>), grid, dim3(512), 0, s, g, q, (int)nbn);
  TFA_LAUNCH_CHECK("conv_wino");
}

}  // namespace k
}  // namespace tfa

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
  FastDivU32 fTW, fTH;
};

__device__ __forceinline__ void wglds16(const void* gp, void* lds) {
  __builtin_amdgcn_global_load_lds(gp, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wwait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

__device__ __forceinline__ const float* sel_ptr(const float* p, const float* z, bool ok) {
  // an arithmetic select: a ternary here becomes an exec-masked branch per
  // piece, and a branch between LDS-DMA issues drains the queue (vmcnt(0))
  const uint64_t m = 0ull - (uint64_t)ok;
  return reinterpret_cast<const float*>((reinterpret_cast<uint64_t>(p) & m) | (reinterpret_cast<uint64_t>(z) & ~m));
}

template <int T, int BN, int S>
__global__ __launch_bounds__(256, 1) void wino23_kernel(GemmArgs g, WinoGeom q, int nbn) {
  constexpr int TG = T / 16, CG = BN / 16;                    // 16x16 MFMA tiles: tile groups, oc groups
  constexpr int IN_BYTES = 16 * T * 16, U_BYTES = 16 * BN * 16, STAGE = IN_BYTES + U_BYTES;
  constexpr int GI = T / 16, GU = BN / 16, G = GI + GU;       // DMA pieces per wave per stage
  constexpr int EP = BN + 4;                                  // epilogue row pitch (floats)
  constexpr int E_BYTES = 4 * 2 * T * EP * 4;
  constexpr int SMEM = S * STAGE > E_BYTES ? S * STAGE : E_BYTES;
  static_assert(T % 64 == 0 && BN % 32 == 0 && S >= 3, "whole DMA pieces per wave, >= 3 stages");
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(4 * TG * CG * 4 <= 256, "accumulators");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int li = lane & 15, lq = lane >> 4;
  const int nwg = gridDim.x;
  const int wg = f32core::xcd_remap(blockIdx.x, nwg);
  const int64_t t0 = (int64_t)(wg / nbn) * T;
  const int n0 = (wg % nbn) * BN;
  const float* x = static_cast<const float*>(g.A);
  const float* u = static_cast<const float*>(g.B);
  const float* zero = f32core::kZeroPage;
  const int KT = q.KT;

  // ---- DMA sources. Input piece i of wave w: patch row py = w, column
  // px = i / (T/64), tiles (i % (T/64)) * 64 + lane; fixed per lane except
  // for the channel offset (advanced by 4 floats per stage).
  const float* isrc[GI];
  bool iok[GI];
#pragma unroll
  for (int i = 0; i < GI; ++i) {
    const int px = i / (T / 64), sub = i % (T / 64);
    const int64_t t = t0 + sub * 64 + lane;
    const bool live = t < q.ntiles;
    const uint32_t tc = live ? (uint32_t)t : 0u;
    const uint32_t qa = fdiv(tc, q.fTW), tx = tc - qa * (uint32_t)q.TW;
    const uint32_t n = fdiv(qa, q.fTH), ty = qa - n * (uint32_t)q.TH;
    const int ih = 2 * (int)ty - q.pt + wave, iw = 2 * (int)tx - q.pl + px;
    iok[i] = live & ((unsigned)ih < (unsigned)q.H) & ((unsigned)iw < (unsigned)q.W);
    const int64_t off = iok[i] ? (((int64_t)n * q.H + ih) * q.W + iw) * q.C : 0;
    isrc[i] = x + off;
  }
  // filter piece i of wave w: elements i*64 + lane of the wave's [4 xi][BN]
  uint32_t uoff[GU];
#pragma unroll
  for (int i = 0; i < GU; ++i) {
    const int e = i * 64 + lane, xl = e / BN, oc = e % BN;
    uoff[i] = (uint32_t)((xl * q.OCP + oc) * 4);
  }
  const float* ubase = u + ((int64_t)(4 * wave) * q.OCP + n0) * 4;
  const int64_t ustep = (int64_t)16 * q.OCP * 4;  // floats per channel quad
  int64_t coff = 0;                               // input channel offset of the next stage to issue
  int kiss = 0;                                   // index of the next stage to issue

  auto issue = [&](int slot) __attribute__((always_inline)) {
    char* base = smem + slot * STAGE;
    const bool live = kiss < KT;
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int px = i / (T / 64), sub = i % (T / 64);
      wglds16(sel_ptr(isrc[i] + coff, zero, iok[i] & live), base + ((wave * 4 + px) * T + sub * 64) * 16);
    }
#pragma unroll
    for (int i = 0; i < GU; ++i)
      wglds16(sel_ptr(ubase + uoff[i], zero, live), base + IN_BYTES + (4 * wave * BN + i * 64) * 16);
    coff += 4;
    ubase += ustep;
    ++kiss;
  };

  // ---- fragments of one stage: A[xi_x][tile group], B[xi_x][oc group]
  struct Frag {
    float a[4][TG];
    float b[4][CG];
  };
  // B^T row `wave`: t = d[ra] + sgn * d[rb]
  const int ra = wave == 0 ? 0 : (wave == 2 ? 2 : 1);
  const int rb = wave == 0 ? 2 : (wave == 1 ? 2 : (wave == 2 ? 1 : 3));
  const float sgn = wave == 1 ? 1.f : -1.f;
  auto read = [&](int kt, Frag& f) __attribute__((always_inline)) {
    const char* st = smem + (kt % S) * STAGE;
    const float* in = reinterpret_cast<const float*>(st);
    const float* us = reinterpret_cast<const float*>(st + IN_BYTES);
#pragma unroll
    for (int gi = 0; gi < TG; ++gi) {
      const int tile = 16 * gi + li;
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
      for (int cg = 0; cg < CG; ++cg) f.b[j][cg] = us[((4 * wave + j) * BN + 16 * cg + li) * 4 + lq];
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
  auto stage = [&](int kt, auto do_issue, auto do_read) __attribute__((always_inline)) {
    constexpr bool ISSUE = decltype(do_issue)::value, READ = decltype(do_read)::value;
    if constexpr (ISSUE) wwait_vm<G * (S - 3)>();  // stage kt+1 landed (kt+2 .. kt+S-2 may fly)
    else wwait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if constexpr (ISSUE) issue((kt + S - 1) % S);
    Frag nxt;
    if constexpr (READ) read(kt + 1, nxt);
    (void)nxt;
    return nxt;
  };
  Frag cur;
  auto compute = [&](const Frag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int gi = 0; gi < TG; ++gi)
#pragma unroll
        for (int cg = 0; cg < CG; ++cg)
          acc[j][gi][cg] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[j][gi], f.b[j][cg], acc[j][gi][cg], 0, 0, 0);
  };

  // prologue: stages 0 .. S-2 (stages past KT read zero pages only)
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);
  wwait_vm<G * (S - 2)>();  // stage 0 landed
  __builtin_amdgcn_s_barrier();
  read(0, cur);
  int kt = 0;
  for (; kt + S - 1 < KT; ++kt) {
    Frag nxt = stage(kt, std::true_type{}, std::true_type{});
    compute(cur);
    // MFMA, DMA piece, MFMA, ..., then MFMA, LDS read, MFMA, LDS read, ...
    f32core::sched_interleave<0, NM, G + NR, G, f32core::kSchedVmemRead, f32core::kSchedDsRead>();
    cur = nxt;
  }
  for (; kt + 1 < KT; ++kt) {
    Frag nxt = stage(kt, std::false_type{}, std::true_type{});
    compute(cur);
    f32core::sched_interleave<0, NM, NR, 0, f32core::kSchedVmemRead, f32core::kSchedDsRead>();
    cur = nxt;
  }
  (void)stage(kt, std::false_type{}, std::false_type{});
  compute(cur);
  __syncthreads();  // every wave is done with the ring: it becomes the epilogue exchange

  // ---- epilogue. A^T along x: this wave's rows m'[w][px] (C/D layout of
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
        const int tile = 16 * gi + 4 * lq + r, oc = 16 * cg + li;
        E[((wave * 2 + 0) * T + tile) * EP + oc] = m0;
        E[((wave * 2 + 1) * T + tile) * EP + oc] = m1;
      }
  __syncthreads();
  // A^T along y over the 4 waves' rows; wave w writes tiles [w T/4, (w+1) T/4)
  constexpr int LPT = BN / 4, TPP = 64 / LPT;  // lanes per tile (float4 of oc), tiles per pass
  const int cq = lane % LPT, tr = lane / LPT;
  const int64_t col = n0 + 4 * cq;
  if (col >= g.N) return;
  float* Cb = static_cast<float*>(g.C);
  float* cbase;
  int64_t cld;
  int cact;
  f32core::out_col(g, Cb, col, cbase, cld, cact);
  const float* bias = static_cast<const float*>(g.bias);
  const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int ps = 0; ps < T / 4 / TPP; ++ps) {
    const int tile = wave * (T / 4) + ps * TPP + tr;
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
      if (ow >= q.OW) continue;
#pragma unroll
      for (int py = 0; py < 2; ++py) {
        const int oh = 2 * (int)ty + py;
        if (oh >= q.OH) continue;
        const f32x4 v = py ? y1 : y0;
        float4 o;
        o.x = act_fast(v[0] + bv.x, cact);
        o.y = act_fast(v[1] + bv.y, cact);
        o.z = act_fast(v[2] + bv.z, cact);
        o.w = act_fast(v[3] + bv.w, cact);
        const int64_t row = ((int64_t)n * q.OH + oh) * q.OW + ow;
        *reinterpret_cast<float4*>(cbase + row * cld) = o;
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

// forced variant (-1 auto, 0: 64 tiles x 64 oc, 1: 128 tiles x 32 oc)
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
  const int64_t ntiles = a.N * ((a.OH + 1) / 2) * ((a.OW + 1) / 2);
  if (ntiles >= (int64_t(1) << 31)) return false;
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
  if (v < 0) v = a.OC <= 32 ? 1 : 0;
  const int T = v == 1 ? 128 : 64, BN = v == 1 ? 32 : 64;
  const int64_t nbt = (q.ntiles + T - 1) / T, nbn = (a.OC + BN - 1) / BN;
  TFA_CHECK(nbt * nbn < (int64_t(1) << 31), "conv_wino: grid too large");
  const dim3 grid((unsigned)(nbt * nbn));
  if (v == 1)
    hipLaunchKernelGGL((wino23_kernel<128, 32, 3>), grid, dim3(256), 0, s, g, q, (int)nbn);
  else
    hipLaunchKernelGGL((wino23_kernel<64, 64, 4>), grid, dim3(256), 0, s, g, q, (int)nbn);
  TFA_LAUNCH_CHECK("conv_wino");
}

}  // namespace k
}  // namespace tfa

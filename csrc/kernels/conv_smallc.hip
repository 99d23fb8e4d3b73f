// Direct f32 Conv2D for tiny reductions (KH*KW*C <= 32: the RGB stem of every
// CNN, e.g. Inception-v3 Conv2d_1a 3x3x3 -> 32 and VGG-16 conv1_1 3x3x3 -> 64)
// on v_mfma_f32_32x32x2f32, NHWC input, HWIO filter.
//
// The implicit-GEMM core (gemm.hip) stages A/B tiles through LDS in k tiles of
// 16; with K = 27 that is two k tiles per block, each paying a barrier, a
// scalar im2col loader with per-element index arithmetic and a full prologue
// and epilogue for 27 MACs per output. Here:
//  * the whole filter lives in registers for the kernel's life: lane l holds
//    W[k = 2s + (l >> 5)][n = 32j + (l & 31)] for every k-step s and column
//    tile j (the B operand layout of 32x32x2), loaded once per wave;
//  * the per-lane tap table (k -> filter row/col offset and channel) is in
//    registers too, so an A element is one bounds test and one global load
//    from the output pixel's window origin (no LDS, no barriers);
//  * each wave walks 32-pixel groups grid-stride, two groups in flight, and
//    writes bias + activation straight from the accumulators.
// The k order of every output (k-steps of 2, ascending) is the implicit-GEMM
// core's, so the results are bitwise identical to it (tests/test_gpu_conv_smallc.py).
#include <atomic>
#include <cstdlib>

#include "gemm_internal.h"
#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct SmallConv {
  int64_t M;  // N * OH * OW output pixels
  int H, W, C, KW, OH, OW, sh, sw, dh, dw, pt, pl, K, OC;
  int64_t ldc;
  const float* x;
  const float* w;
  const float* bias;
  float* y;
  int act;
  FastDivU32 fOW, fOH;
};

template <int KS, int TN, bool FAST, bool PAD = false>
__global__ __launch_bounds__(256) void conv_smallc_kernel(SmallConv p) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5, col = lane & 31;
  // tap table and filter registers (constant-indexed: fully unrolled)
  int toff[KS], tdy[KS], tdx[KS];
  float b[KS][TN];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    // k-step s pairs k = 8(s/4) + s%4 (lanes 0-31) with k + 4 (lanes 32-63),
    // the f32 GEMM cores' order (gemm_g2_core.h), so results match them bitwise
    const int k = 8 * (s >> 2) + (s & 3) + 4 * h;
    if (k < p.K) {
      const int c = k % p.C, t = k / p.C;
      tdy[s] = (t / p.KW) * p.dh;
      tdx[s] = (t % p.KW) * p.dw;
      toff[s] = (tdy[s] * p.W + tdx[s]) * p.C + c;
    } else {
      tdy[s] = 1 << 29;  // never in bounds: the padded k reads 0
      tdx[s] = 0;
      toff[s] = 0;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = 32 * j + col;
      b[s][j] = (k < p.K && n < p.OC) ? p.w[(int64_t)k * p.OC + n] : 0.f;
    }
  }
  float bv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = 32 * j + col;
    bv[j] = (p.bias && n < p.OC) ? p.bias[n] : 0.f;
  }

  const int64_t groups = (p.M + 31) / 32;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wave0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if constexpr (FAST) {
    // every tap of every output pixel is inside the image (no padding, checked
    // on the host) and the input is < 4 GiB (the output is addressed from a
    // 64-bit base per 32-pixel group): a tap is one 32-bit add
    // and one load off the uniform base, pixels past M re-read pixel 0 (never
    // stored), and the epilogue is specialised per activation with one bounds
    // test per group. Same k order and MFMA sequence: bitwise the generic path.
    uint32_t tb[KS];
    bool kv[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      tb[s] = (uint32_t)toff[s] * 4u;
      kv[s] = tdy[s] < (1 << 29);
    }
    const char* xb = reinterpret_cast<const char*>(p.x);
    char* yb = reinterpret_cast<char*>(p.y);
    const uint32_t M = (uint32_t)p.M, HWC = (uint32_t)(p.H * p.W * p.C), ldc = (uint32_t)p.ldc;
    const uint32_t rs = (uint32_t)(p.sh * p.W * p.C), cs = (uint32_t)(p.sw * p.C);
    auto run = [&](auto act_c) __attribute__((always_inline)) {
      constexpr int ACT = decltype(act_c)::value;
      for (uint32_t g0 = 2 * (uint32_t)wave0; g0 < (uint32_t)groups; g0 += 2 * (uint32_t)nwaves) {
        float a[2][KS];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint32_t m = (g0 + q) * 32 + col;
          const uint32_t mm = m < M ? m : 0u;
          const uint32_t t = fdiv(mm, p.fOW);
          const uint32_t ow = mm - t * (uint32_t)p.OW;
          const uint32_t n = fdiv(t, p.fOH);
          const uint32_t oh = t - n * (uint32_t)p.OH;
          if constexpr (PAD) {
            // padded (SAME) convs: a tap outside the image reads the base
            // (any valid address) and contributes 0; 32-bit signed offsets
            const int ih0 = (int)(oh * (uint32_t)p.sh) - p.pt, iw0 = (int)(ow * (uint32_t)p.sw) - p.pl;
            const int ob = (int)(n * HWC) + (ih0 * p.W + iw0) * p.C;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
              const int ih = ih0 + tdy[s], iw = iw0 + tdx[s];
              const bool inb = kv[s] & ((unsigned)ih < (unsigned)p.H) & ((unsigned)iw < (unsigned)p.W);
              const uint32_t off = inb ? (uint32_t)(ob * 4 + (int)tb[s]) : 0u;
              const float v = *reinterpret_cast<const float*>(xb + off);
              a[q][s] = inb ? v : 0.f;
            }
          } else {
            const uint32_t ob = (n * HWC + oh * rs + ow * cs) * 4u;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
              const float v = *reinterpret_cast<const float*>(xb + (ob + tb[s]));
              a[q][s] = kv[s] ? v : 0.f;
            }
          }
        }
        f32x16 acc[2][TN];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[q][j][r] = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[q][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][s], b[s][j], acc[q][j], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (g0 + q >= (uint32_t)groups) break;
          const uint32_t m0 = (g0 + q) * 32 + 4 * h;
          const bool full = (g0 + q + 1) * 32 <= M;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const uint32_t n = 32 * j + col;
            if (n >= (uint32_t)p.OC) continue;
            // 64-bit group base (the output may exceed 4 GiB), 32-bit row offsets
            char* yg = yb + ((uint64_t)m0 * ldc + n) * 4u;
            float v[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              v[r] = acc[q][j][r] + bv[j];
              if (ACT == ACT_RELU) v[r] = v[r] > 0.f ? v[r] : 0.f;
              if (ACT == ACT_RELU6) v[r] = v[r] > 0.f ? (v[r] < 6.f ? v[r] : 6.f) : 0.f;
            }
            if (full) {  // straight-line stores; only the last group is partial
#pragma unroll
              for (int r = 0; r < 16; ++r)
                *reinterpret_cast<float*>(yg + (uint32_t)((r & 3) + 8 * (r >> 2)) * ldc * 4u) = v[r];
            } else {
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                const uint32_t ro = (uint32_t)((r & 3) + 8 * (r >> 2));
                if (m0 + ro < M) *reinterpret_cast<float*>(yg + ro * ldc * 4u) = v[r];
              }
            }
          }
        }
      }
    };
    if (p.act == ACT_RELU) run(std::integral_constant<int, ACT_RELU>{});
    else if (p.act == ACT_RELU6) run(std::integral_constant<int, ACT_RELU6>{});
    else run(std::integral_constant<int, ACT_NONE>{});
    return;
  }
  // two 32-pixel groups per pass: 2*KS independent loads in flight per lane
  for (int64_t g0 = 2 * wave0; g0 < groups; g0 += 2 * nwaves) {
    float a[2][KS];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t m = (g0 + q) * 32 + col;  // A row of this lane = output pixel
      const bool live = (g0 + q) < groups && m < p.M;
      const uint32_t mm = live ? (uint32_t)m : 0u;  // M < 2^32 (conv_smallc_eligible)
      const uint32_t t = fdiv(mm, p.fOW);
      const int ow = (int)(mm - t * (uint32_t)p.OW);
      const uint32_t n = fdiv(t, p.fOH);
      const int oh = (int)(t - n * (uint32_t)p.OH);
      const int ih0 = oh * p.sh - p.pt, iw0 = ow * p.sw - p.pl;
      const float* org = p.x + (int64_t)n * p.H * p.W * p.C + ((int64_t)ih0 * p.W + iw0) * p.C;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int ih = ih0 + tdy[s], iw = iw0 + tdx[s];
        const bool inb = live && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        const float v = *(inb ? org + toff[s] : p.x);  // padding taps read a safe address
        a[q][s] = inb ? v : 0.f;
      }
    }
    f32x16 acc[2][TN];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][j][r] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[q][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][s], b[s][j], acc[q][j], 0, 0, 0);
    // C/D layout: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (g0 + q >= groups) break;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = 32 * j + col;
        if (n >= p.OC) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t m = (g0 + q) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (m < p.M) p.y[m * p.ldc + n] = act_fast(acc[q][j][r] + bv[j], p.act);
        }
      }
    }
  }
}

template <int KS>
void launch_ks(const SmallConv& p, int tn, int fast, hipStream_t s) {
  const int64_t groups = (p.M + 31) / 32;
  const int64_t waves = (groups + 1) / 2;
  // enough waves to fill 256 CUs x 8 waves a few times over; grid-stride beyond
  const int64_t blocks = std::min<int64_t>((waves + 3) / 4, 256 * 16);
  const dim3 g((unsigned)blocks), b(256);
  if (fast == 2) {  // 32-bit offsets, padding taps checked
    if (tn == 1) hipLaunchKernelGGL((conv_smallc_kernel<KS, 1, true, true>), g, b, 0, s, p);
    else hipLaunchKernelGGL((conv_smallc_kernel<KS, 2, true, true>), g, b, 0, s, p);
  } else if (fast) {
    if (tn == 1) hipLaunchKernelGGL((conv_smallc_kernel<KS, 1, true>), g, b, 0, s, p);
    else hipLaunchKernelGGL((conv_smallc_kernel<KS, 2, true>), g, b, 0, s, p);
  } else {
    if (tn == 1) hipLaunchKernelGGL((conv_smallc_kernel<KS, 1, false>), g, b, 0, s, p);
    else hipLaunchKernelGGL((conv_smallc_kernel<KS, 2, false>), g, b, 0, s, p);
  }
}

// TFA_CONV_SMALLC=0 (or set_conv_smallc(0)) sends these convs to the
// implicit-GEMM core instead (A/B and the bitwise-equality test)
std::atomic<int>& smallc_state() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_CONV_SMALLC");
    return (e && std::atoi(e) == 0) ? 0 : 1;
  }());
  return v;
}
bool smallc_enabled() { return smallc_state().load() != 0; }

// ---- VALID 3x3 max pool -> 1x1 conv (+ bias + act), one kernel. The 1x1 conv's
// A element (pixel m, channel k) is the max of the pool window, computed from
// float4 loads of 4 channels (a lane's k-steps 4j..4j+3 take channels
// 8j + 4h + 0..3: the same k order as above, so the conv part matches the
// GEMM cores bitwise); the filter (C x OC, C <= 64) lives in registers.
struct PoolConv {
  uint32_t M;  // N * PH * PW output pixels
  int H, W, C, PH, PW, pkh, pkw, psh, psw, OC;
  uint32_t ldc;
  const float* x;
  const float* w;
  const float* bias;
  float* y;
  int act;
  FastDivU32 fPW, fPH;
};

template <int KS, int TN>
__global__ __launch_bounds__(256) void pool_conv1x1_kernel(PoolConv p) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5, col = lane & 31;
  float b[KS][TN];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 8 * (s >> 2) + (s & 3) + 4 * h;  // < C = 2 KS
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = 32 * j + col;
      b[s][j] = n < p.OC ? p.w[k * p.OC + n] : 0.f;
    }
  }
  float bv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = 32 * j + col;
    bv[j] = (p.bias && n < p.OC) ? p.bias[n] : 0.f;
  }
  const uint32_t groups = (p.M + 31) / 32;
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t wave0 = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const char* xb = reinterpret_cast<const char*>(p.x);
  char* yb = reinterpret_cast<char*>(p.y);
  const uint32_t rowb = (uint32_t)(p.W * p.C) * 4u, pixb = (uint32_t)p.C * 4u;
  const uint64_t imgb = (uint64_t)rowb * (uint32_t)p.H;
  // the group's pooled A tile goes through this wave's LDS rows: the window
  // loads are coalesced (16 lanes x 16 B cover a 64-channel pixel), the
  // fragment reads then take a lane's channels 8j + 4h + 0..3 of its pixel
  constexpr int C = 2 * KS, QPP = C / 4, PPI = 64 / QPP, NIT = 32 / PPI, TP = C + 4;  // TP: row pitch (floats)
  __shared__ __attribute__((aligned(16))) float tile_all[4][32 * TP];
  float* tile = tile_all[threadIdx.x >> 6];
  const int cq = lane % QPP, pr = lane / QPP;
  auto run = [&](auto act_c) __attribute__((always_inline)) {
    constexpr int ACT = decltype(act_c)::value;
    for (uint32_t g0 = wave0; g0 < groups; g0 += nwaves) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int pi = it * PPI + pr;
        const uint32_t m = g0 * 32 + (uint32_t)pi;
        const uint32_t mm = m < p.M ? m : 0u;  // pixels past M re-read pixel 0 (never stored)
        const uint32_t t = fdiv(mm, p.fPW);
        const uint32_t pw = mm - t * (uint32_t)p.PW;
        const uint32_t n = fdiv(t, p.fPH);
        const uint32_t ph = t - n * (uint32_t)p.PH;
        // VALID pool: every window tap is inside the image; 64-bit image
        // base, 32-bit offsets inside one image (< 4 GiB: eligible)
        const char* ib = xb + (uint64_t)n * imgb;
        const uint32_t ob = ((ph * (uint32_t)p.psh) * (uint32_t)p.W + pw * (uint32_t)p.psw) * pixb + (uint32_t)(16 * cq);
        float4 v = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) {
            const float4 u = *reinterpret_cast<const float4*>(ib + (ob + (uint32_t)dy * rowb + (uint32_t)dx * pixb));
            v.x = fmaxf(v.x, u.x);
            v.y = fmaxf(v.y, u.y);
            v.z = fmaxf(v.z, u.z);
            v.w = fmaxf(v.w, u.w);
          }
        *reinterpret_cast<float4*>(&tile[pi * TP + 4 * cq]) = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float a[KS];
#pragma unroll
      for (int j = 0; j < KS / 4; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(&tile[col * TP + 8 * j + 4 * h]);
        a[4 * j] = v.x;
        a[4 * j + 1] = v.y;
        a[4 * j + 2] = v.z;
        a[4 * j + 3] = v.w;
      }
      // the next group's tile writes wait for these reads (they feed the MFMAs below)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      f32x16 acc[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s][j], acc[j], 0, 0, 0);
      const uint32_t m0 = g0 * 32 + 4 * h;
      const bool full = (g0 + 1) * 32 <= p.M;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const uint32_t nn = 32 * j + col;
        if (nn >= (uint32_t)p.OC) continue;
        const uint32_t base = m0 * p.ldc + nn;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          v[r] = acc[j][r] + bv[j];
          if (ACT == ACT_RELU) v[r] = v[r] > 0.f ? v[r] : 0.f;
          if (ACT == ACT_RELU6) v[r] = v[r] > 0.f ? (v[r] < 6.f ? v[r] : 6.f) : 0.f;
        }
        if (full) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            *reinterpret_cast<float*>(yb + (base + (uint32_t)((r & 3) + 8 * (r >> 2)) * p.ldc) * 4u) = v[r];
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t ro = (uint32_t)((r & 3) + 8 * (r >> 2));
            if (m0 + ro < p.M) *reinterpret_cast<float*>(yb + (base + ro * p.ldc) * 4u) = v[r];
          }
        }
      }
    }
  };
  if (p.act == ACT_RELU) run(std::integral_constant<int, ACT_RELU>{});
  else if (p.act == ACT_RELU6) run(std::integral_constant<int, ACT_RELU6>{});
  else run(std::integral_constant<int, ACT_NONE>{});
}

// Wave-specialised variant: waves 0-1 of a block only pool (coalesced window
// loads, many in flight) into a two-set LDS ring, waves 2-3 only run the
// MFMAs and stores of the set the producers filled one step earlier; one
// block barrier per step. Step i of block b covers groups 2 (i B + b) + {0, 1}
// (consumer c takes the + c one), B = gridDim.x.
template <int KS, int TN>
__global__ __launch_bounds__(256) void pool_conv1x1_ws_kernel(PoolConv p) {
  constexpr int C = 2 * KS, QPP = C / 4, TP = C + 4, PER = QPP / 2;  // PER: float4 outputs per producer lane per step
  __shared__ __attribute__((aligned(16))) float ring[2][2][32 * TP];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = lane >> 5, col = lane & 31;
  const uint32_t groups = (p.M + 31) / 32;
  const uint32_t B = gridDim.x, b0 = blockIdx.x;
  const uint32_t nsteps = groups > 2 * b0 ? (groups - 2 * b0 + 2 * B - 1) / (2 * B) : 0;  // block-uniform
  const char* xb = reinterpret_cast<const char*>(p.x);
  char* yb = reinterpret_cast<char*>(p.y);
  const uint32_t rowb = (uint32_t)(p.W * p.C) * 4u, pixb = (uint32_t)p.C * 4u;
  const uint64_t imgb = (uint64_t)rowb * (uint32_t)p.H;
  auto produce = [&](uint32_t i) __attribute__((always_inline)) {
    const int pl = threadIdx.x;  // 0..127
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int el = e * 128 + pl, tt = el / (32 * QPP), px = (el / QPP) % 32, cq = el % QPP;
      const uint32_t g = 2 * (i * B + b0) + (uint32_t)tt;
      const uint32_t m = g * 32 + (uint32_t)px;
      const uint32_t mm = (g < groups && m < p.M) ? m : 0u;  // never stored
      const uint32_t t = fdiv(mm, p.fPW);
      const uint32_t pw = mm - t * (uint32_t)p.PW;
      const uint32_t n = fdiv(t, p.fPH);
      const uint32_t ph = t - n * (uint32_t)p.PH;
      const char* ib = xb + (uint64_t)n * imgb;
      const uint32_t ob = ((ph * (uint32_t)p.psh) * (uint32_t)p.W + pw * (uint32_t)p.psw) * pixb + (uint32_t)(16 * cq);
      float4 v = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const float4 u = *reinterpret_cast<const float4*>(ib + (ob + (uint32_t)dy * rowb + (uint32_t)dx * pixb));
          v.x = fmaxf(v.x, u.x);
          v.y = fmaxf(v.y, u.y);
          v.z = fmaxf(v.z, u.z);
          v.w = fmaxf(v.w, u.w);
        }
      *reinterpret_cast<float4*>(&ring[i & 1][tt][px * TP + 4 * cq]) = v;
    }
  };
  if (nsteps == 0) return;  // block-uniform: no barrier is skipped by part of the block
  if (wave < 2) {
    produce(0);
    __syncthreads();
    for (uint32_t i = 0; i < nsteps; ++i) {
      if (i + 1 < nsteps) produce(i + 1);
      __syncthreads();
    }
    return;
  }
  // consumers: the filter (B operand) and bias in registers
  const int c = wave - 2;
  float bw[KS][TN];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 8 * (s >> 2) + (s & 3) + 4 * h;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = 32 * j + col;
      bw[s][j] = n < p.OC ? p.w[k * p.OC + n] : 0.f;
    }
  }
  float bv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = 32 * j + col;
    bv[j] = (p.bias && n < p.OC) ? p.bias[n] : 0.f;
  }
  __syncthreads();  // the producers' step-0 set
  auto run = [&](auto act_c) __attribute__((always_inline)) {
    constexpr int ACT = decltype(act_c)::value;
    for (uint32_t i = 0; i < nsteps; ++i) {
      const uint32_t g0 = 2 * (i * B + b0) + (uint32_t)c;
      if (g0 < groups) {
        const float* tile = ring[i & 1][c];
        float a[KS];
#pragma unroll
        for (int j = 0; j < KS / 4; ++j) {
          const float4 v = *reinterpret_cast<const float4*>(&tile[col * TP + 8 * j + 4 * h]);
          a[4 * j] = v.x;
          a[4 * j + 1] = v.y;
          a[4 * j + 2] = v.z;
          a[4 * j + 3] = v.w;
        }
        f32x16 acc[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], bw[s][j], acc[j], 0, 0, 0);
        const uint32_t m0 = g0 * 32 + 4 * h;
        const bool full = (g0 + 1) * 32 <= p.M;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const uint32_t nn = 32 * j + col;
          if (nn >= (uint32_t)p.OC) continue;
          const uint32_t base = m0 * p.ldc + nn;
          float v[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            v[r] = acc[j][r] + bv[j];
            if (ACT == ACT_RELU) v[r] = v[r] > 0.f ? v[r] : 0.f;
            if (ACT == ACT_RELU6) v[r] = v[r] > 0.f ? (v[r] < 6.f ? v[r] : 6.f) : 0.f;
          }
          if (full) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
              *reinterpret_cast<float*>(yb + (base + (uint32_t)((r & 3) + 8 * (r >> 2)) * p.ldc) * 4u) = v[r];
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const uint32_t ro = (uint32_t)((r & 3) + 8 * (r >> 2));
              if (m0 + ro < p.M) *reinterpret_cast<float*>(yb + (base + ro * p.ldc) * 4u) = v[r];
            }
          }
        }
      }
      __syncthreads();  // set i & 1 is read: the producers refill it next step
    }
  };
  if (p.act == ACT_RELU) run(std::integral_constant<int, ACT_RELU>{});
  else if (p.act == ACT_RELU6) run(std::integral_constant<int, ACT_RELU6>{});
  else run(std::integral_constant<int, ACT_NONE>{});
}

template <int KS>
void launch_pool_conv(const PoolConv& p, int tn, hipStream_t s) {
  const uint32_t groups = (p.M + 31) / 32;
  static const bool ws = [] {
    const char* e = std::getenv("TFA_POOLCONV_WS");
    return !(e && e[0] == '0');
  }();
  if (ws) {  // two 32-pixel groups per block step
    const unsigned blocks = std::min<uint32_t>((groups + 1) / 2, 256 * 3);
    if (tn == 1) hipLaunchKernelGGL((pool_conv1x1_ws_kernel<KS, 1>), dim3(blocks), dim3(256), 0, s, p);
    else if (tn == 2) hipLaunchKernelGGL((pool_conv1x1_ws_kernel<KS, 2>), dim3(blocks), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((pool_conv1x1_ws_kernel<KS, 3>), dim3(blocks), dim3(256), 0, s, p);
    return;
  }
  const unsigned blocks = std::min<uint32_t>((groups + 3) / 4, 256 * 8);
  if (tn == 1) hipLaunchKernelGGL((pool_conv1x1_kernel<KS, 1>), dim3(blocks), dim3(256), 0, s, p);
  else if (tn == 2) hipLaunchKernelGGL((pool_conv1x1_kernel<KS, 2>), dim3(blocks), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((pool_conv1x1_kernel<KS, 3>), dim3(blocks), dim3(256), 0, s, p);
}

}  // namespace

bool pool_conv1x1_eligible(int64_t N, int64_t H, int64_t W, int64_t C, int64_t PH, int64_t PW, int64_t OC,
                           int64_t ldc, int act) {
  return (C == 16 || C == 32 || C == 64) && OC >= 1 && OC <= 96 && ldc >= OC &&
         (act == ACT_NONE || act == ACT_RELU || act == ACT_RELU6) && H * W * C * 4 < (int64_t(1) << 32) &&
         N * PH * PW * ldc * 4 < (int64_t(1) << 32) && N * PH * PW > 0;
}

void pool_conv1x1(const PoolConvArgs& a, hipStream_t s) {
  TFA_CHECK(pool_conv1x1_eligible(a.N, a.H, a.W, a.C, a.PH, a.PW, a.OC, a.ldc, a.act), "pool_conv1x1: not eligible");
  TFA_CHECK(a.pkh == 3 && a.pkw == 3 && a.psh >= 1 && a.psw >= 1 && (a.PH - 1) * a.psh + a.pkh <= a.H &&
                (a.PW - 1) * a.psw + a.pkw <= a.W,
            "pool_conv1x1: VALID pool geometry");
  TFA_CHECK((reinterpret_cast<uintptr_t>(a.x) & 15) == 0, "pool_conv1x1: input must be 16-byte aligned");
  PoolConv p;
  p.M = (uint32_t)(a.N * a.PH * a.PW);
  p.H = (int)a.H; p.W = (int)a.W; p.C = (int)a.C; p.PH = (int)a.PH; p.PW = (int)a.PW;
  p.pkh = (int)a.pkh; p.pkw = (int)a.pkw; p.psh = (int)a.psh; p.psw = (int)a.psw;
  p.OC = (int)a.OC;
  p.ldc = (uint32_t)a.ldc;
  p.x = static_cast<const float*>(a.x);
  p.w = static_cast<const float*>(a.w);
  p.bias = static_cast<const float*>(a.bias);
  p.y = static_cast<float*>(a.y);
  p.act = a.act;
  p.fPW = make_fastdiv((uint32_t)a.PW);
  p.fPH = make_fastdiv((uint32_t)a.PH);
  const int tn = (int)((a.OC + 31) / 32);
  if (a.C == 16) launch_pool_conv<8>(p, tn, s);
  else if (a.C == 32) launch_pool_conv<16>(p, tn, s);
  else launch_pool_conv<32>(p, tn, s);
  TFA_LAUNCH_CHECK("maxpool -> conv 1x1");
}

void set_conv_smallc(int on) { smallc_state().store(on ? 1 : 0); }

bool conv_smallc_eligible(const ConvArgs& a) {
  const int64_t K = a.KH * a.KW * a.C;
  return smallc_enabled() && K <= 32 && a.OC <= 64 && a.seg.n == 0 && a.epi.n == 0 &&
         (a.act == ACT_NONE || a.act == ACT_RELU || a.act == ACT_RELU6) && a.H * a.W * a.C < (int64_t(1) << 30) &&
         a.N * a.OH * a.OW < (int64_t(1) << 32);
}

void conv_smallc_launch(const ConvArgs& a, hipStream_t s) {
  SmallConv p;
  p.M = a.N * a.OH * a.OW;
  p.H = (int)a.H; p.W = (int)a.W; p.C = (int)a.C; p.KW = (int)a.KW;
  p.OH = (int)a.OH; p.OW = (int)a.OW;
  p.sh = (int)a.sh; p.sw = (int)a.sw; p.dh = (int)a.dh; p.dw = (int)a.dw;
  p.pt = (int)a.pad_t; p.pl = (int)a.pad_l;
  p.K = (int)(a.KH * a.KW * a.C);
  p.OC = (int)a.OC;
  p.ldc = a.ldc > 0 ? a.ldc : a.OC;
  p.x = static_cast<const float*>(a.x);
  p.w = static_cast<const float*>(a.w);
  p.bias = static_cast<const float*>(a.bias);
  p.y = static_cast<float*>(a.y);
  p.act = a.act;
  p.fOW = make_fastdiv((uint32_t)a.OW);
  p.fOH = make_fastdiv((uint32_t)a.OH);
  const int tn = a.OC <= 32 ? 1 : 2;
  const int ks = 4 * ((p.K + 7) / 8);  // whole k octets
  static const bool generic = [] {
    const char* e = std::getenv("TFA_SMALLC_GENERIC");
    return e && e[0] == '1';
  }();
  // 32-bit byte offsets (signed: the padded variant's window origins may
  // be negative); 1 = all taps in bounds (VALID-style), 2 = padding checked
  const int64_t xbytes = a.N * a.H * a.W * a.C * 4;
  const bool ysmall = p.ldc * 4 * 32 < (int64_t(1) << 32);  // per-group row offsets (64-bit group base)
  const bool inside = a.pad_t == 0 && a.pad_l == 0 && (a.OH - 1) * a.sh + (a.KH - 1) * a.dh <= a.H - 1 &&
                      (a.OW - 1) * a.sw + (a.KW - 1) * a.dw <= a.W - 1;
  const int fast = (generic || !ysmall) ? 0
                   : inside                          ? (xbytes < (int64_t(1) << 32) ? 1 : 0)
                                                     : (xbytes < (int64_t(1) << 31) ? 2 : 0);
  if (ks <= 4) launch_ks<4>(p, tn, fast, s);
  else if (ks <= 8) launch_ks<8>(p, tn, fast, s);
  else if (ks <= 12) launch_ks<12>(p, tn, fast, s);
  else launch_ks<16>(p, tn, fast, s);
  TFA_LAUNCH_CHECK("conv2d small-C");
}

}  // namespace k
}  // namespace tfa

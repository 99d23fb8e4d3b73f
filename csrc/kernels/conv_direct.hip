// Direct f32 Conv2D for narrow stem convs: C in {32, 64} input channels,
// OC <= 96 output channels, any KHxKW (>= 2 taps) / stride / dilation on wide
// images (the Inception-v3 stem: Conv2d_2a 3x3x32 -> 32 and Conv2d_2b
// 3x3x32 -> 64 on 111x111 / 109x109 images), on v_mfma_f32_32x32x2f32.
//
// The implicit-GEMM core (gemm.hip) streams A through LDS k tile by k tile
// (16 k = half a 32-channel filter tap per tile, one barrier each) and holds
// these layers at 88-109 TF. Here:
//  * the whole filter [K][OC] sits in LDS for the block's life (persistent
//    blocks walk 32-pixel groups), so B is one conflict-free ds_read_b32 per
//    MFMA and never leaves LDS;
//  * A comes straight from global memory into registers, 16 bytes per lane:
//    for a filter tap, lane (pixel m, half h) loads channels 8g + 4h .. +3 of
//    its pixel's tap (float4), which feed four k-steps; the k order inside each
//    group of 8 channels is permuted (lane half h supplies k = 8g + 4h + q at
//    step q), and B is read in the same order, so the product is exact f32
//    with a different (fixed) summation order than the GEMM core;
//  * the next tap's A loads are issued before the current tap's MFMAs;
//  * the epilogue stages each 32x32 tile in a wave-private LDS tile and stores
//    float4 rows with bias + ReLU/ReLU6.
// The choice of this kernel depends only on the shape (never on a timing), so
// a given conv always produces the same bits (tests/test_gpu_conv_direct.py).
#include <atomic>
#include <cstdlib>

#include "gemm_internal.h"
#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct DirectConv {
  int64_t M;  // N * OH * OW output pixels
  int H, W, C, KH, KW, OH, OW, sh, sw, dh, dw, pt, pl, OC;
  int64_t ldc;
  const float* x;
  const float* w;  // [KH*KW*C][OC]
  const float* bias;
  float* y;
  int act;
  FastDivU32 fOW, fOH, fKW;
};

constexpr int kWaves = 8;
constexpr int kStageF = 32 * 36;  // one wave's epilogue staging tile (floats)

// C8 = C / 8 channel groups per tap, TN = 32-column output tiles (OC <= 32 * TN)
template <int C8, int TN>
__global__ __launch_bounds__(64 * kWaves, 1) void conv_direct_kernel(DirectConv p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int C = 8 * C8, OCP = 32 * TN;
  const int taps = p.KH * p.KW;
  const int K = taps * C;
  float* Bs = lds;                              // [K][OCP]
  float* stage = lds + (size_t)K * OCP;         // kWaves x [32][36]
  // filter -> LDS (zero columns past OC)
  for (int i = threadIdx.x; i < K * OCP; i += blockDim.x) {
    const int kk = i / OCP, n = i % OCP;
    Bs[i] = n < p.OC ? p.w[(int64_t)kk * p.OC + n] : 0.f;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, col = lane & 31;
  __syncthreads();

  const int64_t groups = (p.M + 31) / 32;
  const int64_t nwaves = (int64_t)gridDim.x * kWaves;
  float* st = stage + wave * kStageF;
  for (int64_t gi = (int64_t)blockIdx.x * kWaves + wave; gi < groups; gi += nwaves) {
    // this lane's A row: output pixel m (both halves share the pixel)
    const int64_t m = gi * 32 + col;
    const bool live = m < p.M;
    const uint32_t mm = live ? (uint32_t)m : 0u;
    const uint32_t t = fdiv(mm, p.fOW);
    const int ow = (int)(mm - t * (uint32_t)p.OW);
    const uint32_t nimg = fdiv(t, p.fOH);
    const int oh = (int)(t - nimg * (uint32_t)p.OH);
    const int ih0 = oh * p.sh - p.pt, iw0 = ow * p.sw - p.pl;
    const float* img = p.x + (int64_t)nimg * p.H * p.W * C + 4 * h;

    auto load_tap = [&](int tap, float4 (&a)[C8]) {
      const uint32_t kh = fdiv((uint32_t)tap, p.fKW);
      const int kw = tap - (int)kh * p.KW;
      const int ih = ih0 + (int)kh * p.dh, iw = iw0 + kw * p.dw;
      const bool inb = live && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const float* src = inb ? img + ((int64_t)ih * p.W + iw) * C : p.x;  // padding taps read a safe address
#pragma unroll
      for (int g = 0; g < C8; ++g) {
        const float4 v = *reinterpret_cast<const float4*>(src + 8 * g);
        a[g] = inb ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };

    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    float4 a0[C8], a1[C8];
    load_tap(0, a0);
    for (int tap = 0; tap < taps; tap += 2) {
      // two taps per trip: the next tap's loads are in flight during this one's MFMAs
      if (tap + 1 < taps) load_tap(tap + 1, a1);
      {
        const float* brow = Bs + (size_t)(tap * C + 4 * h) * OCP + col;
#pragma unroll
        for (int g = 0; g < C8; ++g) {
          const float av[4] = {a0[g].x, a0[g].y, a0[g].z, a0[g].w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], brow[(8 * g + q) * OCP + 32 * j], acc[j], 0, 0, 0);
        }
      }
      if (tap + 1 >= taps) break;
      if (tap + 2 < taps) load_tap(tap + 2, a0);
      {
        const float* brow = Bs + (size_t)((tap + 1) * C + 4 * h) * OCP + col;
#pragma unroll
        for (int g = 0; g < C8; ++g) {
          const float av[4] = {a1[g].x, a1[g].y, a1[g].z, a1[g].w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], brow[(8 * g + q) * OCP + 32 * j], acc[j], 0, 0, 0);
        }
      }
    }
    // epilogue: 32x32 tile -> wave-private LDS tile -> float4 rows
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[((r & 3) + 8 * (r >> 2) + 4 * h) * 36 + col] = acc[j][r];
      const int c4 = 32 * j + 4 * (lane & 7);
      if (c4 < p.OC) {
        const float* bp = p.bias ? p.bias + c4 : nullptr;
        const float4 bb = bp ? make_float4(bp[0], bp[1], bp[2], bp[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = 8 * q + (lane >> 3);
          const int64_t row = gi * 32 + rr;
          float4 o = *reinterpret_cast<const float4*>(&st[rr * 36 + 4 * (lane & 7)]);
          o.x = act_fast(o.x + bb.x, p.act);
          o.y = act_fast(o.y + bb.y, p.act);
          o.z = act_fast(o.z + bb.z, p.act);
          o.w = act_fast(o.w + bb.w, p.act);
          if (row < p.M) *reinterpret_cast<float4*>(p.y + row * p.ldc + c4) = o;
        }
      }
    }
  }
}

std::atomic<int>& direct_state() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_CONV_DIRECT");
    return (e && std::atoi(e) == 0) ? 0 : 1;
  }());
  return v;
}

size_t direct_lds_bytes(int64_t K, int tn) { return ((size_t)K * 32 * tn + kWaves * kStageF) * sizeof(float); }

}  // namespace

void set_conv_direct(int on) { direct_state().store(on ? 1 : 0); }

bool conv_direct_eligible(const ConvArgs& a) {
  if (!direct_state().load()) return false;
  if (!(a.C == 32 || a.C == 64) || a.OC > 96 || a.OC % 4 != 0 || a.seg.n != 0 || a.epi.n != 0) return false;
  if (!(a.act == ACT_NONE || a.act == ACT_RELU || a.act == ACT_RELU6)) return false;
  const int64_t ldc = a.ldc > 0 ? a.ldc : a.OC;
  if (ldc % 4 != 0 || (reinterpret_cast<uintptr_t>(a.y) & 15) || (reinterpret_cast<uintptr_t>(a.x) & 15)) return false;
  if (a.N * a.OH * a.OW >= (int64_t(1) << 32) || a.H * a.W * a.C >= (int64_t(1) << 31)) return false;
  // wide images only: the direct kernel pays off where the GEMM core streams
  // many k tiles per 64-byte A segment (the 3x3 stem layers); a 1x1 stem
  // (Conv2d_3b 64 -> 80) is HBM-bound and runs the same on either kernel
  // (profiles/r3_conv_direct/), so pointwise convs stay on the GEMM core
  if (a.KH * a.KW < 2 || a.OH * a.OW < 4096) return false;
  const int tn = (int)((a.OC + 31) / 32);
  return direct_lds_bytes(a.KH * a.KW * a.C, tn) <= 120 * 1024;
}

void conv_direct_launch(const ConvArgs& a, hipStream_t s) {
  DirectConv p;
  p.M = a.N * a.OH * a.OW;
  p.H = (int)a.H; p.W = (int)a.W; p.C = (int)a.C; p.KH = (int)a.KH; p.KW = (int)a.KW;
  p.OH = (int)a.OH; p.OW = (int)a.OW;
  p.sh = (int)a.sh; p.sw = (int)a.sw; p.dh = (int)a.dh; p.dw = (int)a.dw;
  p.pt = (int)a.pad_t; p.pl = (int)a.pad_l;
  p.OC = (int)a.OC;
  p.ldc = a.ldc > 0 ? a.ldc : a.OC;
  p.x = static_cast<const float*>(a.x);
  p.w = static_cast<const float*>(a.w);
  p.bias = static_cast<const float*>(a.bias);
  p.y = static_cast<float*>(a.y);
  p.act = a.act;
  p.fOW = make_fastdiv((uint32_t)a.OW);
  p.fOH = make_fastdiv((uint32_t)a.OH);
  p.fKW = make_fastdiv((uint32_t)a.KW);
  const int tn = (int)((a.OC + 31) / 32);
  const size_t lds = direct_lds_bytes(a.KH * a.KW * a.C, tn);
  const int64_t groups = (p.M + 31) / 32;
  const int per_cu = lds <= 80 * 1024 ? 2 : 1;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((groups + kWaves - 1) / kWaves, 256 * per_cu));
#define TFA_DIRECT(C8_, TN_)                                                                                    \
  do {                                                                                                           \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_direct_kernel<C8_, TN_>),                     \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                            \
    hipLaunchKernelGGL((conv_direct_kernel<C8_, TN_>), dim3((unsigned)blocks), dim3(64 * kWaves), lds, s, p); \
  } while (0)
  if (a.C == 32) {
    if (tn == 1) TFA_DIRECT(4, 1);
    else if (tn == 2) TFA_DIRECT(4, 2);
    else TFA_DIRECT(4, 3);
  } else {
    if (tn == 1) TFA_DIRECT(8, 1);
    else if (tn == 2) TFA_DIRECT(8, 2);
    else TFA_DIRECT(8, 3);
  }
#undef TFA_DIRECT
  TFA_LAUNCH_CHECK("conv2d direct");
}

}  // namespace k
}  // namespace tfa

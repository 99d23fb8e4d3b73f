// f32 MFMA issue-rate probe (v_mfma_f32_32x32x2_f32) on gfx950: how close a
// 4-accumulator wave gets to 64 FLOP/clk/SIMD with and without the LDS
// operand reads a GEMM inner loop needs.
//   hipcc -O3 --offload-arch=gfx950 scripts/mfma_probe.hip -o build/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// MODE 0: registers only; 1: 4 ds_read_b32 per k-step (A/B fragments, one step ahead);
// 2: ds_read_b128 per 4 k-steps per operand; 3: mode 1 + a barrier every 8 k-steps
template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, int iters) {
  __shared__ float lds[2][16][132];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 2 * 16 * 132; i += 256) (&lds[0][0][0])[i] = (float)(i & 7) * 0.001f;
  __syncthreads();
  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  float a0 = lane * 1e-3f, a1 = 0.5f, b0 = 0.25f, b1 = wave * 1e-3f;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[3], 0, 0, 0);
      }
    } else if (MODE == 1 || MODE == 3) {
      const int buf = it & 1;
      float a[2][2], b[2][2];
      auto rd = [&](int x, int kk) {
        const int kr = kk + (lane >> 5);
        a[x][0] = lds[buf][kr][(wave & 1) * 64 + (lane & 31)];
        a[x][1] = lds[buf][kr][(wave & 1) * 64 + 32 + (lane & 31)];
        b[x][0] = lds[buf][kr][(wave >> 1) * 64 + (lane & 31)];
        b[x][1] = lds[buf][kr][(wave >> 1) * 64 + 32 + (lane & 31)];
      };
      rd(0, 0);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        if (s + 1 < 8) rd((s + 1) & 1, 2 * (s + 1));
        __builtin_amdgcn_sched_barrier(0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s & 1][0], b[s & 1][0], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s & 1][0], b[s & 1][1], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s & 1][1], b[s & 1][0], acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s & 1][1], b[s & 1][1], acc[3], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (MODE == 3) __syncthreads();
    } else {
      const int buf = it & 1;
      const float* base = &lds[buf][0][0];
      float4 a4[2][2], b4[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        a4[0][h] = *reinterpret_cast<const float4*>(base + ((lane & 31) * 16 + 8 * (lane >> 5) + 4 * h) % 2000);
        a4[1][h] = *reinterpret_cast<const float4*>(base + ((lane & 31) * 16 + 512 + 8 * (lane >> 5) + 4 * h) % 2000);
        b4[0][h] = *reinterpret_cast<const float4*>(base + ((lane & 31) * 16 + 1024 + 8 * (lane >> 5) + 4 * h) % 2000);
        b4[1][h] = *reinterpret_cast<const float4*>(base + ((lane & 31) * 16 + 1536 + 8 * (lane >> 5) + 4 * h) % 2000);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int h = s >> 2, c = s & 3;
        auto pick = [&](const float4& v) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; };
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(pick(a4[0][h]), pick(b4[0][h]), acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(pick(a4[0][h]), pick(b4[1][h]), acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(pick(a4[1][h]), pick(b4[0][h]), acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(pick(a4[1][h]), pick(b4[1][h]), acc[3], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
int run(const char* name, int blocks_per_cu, float* out) {
  const int iters = 4096, blocks = 256 * blocks_per_cu;
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, out, 16);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double flop = (double)blocks * 4 /*waves*/ * iters * 32 /*mfma*/ * (32.0 * 32 * 2 * 2);
  std::printf("{\"probe\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n", name, blocks_per_cu, ms,
              flop / ms / 1e9);
  return 0;
}

int main() {
  float* out;
  CK(hipMalloc(&out, 256 * 16 * 256 * 4));
  for (int bpc : {1, 2, 4}) {
    run<0>("regs", bpc, out);
    run<1>("ds_read_b32 x4/step", bpc, out);
    run<2>("ds_read_b128", bpc, out);
    run<3>("b32 + barrier/8 steps", bpc, out);
  }
  return 0;
}

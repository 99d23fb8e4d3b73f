// Lab for a one-wave-per-SIMD f32 MFMA GEMM main loop (gfx950): the
// structure the round-4 verdict names as the remaining lever of the f32 core.
//
//   * 4 waves per 256 x BN block (2 x 2), each wave a 128 x BN/2 tile of
//     32x32 accumulators (4 x TN x 16 floats: 128-256 registers, which the
//     compiler puts in AGPRs at one wave per SIMD);
//   * operands staged global -> LDS with global_load_lds_dwordx4 (no VGPR
//     staging, no ds_write): both operands k-contiguous in global memory
//     (A [M][K], B^T [N][K]), LDS images [k/4][row][4] filled lane-linearly
//     (one 1 KB wave instruction = 64 rows x 16 B at one k quad);
//   * k-permuted fragments: a lane reads 4 consecutive k of its row with ONE
//     ds_read_b128 and feeds them to 4 successive MFMA k-steps (half 0 of the
//     wave holds k quad 2j, half 1 quad 2j+1: the same permutation on A and B,
//     so the sum is unchanged);
//   * a ring of STAGES LDS stages (BK = 16 each) with STAGES-1 in flight: a
//     counted vmcnt (never 0 in the loop) + a raw s_barrier per stage.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/g2_lab.hip -o build/g2_lab
// Run:   ./build/g2_lab [M N K]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                        \
    }                                                                                      \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// global -> LDS, 16 bytes per lane: lane i lands at lds + 16 * i
__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// vmcnt(N) alone (expcnt / lgkmcnt left at their maxima): gfx9 encoding
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int BN, int STAGES, int MODE, int NW = 4>
__global__ __launch_bounds__(64 * NW, 1) void g2_kernel(const float* __restrict__ A, const float* __restrict__ Bt,
                                                    float* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                    int ldc, int tiles_n) {
  constexpr int BM = 256, BK = 16, WN = 2, WM = NW / WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int KQ = BK / 4;                     // k quads per stage
  constexpr int A_BYTES = BM * BK * 4, B_BYTES = BN * BK * 4;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int AI = KQ * (BM / 64) / NW;        // A glds per wave per stage
  constexpr int BI = KQ * (BN / 64) / NW;        // B glds per wave per stage
  constexpr int G = AI + BI;
  static_assert(TN >= 1 && (KQ * (BN / 64)) % NW == 0 && (KQ * (BM / 64)) % NW == 0, "glds pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = (int)gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int m0 = (wg / tiles_n) * BM, n0 = (wg % tiles_n) * BN;

  // this wave's glds pieces. MODE < 2: instruction q covers k quad q / (rows/64)
  // of 64 rows (one 16-B piece per row: 64 cache lines per instruction), LDS
  // image [kq][row][4]. MODE >= 2 (coalesced): instruction q covers rows
  // 16q..16q+15 whole (4 lanes per 64-B row segment), LDS image [row][4 slots]
  // with the k quad of slot c = c ^ ((row >> 2) & 3) (the swizzle rides on
  // the source address, so the lane-linear image stays conflict-free for the
  // fragment reads)
  constexpr bool COAL = MODE >= 2;
  const float* ap[AI];
  int aoff[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int q = wave * AI + i;
    if constexpr (COAL) {
      const int r = q * 16 + lane / 4, c = lane % 4;
      ap[i] = A + (size_t)(m0 + r) * lda + 4 * (c ^ ((r >> 2) & 3));
      aoff[i] = q * 1024;
    } else {
      const int kq = q / (BM / 64), mb = q % (BM / 64);
      ap[i] = A + (size_t)(m0 + mb * 64 + lane) * lda + 4 * kq;
      aoff[i] = (kq * BM + mb * 64) * 16;
    }
  }
  const float* bp[BI];
  int boff[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int q = wave * BI + i;
    if constexpr (COAL) {
      const int r = q * 16 + lane / 4, c = lane % 4;
      bp[i] = Bt + (size_t)(n0 + r) * ldb + 4 * (c ^ ((r >> 2) & 3));
      boff[i] = A_BYTES + q * 1024;
    } else {
      const int kq = q / (BN / 64), nb = q % (BN / 64);
      bp[i] = Bt + (size_t)(n0 + nb * 64 + lane) * ldb + 4 * kq;
      boff[i] = A_BYTES + (kq * BN + nb * 64) * 16;
    }
  }
  auto issue = [&](int slot, int kt) __attribute__((always_inline)) {
    char* base = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < AI; ++i) glds16(ap[i] + kt * BK, base + aoff[i]);
#pragma unroll
    for (int i = 0; i < BI; ++i) glds16(bp[i] + kt * BK, base + boff[i]);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){};

  const int KT = K / BK;
  const int h = lane >> 5, r32 = lane & 31;
  struct Frag {
    f32x4 a[TM], b[TN];
  };
  auto read = [&](int stage, int j, Frag& f) __attribute__((always_inline)) {
    const char* st = smem + (stage % STAGES) * STAGE;
    const int kq = 2 * j + h;
    if constexpr (COAL) {
      const int slot = kq ^ ((r32 >> 2) & 3);  // rows of one lane differ by multiples of 32: same swizzle
#pragma unroll
      for (int i = 0; i < TM; ++i) f.a[i] = *reinterpret_cast<const f32x4*>(st + (wm * (BM / WM) + i * 32 + r32) * 64 + slot * 16);
#pragma unroll
      for (int jn = 0; jn < TN; ++jn)
        f.b[jn] = *reinterpret_cast<const f32x4*>(st + A_BYTES + (wn * (BN / 2) + jn * 32 + r32) * 64 + slot * 16);
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) f.a[i] = *reinterpret_cast<const f32x4*>(st + (kq * BM + wm * (BM / WM) + i * 32 + r32) * 16);
#pragma unroll
      for (int jn = 0; jn < TN; ++jn)
        f.b[jn] = *reinterpret_cast<const f32x4*>(st + A_BYTES + (kq * BN + wn * (BN / 2) + jn * 32 + r32) * 16);
    }
  };
  auto mma = [&](const Frag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jn = 0; jn < TN; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[i][s], f.b[jn][s], acc[i][jn], 0, 0, 0);
  };
  if constexpr (MODE == 0) {
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < KT) issue(s, s);
    for (int kt = 0; kt < KT; ++kt) {
      // stage kt landed (for this wave); the later STAGES-2 stages may stay in flight
      if (kt + STAGES - 2 < KT) wait_vm<G * (STAGES - 2)>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();  // every wave's stage kt is in; every wave is done with stage kt-1
      if (kt + STAGES - 1 < KT) issue((kt + STAGES - 1) % STAGES, kt + STAGES - 1);
#pragma unroll
      for (int j = 0; j < KQ / 2; ++j) {
        Frag f;
        read(kt, j, f);
        mma(f);
      }
    }
  } else {  // MODE 1, 2
    // fragments software-pipelined: the next k quad pair (or the next stage's
    // first one) is read while the current one's MFMAs run. Stage kt+1 is
    // retired one stage early (wait + barrier at the top of iteration kt), so
    // its first fragments can be read before the next barrier.
    static_assert(STAGES >= 3, "needs one stage of slack");
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < KT) issue(s, s);
    if (KT > STAGES - 2) wait_vm<G * (STAGES - 2)>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    Frag cur, nxt;
    if (KT > 0) read(0, 0, cur);
    // one stage: [wait + barrier] [glds of stage kt+S-1] [KQ/2 fragment
    // pairs of MFMAs, the next pair's reads in their shadow]. MODE 3 spreads
    // the glds between the first MFMAs (each glds costs ~60 issue cycles
    // when issued back to back) instead of issuing them as one block.
    auto stage = [&](int kt, auto do_issue) __attribute__((always_inline)) {
      constexpr bool ISSUE = decltype(do_issue)::value;
      if (kt + STAGES - 2 < KT) wait_vm<G * (STAGES - 3)>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int j = 0; j < KQ / 2; ++j) {
        if (j + 1 < KQ / 2) read(kt, j + 1, nxt);
        else if (kt + 1 < KT) read(kt + 1, 0, nxt);
        if (ISSUE && j == 0) issue((kt + STAGES - 1) % STAGES, kt + STAGES - 1);
        mma(cur);
        if constexpr (MODE >= 3) {
          if (ISSUE && j == 0) {
            constexpr int NM = 4 * TM * TN, R = TM + TN;
            static_assert(NM >= G + R, "MFMAs to hide the loads behind");
#pragma unroll
            for (int q = 0; q < G; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (glds)
            }
#pragma unroll
            for (int q = 0; q < R; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NM - G - R, 0);
          } else {
            constexpr int NM = 4 * TM * TN, R = TM + TN;
#pragma unroll
            for (int q = 0; q < R; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NM - R, 0);
          }
        }
        cur = nxt;
      }
    };
    int kt = 0;
    for (; kt + STAGES - 1 < KT; ++kt) stage(kt, std::true_type{});
    for (; kt < KT; ++kt) stage(kt, std::false_type{});
  }
  // epilogue: C/D layout row = (r&3) + 8*(r>>2) + 4*(lane>>5), col = lane&31
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jn = 0; jn < TN; ++jn) {
      const int col = n0 + wn * (BN / 2) + jn * 32 + r32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        C[(size_t)row * ldc + col] = acc[i][jn][r];
      }
    }
}

#define G2_INST(BN_, S_, MODE_)  G2_INSTW(BN_, S_, MODE_, 4)
#define G2_INSTW(BN_, S_, MODE_, NW_)                                                                           \
  template __global__ void g2_kernel<BN_, S_, MODE_, NW_>(const float* __restrict__, const float* __restrict__,      \
                                                     float* __restrict__, int, int, int, int, int, int, int);
G2_INST(256, 3, 0)
G2_INST(256, 4, 0)
G2_INST(256, 4, 1)
G2_INST(128, 4, 1)
G2_INST(128, 5, 1)
G2_INST(192, 4, 1)
G2_INST(256, 4, 2)
G2_INST(128, 4, 2)
G2_INST(128, 5, 2)
G2_INST(192, 4, 2)
G2_INST(64, 5, 2)
G2_INSTW(256, 4, 2, 8)
G2_INST(256, 4, 3)
G2_INST(128, 4, 3)
G2_INST(192, 4, 3)
G2_INST(64, 5, 3)
G2_INSTW(256, 4, 3, 8)
G2_INSTW(128, 4, 2, 8)
G2_INSTW(128, 5, 2, 8)

// reference: one thread per output, f64 accumulation
__global__ void ref_kernel(const float* A, const float* Bt, double* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  double s = 0;
  for (int k = 0; k < K; ++k) s += (double)A[(size_t)m * K + k] * Bt[(size_t)n * K + k];
  C[(size_t)m * N + n] = s;
}

__global__ void fill(float* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = ((x & 0xFFFFFF) / 16777216.0f) * 2.f - 1.f;
  }
}

template <int BN, int STAGES, int MODE, int NW = 4>
double run(const float* A, const float* Bt, float* C, int M, int N, int K, int iters) {
  const int tn = N / BN, tm = M / 256;
#define LAUNCH_G2 hipLaunchKernelGGL((g2_kernel<BN, STAGES, MODE, NW>), dim3(tm * tn), dim3(64 * NW), 0, 0, A, Bt, C, M, N, K, K, K, N, tn)
  LAUNCH_G2;
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) LAUNCH_G2;
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

int main(int argc, char** argv) {
  int M = argc > 3 ? std::atoi(argv[1]) : 4096, N = argc > 3 ? std::atoi(argv[2]) : 4096,
      K = argc > 3 ? std::atoi(argv[3]) : 4096;
  if (M % 256 || N % 64 || K % 16) {
    std::fprintf(stderr, "M a multiple of 256, N of 64, K of 16 only\n");
    return 1;
  }
  float *A, *Bt, *C;
  double* R;
  CK(hipMalloc(&A, (size_t)M * K * 4));
  CK(hipMalloc(&Bt, (size_t)N * K * 4));
  CK(hipMalloc(&C, (size_t)M * N * 4));
  CK(hipMalloc(&R, (size_t)256 * N * 8));
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, A, (size_t)M * K, 1u);
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, Bt, (size_t)N * K, 7u);
  hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, 256), dim3(256), 0, 0, A, Bt, R, 256, N, K);  // first 256 rows
  CK(hipDeviceSynchronize());
  std::vector<double> ref((size_t)256 * N);
  CK(hipMemcpy(ref.data(), R, ref.size() * 8, hipMemcpyDeviceToHost));
  auto check = [&](const char* name, double ms) {
    std::vector<float> c((size_t)256 * N);
    CK(hipMemcpy(c.data(), C, c.size() * 4, hipMemcpyDeviceToHost));
    double err = 0;
    for (size_t i = 0; i < c.size(); ++i) err = std::fmax(err, std::fabs(c[i] - ref[i]));
    const double tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12;
    std::printf("{\"kernel\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"ms\": %.4f, \"tflops\": %.2f, \"max_abs_err\": %.3e}\n",
                name, M, N, K, ms, tf, err);
    std::fflush(stdout);
    CK(hipMemset(C, 0, (size_t)M * N * 4));
  };
  const int it = 20;
  if (argc > 4) {  // one variant only (counter runs)
    check("g2 256x256 s4 m3", run<256, 4, 3>(A, Bt, C, M, N, K, it));
    return 0;
  }
  if (N % 256 == 0) {
    check("g2 256x256 s4 m2", run<256, 4, 2>(A, Bt, C, M, N, K, it));
    check("g2 256x256 s4 m3", run<256, 4, 3>(A, Bt, C, M, N, K, it));
    check("g2 256x256 s4 m3 w8", run<256, 4, 3, 8>(A, Bt, C, M, N, K, it));
    check("g2 256x128 s4 m3", run<128, 4, 3>(A, Bt, C, M, N, K, it));
    check("g2 256x256 s4 m2 w8", run<256, 4, 2, 8>(A, Bt, C, M, N, K, it));
    check("g2 256x256 s4 m3 again", run<256, 4, 3>(A, Bt, C, M, N, K, it));
  }
  if (N % 192 == 0) {
    check("g2 256x192 s4 m2", run<192, 4, 2>(A, Bt, C, M, N, K, it));
    check("g2 256x192 s4 m3", run<192, 4, 3>(A, Bt, C, M, N, K, it));
  }
  if (N % 64 == 0 && N % 128 != 0) {
    check("g2 256x64 s5 m2", run<64, 5, 2>(A, Bt, C, M, N, K, it));
    check("g2 256x64 s5 m3", run<64, 5, 3>(A, Bt, C, M, N, K, it));
  }
  return 0;
}

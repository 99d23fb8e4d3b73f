// Tile-shape lab for the f32 MFMA GEMM core (csrc/kernels/gemm.hip): the
// same register-staged, two-LDS-stage main loop, parametrised by block tile,
// wave layout, k depth and occupancy, on row-major A[M,K] x B[K,N] (+bias,
// ReLU). Question it answers: does a wave tile of 128x128 (16 accumulating
// 32x32 MFMA tiles = 256 accumulator registers, one block per CU) beat the
// shipped 64x64 wave tile (two blocks per CU)? hipBLASLt reaches 147 TF at
// 4096^3 f32 on MI355X where the shipped core reaches ~110-126.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/bigtile_lab.hip -o build/bigtile_lab && ./build/bigtile_lab
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// M % BM == 0, N % BN == 0, K % BK == 0 (checked on the host)
template <int BM, int BN, int WM, int WN, int BK, int MINB>
__global__ __launch_bounds__(256, MINB) void tile_gemm(const float* __restrict__ A, const float* __restrict__ B,
                                                       const float* __restrict__ bias, float* __restrict__ C,
                                                       int M, int N, int K, int tiles_n) {
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(WM * WN == 4, "4 waves");
  constexpr int KQ = BK / 4;
  constexpr int AP = BM * BK / 4 / 256, BP = BN * BK / 4 / 256;
  static_assert(AP * 256 * 4 == BM * BK && BP * 256 * 4 == BN * BK, "whole float4 pieces per thread");
  __shared__ __attribute__((aligned(16))) float As[2][BK][LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][LDB];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
  float4 ra[AP], rb[BP];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p, row = idx / KQ, kq = idx % KQ;
      ra[p] = *reinterpret_cast<const float4*>(A + (m0 + row) * K + k0 + 4 * kq);
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p, kr = idx / (BN / 4), nq = idx % (BN / 4);
      rb[p] = *reinterpret_cast<const float4*>(B + (k0 + kr) * N + n0 + 4 * nq);
    }
  };
  auto store = [&](int st) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p, row = idx / KQ, kq = idx % KQ;
      As[st][4 * kq + 0][row] = ra[p].x;
      As[st][4 * kq + 1][row] = ra[p].y;
      As[st][4 * kq + 2][row] = ra[p].z;
      As[st][4 * kq + 3][row] = ra[p].w;
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p, kr = idx / (BN / 4), nq = idx % (BN / 4);
      *reinterpret_cast<float4*>(&Bs[st][kr][4 * nq]) = rb[p];
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int ktiles = K / BK;
  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < ktiles; ++kt) {
    const bool has_next = kt + 1 < ktiles;
    if (has_next) load((int64_t)(kt + 1) * BK);
    float a[2][TM], b[2][TN];
    auto rd = [&](int buf, int kk) {
      const int kr = kk + (lane >> 5);
#pragma unroll
      for (int i = 0; i < TM; ++i) a[buf][i] = As[cur][kr][wm * (BM / WM) + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[buf][j] = Bs[cur][kr][wn * (BN / WN) + j * 32 + (lane & 31)];
    };
    rd(0, 0);
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      if (kk + 1 < BK / 2) rd((kk + 1) & 1, 2 * (kk + 1));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk & 1][i], b[kk & 1][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (has_next) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
    const float bv = bias[col];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        C[row * N + col] = fmaxf(acc[i][j][r] + bv, 0.f);
      }
  }
}


// ---- interleaved variant: no sched_barrier(0) walls; per k-step the memory
// ops (next tile's global loads, next step's LDS reads, next stage's LDS
// writes) are spread between the MFMAs with sched_group_barrier, one
// scheduling region per k tile (the last tile is peeled so the loop body is
// branch-free).
constexpr int kMFMA = 0x008, kVMEM_R = 0x020, kDS_R = 0x100, kDS_W = 0x200;

// ops [J, END) of a step whose first O1 ops have mask M1 and the rest M2
template <int J, int END, int O1, int M1, int M2>
__device__ __forceinline__ void emit_ops() {
  if constexpr (J < END) {
    __builtin_amdgcn_sched_group_barrier(J < O1 ? M1 : M2, 1, 0);
    emit_ops<J + 1, END, O1, M1, M2>();
  }
}
// slot I of NM: the ops assigned to it, then one MFMA
template <int I, int NM, int O, int O1, int M1, int M2>
__device__ __forceinline__ void emit_slots() {
  if constexpr (I < NM) {
    constexpr int lo = (I * O + NM - 1) / NM, hi = ((I + 1) * O + NM - 1) / NM;
    emit_ops<lo, hi, O1, M1, M2>();
    __builtin_amdgcn_sched_group_barrier(kMFMA, 1, 0);
    emit_slots<I + 1, NM, O, O1, M1, M2>();
  }
}

template <int BM, int BN, int WM, int WN, int BK, int MINB, int VAR = 0>
__global__ __launch_bounds__(256, MINB) void tile_gemm_il(const float* __restrict__ A, const float* __restrict__ B,
                                                          const float* __restrict__ bias, float* __restrict__ C,
                                                          int M, int N, int K, int tiles_n) {
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(WM * WN == 4, "4 waves");
  constexpr int KQ = BK / 4;
  constexpr int AP = BM * BK / 4 / 256, BP = BN * BK / 4 / 256;
  constexpr int S = BK / 2, NM = TM * TN, R = TM + TN, L = AP + BP, W = 4 * AP + BP;
  static_assert(AP * 256 * 4 == BM * BK && BP * 256 * 4 == BN * BK, "whole float4 pieces per thread");
  __shared__ __attribute__((aligned(16))) float As[2][BK][LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][LDB];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
  float4 ra[AP], rb[BP];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p, row = idx / KQ, kq = idx % KQ;
      ra[p] = *reinterpret_cast<const float4*>(A + (m0 + row) * K + k0 + 4 * kq);
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p, kr = idx / (BN / 4), nq = idx % (BN / 4);
      rb[p] = *reinterpret_cast<const float4*>(B + (k0 + kr) * N + n0 + 4 * nq);
    }
  };
  auto store = [&](int st) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p, row = idx / KQ, kq = idx % KQ;
      As[st][4 * kq + 0][row] = ra[p].x;
      As[st][4 * kq + 1][row] = ra[p].y;
      As[st][4 * kq + 2][row] = ra[p].z;
      As[st][4 * kq + 3][row] = ra[p].w;
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p, kr = idx / (BN / 4), nq = idx % (BN / 4);
      *reinterpret_cast<float4*>(&Bs[st][kr][4 * nq]) = rb[p];
    }
  };
  auto storeA = [&](int st) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p, row = idx / KQ, kq = idx % KQ;
      As[st][4 * kq + 0][row] = ra[p].x;
      As[st][4 * kq + 1][row] = ra[p].y;
      As[st][4 * kq + 2][row] = ra[p].z;
      As[st][4 * kq + 3][row] = ra[p].w;
    }
  };
  auto storeB = [&](int st) {
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p, kr = idx / (BN / 4), nq = idx % (BN / 4);
      *reinterpret_cast<float4*>(&Bs[st][kr][4 * nq]) = rb[p];
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int ktiles = K / BK;
  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
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
    __builtin_amdgcn_sched_group_barrier(kDS_R, R, 0);
    if constexpr (NEXT) load(knext);
#pragma unroll
    for (int kk = 0; kk < S; ++kk) {
      if (kk + 1 < S) rd((kk + 1) & 1, 2 * (kk + 1));
      if constexpr (VAR == 1) {  // A image written one k-step earlier than B
        if (NEXT && kk == S - 2) storeA(cur ^ 1);
        if (NEXT && kk == S - 1) storeB(cur ^ 1);
      } else {
        if (NEXT && kk == S - 1) store(cur ^ 1);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk & 1][i], b[kk & 1][j], acc[i][j], 0, 0, 0);
      // this step's MFMAs with its memory ops spread between them
      if (VAR == 1 && NEXT && kk == S - 2) {
        emit_slots<0, NM, R + 4 * AP, R, kDS_R, kDS_W>();
      } else if (VAR == 1 && NEXT && kk == S - 1) {
        emit_slots<0, NM, BP, BP, kDS_W, kDS_W>();
      } else if (kk == 0 && NEXT) {
        emit_slots<0, NM, L + R, L, kVMEM_R, kDS_R>();
      } else if (kk == S - 1 && NEXT) {
        emit_slots<0, NM, W, W, kDS_W, kDS_W>();
      } else if (kk + 1 < S) {
        emit_slots<0, NM, R, R, kDS_R, kDS_R>();
      } else {
        __builtin_amdgcn_sched_group_barrier(kMFMA, NM, 0);
      }
    }
    __syncthreads();
    cur ^= 1;
  };
  for (int kt = 0; kt + 1 < ktiles; ++kt) tile((int64_t)(kt + 1) * BK, std::true_type{});
  tile(0, std::false_type{});
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
    const float bv = bias[col];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        C[row * N + col] = fmaxf(acc[i][j][r] + bv, 0.f);
      }
  }
}


// ---- k-permuted variant: A and B^T staged k-contiguous ([m][k], [n][k]
// rows of BK+4 floats, float4 LDS writes, no transposing scalar stores); a
// lane reads 4 consecutive k of its row with one ds_read_b128 and feeds them
// to 4 successive MFMAs, so MFMA step s of an 8-k group pairs k = 8g+s and
// 8g+4+s (lane half 0 / 1). Same interleaved schedule as tile_gemm_il.
// B is given transposed: Bt[N][K] (constant weights are transposed once).
template <int BM, int BN, int WM, int WN, int BK, int MINB>
__global__ __launch_bounds__(256, MINB) void tile_gemm_kp(const float* __restrict__ A, const float* __restrict__ Bt,
                                                          const float* __restrict__ bias, float* __restrict__ C,
                                                          int M, int N, int K, int tiles_n) {
  constexpr int LDK = BK + 4;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(WM * WN == 4 && BK % 8 == 0, "4 waves, 8-k groups");
  constexpr int KQ = BK / 4;
  constexpr int AP = BM * BK / 4 / 256, BP = BN * BK / 4 / 256;
  constexpr int G = BK / 8, NM = TM * TN, R = TM + TN, L = AP + BP, W = AP + BP;
  static_assert(AP * 256 * 4 == BM * BK && BP * 256 * 4 == BN * BK, "whole float4 pieces per thread");
  __shared__ __attribute__((aligned(16))) float As[2][BM][LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][LDK];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
  float4 ra[AP], rb[BP];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p, row = idx / KQ, kq = idx % KQ;
      ra[p] = *reinterpret_cast<const float4*>(A + (m0 + row) * K + k0 + 4 * kq);
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p, col = idx / KQ, kq = idx % KQ;
      rb[p] = *reinterpret_cast<const float4*>(Bt + (n0 + col) * K + k0 + 4 * kq);
    }
  };
  auto store = [&](int st) {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int idx = tid + 256 * p, row = idx / KQ, kq = idx % KQ;
      *reinterpret_cast<float4*>(&As[st][row][4 * kq]) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int idx = tid + 256 * p, col = idx / KQ, kq = idx % KQ;
      *reinterpret_cast<float4*>(&Bs[st][col][4 * kq]) = rb[p];
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int ktiles = K / BK;
  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  const int kh = 4 * (lane >> 5);
  auto tile = [&](int64_t knext, auto more) {
    constexpr bool NEXT = decltype(more)::value;
    float4 a[2][TM], b[2][TN];
    auto rd = [&](int buf, int g) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[buf][i] = *reinterpret_cast<const float4*>(&As[cur][wm * (BM / WM) + i * 32 + (lane & 31)][8 * g + kh]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[buf][j] = *reinterpret_cast<const float4*>(&Bs[cur][wn * (BN / WN) + j * 32 + (lane & 31)][8 * g + kh]);
    };
    rd(0, 0);
    __builtin_amdgcn_sched_group_barrier(kDS_R, R, 0);
    if constexpr (NEXT) load(knext);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (g + 1 < G) rd((g + 1) & 1, g + 1);
      if (NEXT && g == G - 1) store(cur ^ 1);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g & 1][i][s], b[g & 1][j][s], acc[i][j], 0, 0, 0);
      if (g == 0 && NEXT && G > 1) {
        emit_slots<0, 4 * NM, L + R, L, kVMEM_R, kDS_R>();
      } else if (g == 0 && NEXT) {  // one group: loads, then writes
        emit_slots<0, 4 * NM, L + W, L, kVMEM_R, kDS_W>();
      } else if (g == G - 1 && NEXT) {
        emit_slots<0, 4 * NM, W, W, kDS_W, kDS_W>();
      } else if (g + 1 < G) {
        emit_slots<0, 4 * NM, R, R, kDS_R, kDS_R>();
      } else {
        __builtin_amdgcn_sched_group_barrier(kMFMA, 4 * NM, 0);
      }
    }
    __syncthreads();
    cur ^= 1;
  };
  for (int kt = 0; kt + 1 < ktiles; ++kt) tile((int64_t)(kt + 1) * BK, std::true_type{});
  tile(0, std::false_type{});
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
    const float bv = bias[col];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        C[row * N + col] = fmaxf(acc[i][j][r] + bv, 0.f);
      }
  }
}

__global__ void transpose(const float* in, float* out, int R, int Cc) {  // in [R][C] -> out [C][R]
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)R * Cc;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / Cc, c = i % Cc;
    out[c * R + r] = in[i];
  }
}

// f64-accumulated reference for sampled rows
__global__ void ref_rows(const float* A, const float* B, const float* bias, const int* rows, int nrows, int N, int K,
                         double* out) {
  const int r = blockIdx.x, n = threadIdx.x + blockIdx.y * blockDim.x;
  if (r >= nrows || n >= N) return;
  const int64_t m = rows[r];
  double s = 0;
  for (int k = 0; k < K; ++k) s += (double)A[m * K + k] * (double)B[(int64_t)k * N + n];
  s += bias[n];
  out[(int64_t)r * N + n] = s > 0 ? s : 0;
}

__global__ void fill(float* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = ((x & 0xffffff) / 16777216.0f - 0.5f) * scale;
  }
}

struct Shape {
  int M, N, K;
};

template <int BM, int BN, int WM, int WN, int BK, int MINB, int IL = 0>
void run(const char* name, const Shape& s, const float* A, const float* B, const float* bias, float* C, int iters,
         const float* Bt = nullptr) {
  if (s.M % BM || s.N % BN || s.K % BK) return;
  const int tn = s.N / BN, nwg = (s.M / BM) * tn;
  auto launch = [&] {
    if constexpr (IL == 2)
      hipLaunchKernelGGL((tile_gemm_kp<BM, BN, WM, WN, BK, MINB>), dim3(nwg), dim3(256), 0, 0, A, Bt, bias, C, s.M,
                         s.N, s.K, tn);
    else if constexpr (IL == 3)
      hipLaunchKernelGGL((tile_gemm_il<BM, BN, WM, WN, BK, MINB, 1>), dim3(nwg), dim3(256), 0, 0, A, B, bias, C, s.M,
                         s.N, s.K, tn);
    else if constexpr (IL == 1)
      hipLaunchKernelGGL((tile_gemm_il<BM, BN, WM, WN, BK, MINB>), dim3(nwg), dim3(256), 0, 0, A, B, bias, C, s.M,
                         s.N, s.K, tn);
    else
      hipLaunchKernelGGL((tile_gemm<BM, BN, WM, WN, BK, MINB>), dim3(nwg), dim3(256), 0, 0, A, B, bias, C, s.M, s.N,
                         s.K, tn);
  };
  launch();
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  // numerics: 64 sampled rows against the f64 reference
  const int nr = 64;
  std::vector<int> rows(nr);
  for (int i = 0; i < nr; ++i) rows[i] = (int)(((int64_t)i * 7919 * 104729) % s.M);
  int* drows;
  double* dref;
  CHECK(hipMalloc(&drows, nr * sizeof(int)));
  CHECK(hipMalloc(&dref, (size_t)nr * s.N * sizeof(double)));
  CHECK(hipMemcpy(drows, rows.data(), nr * sizeof(int), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ref_rows, dim3(nr, (s.N + 255) / 256), dim3(256), 0, 0, A, B, bias, drows, nr, s.N, s.K, dref);
  CHECK(hipDeviceSynchronize());
  std::vector<double> ref((size_t)nr * s.N);
  std::vector<float> got((size_t)s.N);
  CHECK(hipMemcpy(ref.data(), dref, ref.size() * sizeof(double), hipMemcpyDeviceToHost));
  double maxerr = 0;
  for (int i = 0; i < nr; ++i) {
    CHECK(hipMemcpy(got.data(), C + (int64_t)rows[i] * s.N, s.N * sizeof(float), hipMemcpyDeviceToHost));
    for (int n = 0; n < s.N; ++n) maxerr = std::fmax(maxerr, std::fabs(got[n] - ref[(size_t)i * s.N + n]));
  }
  CHECK(hipFree(drows));
  CHECK(hipFree(dref));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  const double tf = 2.0 * s.M * (double)s.N * s.K / ms / 1e9;
  std::printf("{\"tile\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"ms\": %.4f, \"tflops\": %.1f, \"max_abs_err\": %.2e}\n",
              name, s.M, s.N, s.K, ms, tf, maxerr);
  std::fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 10;
  const Shape shapes[] = {{2500096, 512, 512}, {262144, 512, 512}, {4096, 4096, 4096}, {8192, 1024, 1024}};
  for (const Shape& s : shapes) {
    float *A, *B, *bias, *C;
    CHECK(hipMalloc(&A, (size_t)s.M * s.K * 4));
    CHECK(hipMalloc(&B, (size_t)s.K * s.N * 4));
    CHECK(hipMalloc(&bias, (size_t)s.N * 4));
    CHECK(hipMalloc(&C, (size_t)s.M * s.N * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, A, (int64_t)s.M * s.K, 1u, 2.f);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, B, (int64_t)s.K * s.N, 2u, 2.f / std::sqrt((float)s.K));
    hipLaunchKernelGGL(fill, dim3(16), dim3(256), 0, 0, bias, (int64_t)s.N, 3u, 1.f);
    CHECK(hipDeviceSynchronize());
    float* Bt;
    CHECK(hipMalloc(&Bt, (size_t)s.K * s.N * 4));
    hipLaunchKernelGGL(transpose, dim3(1024), dim3(256), 0, 0, B, Bt, s.K, s.N);
    CHECK(hipDeviceSynchronize());
    run<128, 128, 2, 2, 16, 2>("128x128 w64x64 bk16 occ2 (walls)", s, A, B, bias, C, iters);
    run<128, 128, 2, 2, 16, 2, 1>("IL 128x128 occ2", s, A, B, bias, C, iters);
    run<128, 128, 2, 2, 16, 3, 1>("IL 128x128 occ3", s, A, B, bias, C, iters);
    run<128, 128, 2, 2, 16, 2, 3>("IL+splitW 128x128 occ2", s, A, B, bias, C, iters);
    run<256, 128, 2, 2, 16, 2, 1>("IL 256x128 occ2", s, A, B, bias, C, iters);
    run<256, 128, 2, 2, 16, 1, 1>("IL 256x128 occ1", s, A, B, bias, C, iters);
    run<256, 128, 2, 2, 16, 2, 3>("IL+splitW 256x128 occ2", s, A, B, bias, C, iters);
    run<256, 64, 4, 1, 16, 2, 1>("IL 256x64 w64x64 occ2", s, A, B, bias, C, iters);
    run<256, 64, 4, 1, 16, 3, 1>("IL 256x64 w64x64 occ3", s, A, B, bias, C, iters);
    CHECK(hipFree(Bt));
    CHECK(hipFree(A));
    CHECK(hipFree(B));
    CHECK(hipFree(bias));
    CHECK(hipFree(C));
  }
  return 0;
}

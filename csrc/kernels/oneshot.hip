// One-shot all-reduce for small payloads over xGMI peer mappings (gfx950).
//
// The reference combines one partial per partition on the Spark driver
// (RDD.reduce: reference src/main/scala/org/tensorframes/impl/DebugRowOps.scala:500,
// :524-525, pairwise combine :732-750). Here the partials of the ranks (one
// process per GPU) are combined on the GPUs: a reduce_blocks / reduce_rows
// partial is a few KB (one output cell, e.g. 4 KB for f32[1024]), so the cost
// is latency, not bandwidth. A ring all-reduce takes 2(N-1)
// dependent hops; this takes ONE: every rank publishes its partial in its own
// IPC-exported buffer, tells each peer with a flag word written straight into
// the peer's buffer, and, once all N flags are in, reads the N partials over
// the point-to-point xGMI links (all 7 in parallel on an 8-GPU node) and folds
// them in rank order. Every rank folds the same values in the same order, so
// all ranks hold bitwise the same result (deterministic, also for floats).
//
// Buffer of each rank (allocated UNCACHED by comm/comm.cpp OneShotComm, so no
// GPU's L2 keeps a copy of a line another GPU writes over xGMI; exported with
// hipIpcGetMemHandle, opened by every peer):
//   [slot 0 data: 64 KB][slot 1 data: 64 KB][flags: 2 slots x 8 ranks u32]
// Call e uses slot e & 1 and writes epoch e into the flags. Reusing a slot two
// calls later is safe: a rank reaches call e+2 only after its call e+1 saw
// every peer's e+1 flag, which each peer wrote after its call e (same stream,
// in order) had finished reading. Every access to the shared buffers is a
// system-scope atomic (sc0 sc1: coherent across XCD L2s and across GPUs, so it
// does not depend on how an importing process maps the pages), and the flag
// wait is bounded (Config.collective_timeout_s of s_memrealtime, passed per
// launch) so a missing peer ends in an error word, never in a wave that spins
// forever.
#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

template <typename T, int OP>
__device__ __forceinline__ T fold(T a, T b) {
  if constexpr (OP == (int)RedOp::SUM) return a + b;
  if constexpr (OP == (int)RedOp::PROD) return a * b;
  if constexpr (OP == (int)RedOp::MIN) return b < a ? b : a;
  return b > a ? b : a;
}

constexpr int kThreads = 1024;
constexpr uint64_t kTicksPerUs = 100;  // the realtime counter runs at 100 MHz

// 8-byte granules: the shared buffers are touched with 64-bit system-scope
// atomics (half the transactions of 4-byte ones for f32 / i32 payloads)
template <typename T>
union Granule {
  uint64_t u;
  T v[8 / sizeof(T)];
};

template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void oneshot_kernel(const T* in, T* out, int64_t n,
                                                          int rank, int world, OneShotPeers p, uint32_t epoch,
                                                          int slot, uint64_t spin_ticks) {
  constexpr int E = 8 / sizeof(T);  // elements per granule
  const int tid = threadIdx.x;
  const int64_t ng = (n + E - 1) / E;
  // 1. publish this rank's partial in its own buffer
  uint64_t* mine = reinterpret_cast<uint64_t*>(static_cast<char*>(p.buf[rank]) + slot * kOneShotSlotBytes);
  for (int64_t g = tid; g < ng; g += kThreads) {
    Granule<T> x;
    x.u = 0;
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (g * E + e < n) x.v[e] = in[g * E + e];
    __hip_atomic_store(mine + g, x.u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 2. tell every peer (lane r writes rank r's flag word for this rank)
  if (tid < world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t* f = reinterpret_cast<uint32_t*>(static_cast<char*>(p.buf[tid]) + kOneShotFlagOffset) + slot * 8 + rank;
    __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every peer's flag (bounded)
  if (tid < world) {
    const uint32_t* f =
        reinterpret_cast<const uint32_t*>(static_cast<char*>(p.buf[rank]) + kOneShotFlagOffset) + slot * 8 + tid;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > spin_ticks) {
        int* err = reinterpret_cast<int*>(static_cast<char*>(p.buf[rank]) + kOneShotErrOffset);
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 4. fold the N partials in rank order
  for (int64_t g = tid; g < ng; g += kThreads) {
    Granule<T> acc;
    acc.u = __hip_atomic_load(reinterpret_cast<const uint64_t*>(static_cast<const char*>(p.buf[0]) +
                                                                 slot * kOneShotSlotBytes) + g,
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int r = 1; r < world; ++r) {
      Granule<T> x;
      x.u = __hip_atomic_load(reinterpret_cast<const uint64_t*>(static_cast<const char*>(p.buf[r]) +
                                                                 slot * kOneShotSlotBytes) + g,
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
      for (int e = 0; e < E; ++e) acc.v[e] = fold<T, OP>(acc.v[e], x.v[e]);
    }
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (g * E + e < n) out[g * E + e] = acc.v[e];
  }
}

// fault injection (device_stall): spin, bounded, then exit
__global__ __launch_bounds__(64) void stall_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

template <typename T>
void launch_t(RedOp op, const void* in, void* out, int64_t n, int rank, int world, const OneShotPeers& p,
              uint32_t epoch, uint64_t ticks, hipStream_t s) {
  const int slot = static_cast<int>(epoch & 1u);
  const T* x = static_cast<const T*>(in);
  T* y = static_cast<T*>(out);
#define TFA_OS(OP_)                                                                                        \
  hipLaunchKernelGGL((oneshot_kernel<T, (int)OP_>), dim3(1), dim3(kThreads), 0, s, x, y, n, rank, world, p, \
                     epoch, slot, ticks)
  switch (op) {
    case RedOp::SUM: TFA_OS(RedOp::SUM); break;
    case RedOp::PROD: TFA_OS(RedOp::PROD); break;
    case RedOp::MIN: TFA_OS(RedOp::MIN); break;
    case RedOp::MAX: TFA_OS(RedOp::MAX); break;
    default: TFA_CHECK(false, "oneshot all-reduce: unsupported op");
  }
#undef TFA_OS
}

}  // namespace

void oneshot_all_reduce(RedOp op, DType dt, const void* in, void* out, int64_t n, int rank, int world,
                        const OneShotPeers& p, uint32_t epoch, uint64_t timeout_us, hipStream_t s) {
  TFA_CHECK(world >= 1 && world <= kOneShotMaxRanks && rank >= 0 && rank < world, "oneshot: bad rank/world");
  TFA_CHECK(n >= 0 && n * dtype_size(dt) <= static_cast<int64_t>(kOneShotSlotBytes), "oneshot: payload over ",
            kOneShotSlotBytes, " bytes");
  for (int r = 0; r < world; ++r) TFA_CHECK(p.buf[r] != nullptr, "oneshot: peer ", r, " not mapped");
  // every wait is bounded: at least 1 ms, at most one hour
  const uint64_t ticks = std::min<uint64_t>(std::max<uint64_t>(timeout_us, 1000), 3600ull * 1000000ull) * kTicksPerUs;
  switch (dt) {
    case DType::F32: launch_t<float>(op, in, out, n, rank, world, p, epoch, ticks, s); break;
    case DType::F64: launch_t<double>(op, in, out, n, rank, world, p, epoch, ticks, s); break;
    case DType::I32: launch_t<int32_t>(op, in, out, n, rank, world, p, epoch, ticks, s); break;
    case DType::I64: launch_t<int64_t>(op, in, out, n, rank, world, p, epoch, ticks, s); break;
    default: TFA_CHECK(false, "oneshot all-reduce: dtype ", dtype_name(dt), " not supported");
  }
  TFA_LAUNCH_CHECK("oneshot_all_reduce");
}

void device_stall(uint64_t us, hipStream_t s) {
  const uint64_t ticks = std::min<uint64_t>(us, 60ull * 1000000ull) * kTicksPerUs;
  hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, s, ticks);
  TFA_LAUNCH_CHECK("device_stall");
}

}  // namespace k
}  // namespace tfa

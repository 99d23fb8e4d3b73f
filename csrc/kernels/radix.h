// Device sort / scan primitives for gfx950, written for the groupBy paths
// (groupby.hip): a stable LSD radix sort of (key, value) pairs and a
// reduce-then-scan prefix sum. No rocPRIM / hipCUB.
//
// Radix sort, per 8-bit digit pass (3 launches + a scan):
//   hist    one block per 4096-key tile: per-wave LDS histograms (ds_add),
//           folded and stored digit-major: counts[digit * tiles + tile]
//   scan    exclusive prefix of counts (the digit-major order makes each
//           (digit, tile) offset the stable global position of its first key)
//   scatter the tile is walked in 16 steps of 256 keys (striped, coalesced
//           loads); inside a wave, keys of equal digit find each other with
//           8 ballots (wave64 multisplit: peers = AND of the matching bit
//           masks), rank = popcount of lower peers; per-wave digit counts go
//           through LDS for the cross-wave prefix and a running per-digit
//           cursor keeps the order across steps. Stable.
// Keys are unsigned (callers map signed / float keys to an order-preserving
// unsigned form first). Values may be generated (iota) in the first pass.
#pragma once

#include <algorithm>
#include <cstdint>

#include "hip_common.h"

namespace tfa {
namespace k {
namespace radix {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kSteps = 16;
constexpr int kTile = kThreads * kSteps;  // keys per block
constexpr int kBits = 8;
constexpr int kRadix = 1 << kBits;

inline size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }
inline int64_t tiles(int64_t n) { return (n + kTile - 1) / kTile; }

// ------------------------------------------------------------------ scan
// tile of the scan: 256 threads x 8 consecutive items
constexpr int kScanItems = 8;
constexpr int kScanTile = kThreads * kScanItems;

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// exclusive prefix of `v` over the block (returns it; *total = block sum)
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* lds_waves /*[kWaves]*/, T* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T incl = wave_incl_scan(v, lane);
  if (lane == 63) lds_waves[w] = incl;
  __syncthreads();
  T before = 0, sum = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    const T x = lds_waves[i];
    before += i < w ? x : T(0);
    sum += x;
  }
  __syncthreads();
  *total = sum;
  return before + incl - v;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void scan_tile_sums(const T* __restrict__ in, int64_t n, T* __restrict__ sums) {
  __shared__ T lw[kWaves];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  T s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j)
    if (base + j < n) s += in[base + j];
  T total;
  (void)block_excl_scan(s, lw, &total);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// one block: exclusive scan of the tile sums in place (any count)
template <typename T>
__global__ __launch_bounds__(kThreads) void scan_sums_single(T* __restrict__ sums, int64_t m) {
  __shared__ T lw[kWaves];
  T carry = 0;
  for (int64_t c = 0; c < m; c += kScanTile) {
    const int64_t base = c + (int64_t)threadIdx.x * kScanItems;
    T v[kScanItems];
    T s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      v[j] = base + j < m ? sums[base + j] : T(0);
      s += v[j];
    }
    T total;
    T run = carry + block_excl_scan(s, lw, &total);
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      if (base + j < m) sums[base + j] = run;
      run += v[j];
    }
    carry += total;
  }
}

// out = scan(in) + tile offset; in and out may alias (each block reads its
// tile before writing it)
template <typename T, bool INCLUSIVE>
__global__ __launch_bounds__(kThreads) void scan_tiles(const T* in, T* out, int64_t n, const T* __restrict__ offs) {
  __shared__ T lw[kWaves];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  T v[kScanItems];
  T s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = base + j < n ? in[base + j] : T(0);
    s += v[j];
  }
  T total;
  T run = block_excl_scan(s, lw, &total) + (offs ? offs[blockIdx.x] : T(0));
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (INCLUSIVE) run += v[j];
    if (base + j < n) out[base + j] = run;
    if (!INCLUSIVE) run += v[j];
  }
}

template <typename T>
size_t scan_ws_bytes(int64_t n) {
  return align_up(static_cast<size_t>((n + kScanTile - 1) / kScanTile + 1) * sizeof(T));
}

// prefix sum of n elements (exclusive or inclusive); in may equal out
template <typename T>
void scan(const T* in, T* out, int64_t n, bool inclusive, void* ws, hipStream_t s) {
  if (n <= 0) return;
  const int64_t nt = (n + kScanTile - 1) / kScanTile;
  T* sums = static_cast<T*>(ws);
  if (nt == 1) {
    if (inclusive) hipLaunchKernelGGL((scan_tiles<T, true>), dim3(1), dim3(kThreads), 0, s, in, out, n, (const T*)nullptr);
    else hipLaunchKernelGGL((scan_tiles<T, false>), dim3(1), dim3(kThreads), 0, s, in, out, n, (const T*)nullptr);
    return;
  }
  hipLaunchKernelGGL((scan_tile_sums<T>), dim3((unsigned)nt), dim3(kThreads), 0, s, in, n, sums);
  hipLaunchKernelGGL((scan_sums_single<T>), dim3(1), dim3(kThreads), 0, s, sums, nt);
  if (inclusive) hipLaunchKernelGGL((scan_tiles<T, true>), dim3((unsigned)nt), dim3(kThreads), 0, s, in, out, n, (const T*)sums);
  else hipLaunchKernelGGL((scan_tiles<T, false>), dim3((unsigned)nt), dim3(kThreads), 0, s, in, out, n, (const T*)sums);
}

// ------------------------------------------------------------------ radix sort
template <typename K>
__device__ __forceinline__ uint32_t digit_of(K k, int shift) {
  return static_cast<uint32_t>(k >> shift) & (kRadix - 1);
}

template <typename K>
__global__ __launch_bounds__(kThreads) void hist_kernel(const K* __restrict__ keys, int64_t n, int shift,
                                                        uint32_t* __restrict__ counts, int64_t ntiles) {
  __shared__ uint32_t h[kWaves][kRadix];
  const int w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&h[0][0])[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile + threadIdx.x;
#pragma unroll 4
  for (int j = 0; j < kSteps; ++j) {
    const int64_t i = base + (int64_t)j * kThreads;
    if (i < n) atomicAdd(&h[w][digit_of(keys[i], shift)], 1u);
  }
  __syncthreads();
  const int d = threadIdx.x;  // kThreads == kRadix
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) c += h[i][d];
  counts[(int64_t)d * ntiles + blockIdx.x] = c;
}

// vals_in == nullptr: the value of key i is i (first pass of an argsort)
template <typename K, typename V>
__global__ __launch_bounds__(kThreads) void scatter_kernel(const K* __restrict__ keys_in, const V* __restrict__ vals_in,
                                                           K* __restrict__ keys_out, V* __restrict__ vals_out,
                                                           int64_t n, int shift,
                                                           const uint32_t* __restrict__ offsets, int64_t ntiles) {
  __shared__ uint32_t run[kRadix];
  __shared__ uint32_t wcnt[kWaves][kRadix];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  run[threadIdx.x] = offsets[(int64_t)threadIdx.x * ntiles + blockIdx.x];
#pragma unroll
  for (int i = 0; i < kWaves; ++i) wcnt[i][threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile + threadIdx.x;
  for (int j = 0; j < kSteps; ++j) {
    const int64_t i = base + (int64_t)j * kThreads;
    const bool valid = i < n;
    K key = 0;
    V val = 0;
    uint32_t d = 0;
    if (valid) {
      key = keys_in[i];
      val = vals_in ? vals_in[i] : static_cast<V>(i);
      d = digit_of(key, shift);
    }
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kBits; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint64_t lower = peers & lt;
    if (valid && lower == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = run[d] + (uint32_t)__popcll(lower);
      for (int q = 0; q < w; ++q) pos += wcnt[q][d];
      keys_out[pos] = key;
      vals_out[pos] = val;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int q = 0; q < kWaves; ++q) {
      add += wcnt[q][threadIdx.x];
      wcnt[q][threadIdx.x] = 0;
    }
    run[threadIdx.x] += add;
    __syncthreads();
  }
}

// workspace: alternate key/value buffers, digit counts, scan scratch
template <typename K, typename V>
size_t sort_ws_bytes(int64_t n) {
  const int64_t cnt = (int64_t)kRadix * tiles(n);
  return align_up(n * sizeof(K)) + align_up(n * sizeof(V)) + align_up(cnt * sizeof(uint32_t)) +
         scan_ws_bytes<uint32_t>(cnt);
}

// stable sort of (keys, vals) by key bits [0, bits); results in keys_out /
// vals_out (which must not alias the inputs). vals_in == nullptr sorts
// (key, index) pairs.
template <typename K, typename V>
void sort_pairs(const K* keys_in, const V* vals_in, K* keys_out, V* vals_out, int64_t n, int bits, void* ws,
                size_t ws_size, hipStream_t s) {
  const size_t need = sort_ws_bytes<K, V>(n);
  TFA_CHECK(ws_size >= need, "radix sort: workspace too small");
  TFA_CHECK(n < (int64_t(1) << 32) - 1, "radix sort: more than 2^32 keys");
  if (n <= 0) return;
  const int64_t nt = tiles(n);
  TFA_CHECK(nt <= 0x7fffffff, "radix sort: too many tiles");
  char* p = static_cast<char*>(ws);
  K* kalt = reinterpret_cast<K*>(p);
  p += align_up(n * sizeof(K));
  V* valt = reinterpret_cast<V*>(p);
  p += align_up(n * sizeof(V));
  uint32_t* counts = reinterpret_cast<uint32_t*>(p);
  p += align_up((int64_t)kRadix * nt * sizeof(uint32_t));
  void* scan_ws = p;
  bits = std::max(1, std::min(bits, int(sizeof(K) * 8)));
  const int passes = (bits + kBits - 1) / kBits;
  const K* kin = keys_in;
  const V* vin = vals_in;
  for (int ps = 0; ps < passes; ++ps) {
    // the last pass lands in the caller's buffers
    const bool to_out = ((passes - 1 - ps) % 2) == 0;
    K* kout = to_out ? keys_out : kalt;
    V* vout = to_out ? vals_out : valt;
    const int shift = ps * kBits;
    hipLaunchKernelGGL((hist_kernel<K>), dim3((unsigned)nt), dim3(kThreads), 0, s, kin, n, shift, counts, nt);
    scan<uint32_t>(counts, counts, (int64_t)kRadix * nt, false, scan_ws, s);
    hipLaunchKernelGGL((scatter_kernel<K, V>), dim3((unsigned)nt), dim3(kThreads), 0, s, kin, vin, kout, vout, n,
                       shift, (const uint32_t*)counts, nt);
    kin = kout;
    vin = vout;
  }
}

}  // namespace radix
}  // namespace k
}  // namespace tfa

// Device-side groupBy segmentation for gfx950: key factorisation by radix
// sort (rocPRIM) + head flags + scan, and a key hash for the cross-rank
// shuffle.
//
// The reference groups rows with a Spark shuffle + UDAF that compacts every
// 10 rows through a TF session (reference:
// src/main/scala/org/tensorframes/impl/DebugRowOps.scala:547-695). Here the
// keys of a block never leave HBM: they are sorted once, every row gets its
// group id (groups in ascending key order, like np.unique), and the values
// are then reduced per group by the segmented-reduction kernels (reduce.hip)
// without being moved.
#include <algorithm>
#include <climits>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

template <typename I>
__global__ __launch_bounds__(256) void iota_kernel(I* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (I)i;
}

// head[i] = 1 where sorted[i] starts a new group
template <typename K, typename I>
__global__ __launch_bounds__(256) void head_kernel(const K* __restrict__ sorted, I* __restrict__ head, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    head[i] = (i == 0 || !(sorted[i] == sorted[i - 1])) ? I(1) : I(0);
}

// ids[perm[i]] = seg[i] - 1; uniq[seg[i] - 1] = sorted[i] at heads
template <typename K, typename I>
__global__ __launch_bounds__(256) void scatter_kernel(const K* __restrict__ sorted, const I* __restrict__ perm,
                                                      const I* __restrict__ seg, int64_t* __restrict__ ids,
                                                      K* __restrict__ uniq, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t g = (int64_t)seg[i] - 1;
    ids[perm[i]] = g;
    if (i == 0 || !(sorted[i] == sorted[i - 1])) uniq[g] = sorted[i];
  }
}

// 64-bit finaliser (splitmix64): the same value on every rank for the same key
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

template <typename K>
__device__ __forceinline__ uint64_t key_bits(K v) {
  if constexpr (std::is_floating_point<K>::value) {
    if (v == K(0)) v = K(0);  // -0.0 and 0.0 are one key
    if constexpr (sizeof(K) == 8) return __double_as_longlong(v);
    else return (uint64_t)(uint32_t)__float_as_int(v);
  } else {
    return (uint64_t)(int64_t)v;
  }
}

template <typename K>
__global__ __launch_bounds__(256) void hash_kernel(const K* __restrict__ keys, int64_t n, uint64_t* __restrict__ h,
                                                   int accumulate) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t v = mix64(key_bits(keys[i]));
    h[i] = accumulate ? mix64(h[i] * 1000003ull ^ v) : v;
  }
}

// dest[i] = h[i] % world
__global__ __launch_bounds__(256) void mod_kernel(const uint64_t* __restrict__ h, int64_t n, int64_t world,
                                                  int64_t* __restrict__ dest) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dest[i] = (int64_t)(h[i] % (uint64_t)world);
}

// rep[ids[i]] = i: any row of a group represents it (concurrent writers all
// store valid rows of the same group)
__global__ __launch_bounds__(256) void rep_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t* __restrict__ rep) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) rep[ids[i]] = i;
}

// counts[d] = rows with dest d (world is small: one LDS histogram per block)
__global__ __launch_bounds__(256) void dest_hist_kernel(const int64_t* __restrict__ dest, int64_t n, int64_t world,
                                                        unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    atomicAdd(&h[dest[i]], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < world; i += blockDim.x)
    if (h[i]) atomicAdd(&counts[i], (unsigned long long)h[i]);
}

__global__ __launch_bounds__(256) void widen_kernel(const int32_t* __restrict__ a, int64_t* __restrict__ b, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = a[i];
}

// offsets[g] = first sorted position with id >= g, for g in (prev, cur]
// (ids clamped to [-1, nseg]: out-of-range ids drop out of every segment)
template <typename I>
__global__ __launch_bounds__(256) void offsets_kernel(const I* __restrict__ sorted, int64_t n, int64_t nseg,
                                                      int64_t* __restrict__ off) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
    int64_t prev = i == 0 ? -1 : (int64_t)sorted[i - 1];
    int64_t cur = i == n ? nseg : (int64_t)sorted[i];
    prev = prev < -1 ? -1 : (prev > nseg ? nseg : prev);
    cur = cur < -1 ? -1 : (cur > nseg ? nseg : cur);
    for (int64_t g = prev + 1; g <= cur; ++g) off[g] = i;
  }
}

template <typename I>
__global__ __launch_bounds__(256) void seg_key_kernel(const I* __restrict__ ids, uint32_t* __restrict__ key, int64_t n,
                                                      int64_t nseg) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t v = (int64_t)ids[i];
    v = v < -1 ? -1 : (v > nseg ? nseg : v);
    key[i] = (uint32_t)(v + 1);
  }
}

// sorted keys are (segment + 1): offsets[g] = first position with segment >= g
__global__ __launch_bounds__(256) void offsets_u32_kernel(const uint32_t* __restrict__ sorted, int64_t n, int64_t nseg,
                                                          int64_t* __restrict__ off) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
    const int64_t prev = i == 0 ? -1 : (int64_t)sorted[i - 1] - 1;
    const int64_t cur = i == n ? nseg : (int64_t)sorted[i] - 1;
    for (int64_t g = prev + 1; g <= cur; ++g) off[g] = i;
  }
}

// integer keys: min / max (one block-level pass + atomics), so only the bits of
// (key - min) are radix-sorted
template <typename K>
__global__ __launch_bounds__(256) void minmax_kernel(const K* __restrict__ keys, int64_t n,
                                                     long long* __restrict__ mm) {
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long long v = (long long)keys[i];
    lo = v < lo ? v : lo;
    hi = v > hi ? v : hi;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const long long ol = __shfl_xor(lo, off, 64), oh = __shfl_xor(hi, off, 64);
    lo = ol < lo ? ol : lo;
    hi = oh > hi ? oh : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

__global__ void minmax_init_kernel(long long* mm) {
  if (threadIdx.x == 0) {
    mm[0] = LLONG_MAX;
    mm[1] = LLONG_MIN;
  }
}

template <typename K, typename U>
__global__ __launch_bounds__(256) void shift_kernel(const K* __restrict__ keys, int64_t n, long long lo,
                                                    U* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = (U)((unsigned long long)((long long)keys[i] - lo));
}

// ids[perm[i]] = seg[i] - 1; uniq[g] = sorted + lo at heads
template <typename K, typename U, typename I>
__global__ __launch_bounds__(256) void scatter_shifted_kernel(const U* __restrict__ sorted, const I* __restrict__ perm,
                                                              const I* __restrict__ seg, int64_t* __restrict__ ids,
                                                              K* __restrict__ uniq, int64_t n, long long lo) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t g = (int64_t)seg[i] - 1;
    ids[perm[i]] = g;
    if (i == 0 || sorted[i] != sorted[i - 1]) uniq[g] = (K)((long long)sorted[i] + lo);
  }
}

size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

template <typename K, typename I>
size_t ws_bytes(int64_t n) {
  size_t sort_tmp = 0, scan_tmp = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_tmp, (const K*)nullptr, (K*)nullptr, (const I*)nullptr, (I*)nullptr,
                                  (size_t)n);
  (void)rocprim::inclusive_scan(nullptr, scan_tmp, (const I*)nullptr, (I*)nullptr, (size_t)n, rocprim::plus<I>());
  size_t narrow_tmp = 0;
  (void)rocprim::radix_sort_pairs(nullptr, narrow_tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const I*)nullptr, (I*)nullptr, (size_t)n);
  // sorted keys, iota, perm, head/seg, scratch of the larger primitive, nseg cell
  // (the narrow integer layout needs two uint32 key arrays in place of the sorted keys)
  return std::max(align_up(n * sizeof(K)), 2 * align_up(n * sizeof(uint32_t))) + 3 * align_up(n * sizeof(I)) +
         align_up(std::max({sort_tmp, scan_tmp, narrow_tmp})) + 256;
}

// integer keys spanning < 2^32 values: radix-sort only the bits of key - min
// (10M keys in [0, 100k): 17 bits = 3 passes instead of 8 for int64)
template <typename K, typename I>
bool factorize_int_narrow(const K* keys, int64_t n, int64_t* ids, K* uniq, void* ws, size_t ws_size,
                          int64_t* nseg_host, hipStream_t s) {
  char* p = static_cast<char*>(ws);
  long long* mm = reinterpret_cast<long long*>(p + ws_size - 256);  // the reserved cell at the end
  hipLaunchKernelGGL(minmax_init_kernel, dim3(1), dim3(64), 0, s, mm);
  hipLaunchKernelGGL((minmax_kernel<K>), dim3(std::min(ew_grid(n), 1024)), dim3(256), 0, s, keys, n, mm);
  long long got[2] = {0, 0};
  TFA_CHECK(hipMemcpyAsync(got, mm, sizeof(got), hipMemcpyDeviceToHost, s) == hipSuccess, "factorize: D2H failed");
  TFA_CHECK(hipStreamSynchronize(s) == hipSuccess, "factorize: sync failed");
  const unsigned long long range = (unsigned long long)(got[1] - got[0]);
  if (range >= (1ull << 32)) return false;
  int bits = 1;
  while (bits < 32 && (1ull << bits) <= range) ++bits;
  uint32_t* key = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  uint32_t* sorted = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  I* iota = reinterpret_cast<I*>(p);
  p += align_up(n * sizeof(I));
  I* perm = reinterpret_cast<I*>(p);
  p += align_up(n * sizeof(I));
  I* seg = reinterpret_cast<I*>(p);
  p += align_up(n * sizeof(I));
  size_t tmp_size = ws_size - 256 - static_cast<size_t>(p - static_cast<char*>(ws));
  const int grid = ew_grid(n);
  hipLaunchKernelGGL((shift_kernel<K, uint32_t>), dim3(grid), dim3(256), 0, s, keys, n, got[0], key);
  hipLaunchKernelGGL((iota_kernel<I>), dim3(grid), dim3(256), 0, s, iota, n);
  size_t sz = tmp_size;
  TFA_CHECK(rocprim::radix_sort_pairs(p, sz, key, sorted, iota, perm, (size_t)n, 0, bits, s) == hipSuccess,
            "factorize: radix sort failed");
  hipLaunchKernelGGL((head_kernel<uint32_t, I>), dim3(grid), dim3(256), 0, s, sorted, iota, n);
  sz = tmp_size;
  TFA_CHECK(rocprim::inclusive_scan(p, sz, iota, seg, (size_t)n, rocprim::plus<I>(), s) == hipSuccess,
            "factorize: scan failed");
  hipLaunchKernelGGL((scatter_shifted_kernel<K, uint32_t, I>), dim3(grid), dim3(256), 0, s, sorted, perm, seg, ids,
                     uniq, n, got[0]);
  I count = 0;
  TFA_CHECK(hipMemcpyAsync(&count, seg + (n - 1), sizeof(I), hipMemcpyDeviceToHost, s) == hipSuccess,
            "factorize: D2H failed");
  TFA_CHECK(hipStreamSynchronize(s) == hipSuccess, "factorize: sync failed");
  *nseg_host = static_cast<int64_t>(count);
  return true;
}

template <typename K, typename I>
void factorize_typed(const K* keys, int64_t n, int64_t* ids, K* uniq, void* ws, size_t ws_size, int64_t* nseg_host,
                     hipStream_t s) {
  if constexpr (std::is_integral<K>::value) {
    if (factorize_int_narrow<K, I>(keys, n, ids, uniq, ws, ws_size, nseg_host, s)) return;
  }
  char* p = static_cast<char*>(ws);
  K* sorted = reinterpret_cast<K*>(p);
  p += align_up(n * sizeof(K));
  I* iota = reinterpret_cast<I*>(p);
  p += align_up(n * sizeof(I));
  I* perm = reinterpret_cast<I*>(p);
  p += align_up(n * sizeof(I));
  I* seg = reinterpret_cast<I*>(p);
  p += align_up(n * sizeof(I));
  I* last = reinterpret_cast<I*>(p);  // 256-byte cell at the end holds the group count
  p += 256;
  void* tmp = p;
  size_t tmp_size = ws_size - static_cast<size_t>(p - static_cast<char*>(ws));
  const int grid = ew_grid(n);
  hipLaunchKernelGGL((iota_kernel<I>), dim3(grid), dim3(256), 0, s, iota, n);
  size_t sz = tmp_size;
  TFA_CHECK(rocprim::radix_sort_pairs(tmp, sz, keys, sorted, iota, perm, (size_t)n, 0, int(sizeof(K) * 8), s) ==
                hipSuccess,
            "factorize: radix sort failed");
  // head flags into `iota` (free now), inclusive scan into `seg`
  hipLaunchKernelGGL((head_kernel<K, I>), dim3(grid), dim3(256), 0, s, sorted, iota, n);
  sz = tmp_size;
  TFA_CHECK(rocprim::inclusive_scan(tmp, sz, iota, seg, (size_t)n, rocprim::plus<I>(), s) == hipSuccess,
            "factorize: scan failed");
  hipLaunchKernelGGL((scatter_kernel<K, I>), dim3(grid), dim3(256), 0, s, sorted, perm, seg, ids, uniq, n);
  TFA_CHECK(hipMemcpyAsync(last, seg + (n - 1), sizeof(I), hipMemcpyDeviceToDevice, s) == hipSuccess,
            "factorize: copy failed");
  I count = 0;
  TFA_CHECK(hipMemcpyAsync(&count, last, sizeof(I), hipMemcpyDeviceToHost, s) == hipSuccess, "factorize: D2H failed");
  TFA_CHECK(hipStreamSynchronize(s) == hipSuccess, "factorize: sync failed");
  *nseg_host = static_cast<int64_t>(count);
}

}  // namespace

size_t factorize_workspace_bytes(DType dt, int64_t n) {
  const bool small = n < (int64_t(1) << 31);
  switch (dt) {
    case DType::I32: return small ? ws_bytes<int32_t, int32_t>(n) : ws_bytes<int32_t, int64_t>(n);
    case DType::I64: return small ? ws_bytes<int64_t, int32_t>(n) : ws_bytes<int64_t, int64_t>(n);
    case DType::F32: return small ? ws_bytes<float, int32_t>(n) : ws_bytes<float, int64_t>(n);
    case DType::F64: return small ? ws_bytes<double, int32_t>(n) : ws_bytes<double, int64_t>(n);
    default: TFA_CHECK(false, "factorize: unsupported key dtype ", dtype_name(dt));
  }
  return 0;
}

int64_t factorize(DType dt, const void* keys, int64_t n, int64_t* ids, void* uniq, void* ws, size_t ws_size,
                  hipStream_t s) {
  TFA_CHECK(n > 0, "factorize: empty key column");
  TFA_CHECK(ws_size >= factorize_workspace_bytes(dt, n), "factorize: workspace too small");
  int64_t nseg = 0;
  const bool small = n < (int64_t(1) << 31);
#define TFA_FACT(K)                                                                                          \
  if (small)                                                                                                 \
    factorize_typed<K, int32_t>((const K*)keys, n, ids, (K*)uniq, ws, ws_size, &nseg, s);                     \
  else                                                                                                       \
    factorize_typed<K, int64_t>((const K*)keys, n, ids, (K*)uniq, ws, ws_size, &nseg, s);
  switch (dt) {
    case DType::I32: TFA_FACT(int32_t) break;
    case DType::I64: TFA_FACT(int64_t) break;
    case DType::F32: TFA_FACT(float) break;
    case DType::F64: TFA_FACT(double) break;
    default: TFA_CHECK(false, "factorize: unsupported key dtype ", dtype_name(dt));
  }
#undef TFA_FACT
  return nseg;
}

void key_hash(DType dt, const void* keys, int64_t n, uint64_t* h, bool accumulate, hipStream_t s) {
  if (n == 0) return;
  const int grid = ew_grid(n);
  const int acc = accumulate ? 1 : 0;
  switch (dt) {
    case DType::I32: hipLaunchKernelGGL((hash_kernel<int32_t>), dim3(grid), dim3(256), 0, s, (const int32_t*)keys, n, h, acc); break;
    case DType::I64: hipLaunchKernelGGL((hash_kernel<int64_t>), dim3(grid), dim3(256), 0, s, (const int64_t*)keys, n, h, acc); break;
    case DType::F32: hipLaunchKernelGGL((hash_kernel<float>), dim3(grid), dim3(256), 0, s, (const float*)keys, n, h, acc); break;
    case DType::F64: hipLaunchKernelGGL((hash_kernel<double>), dim3(grid), dim3(256), 0, s, (const double*)keys, n, h, acc); break;
    default: TFA_CHECK(false, "key_hash: unsupported key dtype ", dtype_name(dt));
  }
}

size_t segment_csr_workspace_bytes(int64_t n, int64_t nseg) {
  (void)nseg;
  size_t tmp = 0;
  (void)rocprim::radix_sort_pairs(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const int64_t*)nullptr,
                                  (int64_t*)nullptr, (size_t)n);
  return align_up(n * sizeof(int64_t)) + 2 * align_up(n * sizeof(uint32_t)) + align_up(tmp) + 256;
}

void segment_csr(DType idt, const void* ids, int64_t n, int64_t nseg, int64_t* perm, int64_t* offsets, void* ws,
                 size_t ws_size, hipStream_t s) {
  TFA_CHECK(idt == DType::I32 || idt == DType::I64, "segment_csr: int32/int64 ids");
  TFA_CHECK(nseg + 2 < (int64_t(1) << 32), "segment_csr: too many segments");
  TFA_CHECK(ws_size >= segment_csr_workspace_bytes(n, nseg), "segment_csr: workspace too small");
  char* p = static_cast<char*>(ws);
  int64_t* iota = reinterpret_cast<int64_t*>(p);
  p += align_up(n * sizeof(int64_t));
  uint32_t* key = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  uint32_t* sorted = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  size_t tmp = ws_size - static_cast<size_t>(p - static_cast<char*>(ws));
  const int grid = ew_grid(n + 1);
  hipLaunchKernelGGL((iota_kernel<int64_t>), dim3(grid), dim3(256), 0, s, iota, n);
  // key = clamp(id, -1, nseg) + 1: only the bits of [0, nseg + 1] are sorted
  if (idt == DType::I32)
    hipLaunchKernelGGL((seg_key_kernel<int32_t>), dim3(grid), dim3(256), 0, s, static_cast<const int32_t*>(ids), key, n, nseg);
  else
    hipLaunchKernelGGL((seg_key_kernel<int64_t>), dim3(grid), dim3(256), 0, s, static_cast<const int64_t*>(ids), key, n, nseg);
  int bits = 1;
  while (bits < 32 && (int64_t(1) << bits) <= nseg + 1) ++bits;
  TFA_CHECK(rocprim::radix_sort_pairs(p, tmp, key, sorted, iota, perm, (size_t)n, 0, bits, s) == hipSuccess,
            "segment_csr: radix sort failed");
  hipLaunchKernelGGL(offsets_u32_kernel, dim3(grid), dim3(256), 0, s, sorted, n, nseg, offsets);
}

void group_representatives(const int64_t* ids, int64_t n, int64_t* rep, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(rep_kernel, dim3(ew_grid(n)), dim3(256), 0, s, ids, n, rep);
}

size_t partition_workspace_bytes(int64_t n) {
  size_t tmp = 0;
  (void)rocprim::radix_sort_pairs(nullptr, tmp, (const int64_t*)nullptr, (int64_t*)nullptr, (const int64_t*)nullptr,
                                  (int64_t*)nullptr, (size_t)n);
  return 2 * align_up(n * sizeof(int64_t)) + align_up(tmp) + 256;
}

void partition_rows(const int64_t* dest, int64_t n, int64_t world, int64_t* perm, int64_t* counts, void* ws,
                    size_t ws_size, hipStream_t s) {
  TFA_CHECK(world >= 1 && world <= 256, "partition_rows: world must be in [1, 256]");
  TFA_CHECK(ws_size >= partition_workspace_bytes(n), "partition_rows: workspace too small");
  TFA_CHECK(hipMemsetAsync(counts, 0, world * sizeof(int64_t), s) == hipSuccess, "partition_rows: memset failed");
  if (n == 0) return;
  char* p = static_cast<char*>(ws);
  int64_t* iota = reinterpret_cast<int64_t*>(p);
  p += align_up(n * sizeof(int64_t));
  int64_t* sorted_dest = reinterpret_cast<int64_t*>(p);
  p += align_up(n * sizeof(int64_t));
  size_t tmp = ws_size - static_cast<size_t>(p - static_cast<char*>(ws));
  hipLaunchKernelGGL((iota_kernel<int64_t>), dim3(ew_grid(n)), dim3(256), 0, s, iota, n);
  int bits = 1;
  while ((int64_t(1) << bits) < world) ++bits;
  // stable: rows keep their order within a destination
  TFA_CHECK(rocprim::radix_sort_pairs(p, tmp, dest, sorted_dest, iota, perm, (size_t)n, 0, bits, s) == hipSuccess,
            "partition_rows: radix sort failed");
  hipLaunchKernelGGL(dest_hist_kernel, dim3(std::min<int64_t>(ew_grid(n), 1024)), dim3(256), 0, s, dest, n, world,
                     reinterpret_cast<unsigned long long*>(counts));
}

void hash_mod(const uint64_t* h, int64_t n, int64_t world, int64_t* dest, hipStream_t s) {
  if (n == 0) return;
  TFA_CHECK(world >= 1, "hash_mod: world must be >= 1");
  hipLaunchKernelGGL(mod_kernel, dim3(ew_grid(n)), dim3(256), 0, s, h, n, world, dest);
}

}  // namespace k
}  // namespace tfa

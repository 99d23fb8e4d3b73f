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

size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

template <typename K, typename I>
size_t ws_bytes(int64_t n) {
  size_t sort_tmp = 0, scan_tmp = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_tmp, (const K*)nullptr, (K*)nullptr, (const I*)nullptr, (I*)nullptr,
                                  (size_t)n);
  (void)rocprim::inclusive_scan(nullptr, scan_tmp, (const I*)nullptr, (I*)nullptr, (size_t)n, rocprim::plus<I>());
  // sorted keys, iota, perm, head/seg, scratch of the larger primitive, nseg cell
  return align_up(n * sizeof(K)) + 3 * align_up(n * sizeof(I)) + align_up(std::max(sort_tmp, scan_tmp)) + 256;
}

template <typename K, typename I>
void factorize_typed(const K* keys, int64_t n, int64_t* ids, K* uniq, void* ws, size_t ws_size, int64_t* nseg_host,
                     hipStream_t s) {
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

void hash_mod(const uint64_t* h, int64_t n, int64_t world, int64_t* dest, hipStream_t s) {
  if (n == 0) return;
  TFA_CHECK(world >= 1, "hash_mod: world must be >= 1");
  hipLaunchKernelGGL(mod_kernel, dim3(ew_grid(n)), dim3(256), 0, s, h, n, world, dest);
}

}  // namespace k
}  // namespace tfa

// Device-side groupBy segmentation for gfx950: key factorisation, the
// segment CSR of a group-id column, the keyed shuffle's hash / partition.
// Every kernel is our own: the sort and scan primitives are in radix.h.
//
// The reference groups rows with a Spark shuffle + UDAF that compacts every
// 10 rows through a TF session (reference:
// src/main/scala/org/tensorframes/impl/DebugRowOps.scala:547-695). Here the
// keys of a block never leave HBM and every row gets its group id, groups in
// ascending key order (like np.unique; NaN keys form one group after +inf,
// -0.0 and 0.0 are one key). Two factorisation strategies:
//   dense  integer keys whose range (max - min) is at most a few times the
//          row count: direct addressing, no sort. flags[key - min] = 1, one
//          exclusive scan turns the flags into group ids in key order, then
//          ids[i] = slot[key_i - min]. 10M keys over 100k values: five
//          streaming passes.
//   sort   anything else: keys mapped to an order-preserving unsigned form
//          (floats: NaN canonicalised, -0 -> +0), stable radix sort of
//          (key, row) over the significant bits only, head flags + scan,
//          scatter of ids and distinct keys.
#include <algorithm>
#include <climits>
#include <cstring>

#include "hip_common.h"
#include "radix.h"

namespace tfa {
namespace k {

namespace {

using radix::align_up;
constexpr int kT = 256;

// ---------------------------------------------------------------- key maps
// order-preserving signed integer image of a key: ints as they are; floats
// with -0.0 -> +0.0, every NaN -> one canonical NaN, negative values' bits
// flipped so the signed compare of the images is the float order (NaN last)
template <typename K> struct KeyImage { using S = int64_t; using U = uint64_t; };
template <> struct KeyImage<int32_t> { using S = int32_t; using U = uint32_t; };
template <> struct KeyImage<float> { using S = int32_t; using U = uint32_t; };

template <typename K>
__host__ __device__ __forceinline__ typename KeyImage<K>::S key_image(K v) {
  using S = typename KeyImage<K>::S;
  if constexpr (std::is_floating_point<K>::value) {
    if (v != v) return sizeof(K) == 8 ? S(0x7ff8000000000000ll) : S(0x7fc00000);
    if (v == K(0)) v = K(0);
    S b;
    memcpy(&b, &v, sizeof(b));
    return b < 0 ? S(b ^ (sizeof(K) == 8 ? S(0x7fffffffffffffffll) : S(0x7fffffff))) : b;
  } else {
    return S(v);
  }
}

template <typename K>
__host__ __device__ __forceinline__ K key_from_image(typename KeyImage<K>::S b) {
  using S = typename KeyImage<K>::S;
  if constexpr (std::is_floating_point<K>::value) {
    if (b < 0) b = S(b ^ (sizeof(K) == 8 ? S(0x7fffffffffffffffll) : S(0x7fffffff)));
    K v;
    memcpy(&v, &b, sizeof(v));
    return v;
  } else {
    return K(b);
  }
}

// unsigned sort key: the signed image with its sign bit flipped
template <typename K>
__device__ __forceinline__ typename KeyImage<K>::U sort_key(K v) {
  using U = typename KeyImage<K>::U;
  return U(key_image<K>(v)) ^ (U(1) << (sizeof(U) * 8 - 1));
}

template <typename K>
__device__ __forceinline__ K key_from_sort(typename KeyImage<K>::U u) {
  using S = typename KeyImage<K>::S;
  using U = typename KeyImage<K>::U;
  return key_from_image<K>(S(u ^ (U(1) << (sizeof(U) * 8 - 1))));
}

// ---------------------------------------------------------------- min / max
// integer keys: per-block min/max into partials (no atomics), then one block
// folds the partials
template <typename K>
__global__ __launch_bounds__(kT) void minmax_partial_kernel(const K* __restrict__ keys, int64_t n,
                                                            long long* __restrict__ part) {
  __shared__ long long slo[kT / 64], shi[kT / 64];
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
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    slo[w] = lo;
    shi[w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kT / 64; ++i) {
      lo = slo[i] < lo ? slo[i] : lo;
      hi = shi[i] > hi ? shi[i] : hi;
    }
    part[2 * blockIdx.x] = lo;
    part[2 * blockIdx.x + 1] = hi;
  }
}

__global__ __launch_bounds__(kT) void minmax_final_kernel(const long long* __restrict__ part, int nb,
                                                          long long* __restrict__ mm) {
  __shared__ long long slo[kT / 64], shi[kT / 64];
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    lo = part[2 * i] < lo ? part[2 * i] : lo;
    hi = part[2 * i + 1] > hi ? part[2 * i + 1] : hi;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const long long ol = __shfl_xor(lo, off, 64), oh = __shfl_xor(hi, off, 64);
    lo = ol < lo ? ol : lo;
    hi = oh > hi ? oh : hi;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    slo[w] = lo;
    shi[w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kT / 64; ++i) {
      lo = slo[i] < lo ? slo[i] : lo;
      hi = shi[i] > hi ? shi[i] : hi;
    }
    mm[0] = lo;
    mm[1] = hi;
  }
}

constexpr int kMinmaxBlocks = 1024;

// ---------------------------------------------------------------- dense path
__global__ __launch_bounds__(kT) void zero_u32_kernel(uint32_t* __restrict__ p, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0;
}

// flags[key - lo] = 1 (concurrent writers store the same value)
template <typename K>
__global__ __launch_bounds__(kT) void dense_mark_kernel(const K* __restrict__ keys, int64_t n, long long lo,
                                                        uint32_t* __restrict__ flags) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    flags[(long long)keys[i] - lo] = 1u;
}

template <typename K>
__global__ __launch_bounds__(kT) void dense_ids_kernel(const K* __restrict__ keys, int64_t n, long long lo,
                                                       const uint32_t* __restrict__ slot, int64_t* __restrict__ ids) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    ids[i] = (int64_t)slot[(long long)keys[i] - lo];
}

// slot = exclusive scan of the flags over range + 1 entries: value v is
// present iff slot[v + 1] != slot[v]
template <typename K>
__global__ __launch_bounds__(kT) void dense_uniq_kernel(const uint32_t* __restrict__ slot, int64_t range1,
                                                        long long lo, K* __restrict__ uniq) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < range1; v += stride)
    if (slot[v + 1] != slot[v]) uniq[slot[v]] = (K)(lo + v);
}

// ---------------------------------------------------------------- sort path
// narrow unsigned key: key - lo (integer keys spanning < 2^32 values)
template <typename K>
__global__ __launch_bounds__(kT) void shift_kernel(const K* __restrict__ keys, int64_t n, long long lo,
                                                   uint32_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = (uint32_t)((unsigned long long)((long long)keys[i] - lo));
}

template <typename K>
__global__ __launch_bounds__(kT) void sort_key_kernel(const K* __restrict__ keys, int64_t n,
                                                      typename KeyImage<K>::U* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = sort_key<K>(keys[i]);
}

template <typename U>
__global__ __launch_bounds__(kT) void head_kernel(const U* __restrict__ sorted, uint32_t* __restrict__ head, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    head[i] = (i == 0 || sorted[i] != sorted[i - 1]) ? 1u : 0u;
}

// ids[perm[i]] = seg[i] - 1; uniq[seg - 1] = decode(sorted[i]) at heads.
// NARROW: sorted holds key - lo
template <typename K, typename U, bool NARROW>
__global__ __launch_bounds__(kT) void scatter_ids_kernel(const U* __restrict__ sorted, const uint32_t* __restrict__ perm,
                                                         const uint32_t* __restrict__ seg, int64_t* __restrict__ ids,
                                                         K* __restrict__ uniq, int64_t n, long long lo) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t g = (int64_t)seg[i] - 1;
    ids[perm[i]] = g;
    if (i == 0 || sorted[i] != sorted[i - 1]) {
      if constexpr (NARROW) uniq[g] = (K)((long long)sorted[i] + lo);
      else uniq[g] = key_from_sort<K>(sorted[i]);
    }
  }
}

// ---------------------------------------------------------------- shuffle
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
__global__ __launch_bounds__(kT) void hash_kernel(const K* __restrict__ keys, int64_t n, uint64_t* __restrict__ h,
                                                  int accumulate) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    // the key image: equal keys (all NaNs, +-0) hash alike on every rank
    const uint64_t v = mix64((uint64_t)(int64_t)key_image<K>(keys[i]));
    h[i] = accumulate ? mix64(h[i] * 1000003ull ^ v) : v;
  }
}

// dest[i] = h[i] % world
__global__ __launch_bounds__(kT) void mod_kernel(const uint64_t* __restrict__ h, int64_t n, int64_t world,
                                                 int64_t* __restrict__ dest) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dest[i] = (int64_t)(h[i] % (uint64_t)world);
}

// rep[ids[i]] = i: any row of a group represents it (concurrent writers all
// store valid rows of the same group)
__global__ __launch_bounds__(kT) void rep_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t* __restrict__ rep) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) rep[ids[i]] = i;
}

// ---------------------------------------------------------------- segment CSR
// key = clamp(id, -1, nseg) + 1
template <typename I>
__global__ __launch_bounds__(kT) void seg_key_kernel(const I* __restrict__ ids, uint32_t* __restrict__ key, int64_t n,
                                                     int64_t nseg) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t v = (int64_t)ids[i];
    v = v < -1 ? -1 : (v > nseg ? nseg : v);
    key[i] = (uint32_t)(v + 1);
  }
}

// sorted keys are (segment + 1): offsets[g] = first position with segment >= g
__global__ __launch_bounds__(kT) void offsets_u32_kernel(const uint32_t* __restrict__ sorted, int64_t n, int64_t nseg,
                                                         int64_t* __restrict__ off) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
    const int64_t prev = i == 0 ? -1 : (int64_t)sorted[i - 1] - 1;
    const int64_t cur = i == n ? nseg : (int64_t)sorted[i] - 1;
    for (int64_t g = prev + 1; g <= cur; ++g) off[g] = i;
  }
}

// dest (int64 in [0, world)) -> uint32 sort key; counts[d] = rows with dest d
// (one LDS histogram per block, world <= 256)
__global__ __launch_bounds__(kT) void dest_key_hist_kernel(const int64_t* __restrict__ dest, int64_t n, int64_t world,
                                                           uint32_t* __restrict__ key,
                                                           unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t d = (uint32_t)dest[i];
    key[i] = d;
    atomicAdd(&h[d], 1u);
  }
  __syncthreads();
  if (threadIdx.x < world && h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

__global__ __launch_bounds__(kT) void zero_i64_kernel(int64_t* __restrict__ p, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0;
}

int bits_for(unsigned long long maxval) {
  int bits = 1;
  while (bits < 64 && (1ull << bits) <= maxval) ++bits;
  return bits;
}

// ---------------------------------------------------------------- factorize
// workspace layout (bytes): [0, 256) min/max + count cells, then the path's
// buffers. Sized for the widest path; the dense path takes it when its flag
// array fits in what the sort path would have used.
template <typename K>
size_t fact_ws_bytes(int64_t n) {
  using U = typename KeyImage<K>::U;
  const size_t cells = 256 + align_up(2 * kMinmaxBlocks * sizeof(long long));
  // sort path: sort keys (U), sorted keys (U), perm (u32), seg/head (u32), sort scratch
  const size_t sort = 2 * align_up(n * sizeof(U)) + 2 * align_up(n * sizeof(uint32_t)) +
                      std::max(radix::sort_ws_bytes<U, uint32_t>(n), radix::scan_ws_bytes<uint32_t>(n));
  return cells + sort;
}

template <typename K>
int64_t factorize_typed(const K* keys, int64_t n, int64_t* ids, K* uniq, void* ws, size_t ws_size, hipStream_t s) {
  using U = typename KeyImage<K>::U;
  char* base = static_cast<char*>(ws);
  long long* mm = reinterpret_cast<long long*>(base);           // [lo, hi, count]
  long long* part = reinterpret_cast<long long*>(base + 256);   // minmax partials
  char* p = base + 256 + align_up(2 * kMinmaxBlocks * sizeof(long long));
  const size_t avail = ws_size - static_cast<size_t>(p - base);
  const int grid = ew_grid(n);
  long long lo = 0;
  bool narrow = false;
  int nbits = int(sizeof(U) * 8);
  if constexpr (std::is_integral<K>::value) {
    const int nb = std::min(ew_grid(n), kMinmaxBlocks);
    hipLaunchKernelGGL((minmax_partial_kernel<K>), dim3(nb), dim3(kT), 0, s, keys, n, part);
    hipLaunchKernelGGL(minmax_final_kernel, dim3(1), dim3(kT), 0, s, (const long long*)part, nb, mm);
    long long got[2] = {0, 0};
    TFA_CHECK(hipMemcpyAsync(got, mm, sizeof(got), hipMemcpyDeviceToHost, s) == hipSuccess, "factorize: D2H failed");
    TFA_CHECK(hipStreamSynchronize(s) == hipSuccess, "factorize: sync failed");
    lo = got[0];
    const unsigned long long range = (unsigned long long)got[1] - (unsigned long long)got[0];
    // dense: flags + slots over range + 2 u32 entries, plus the scan scratch
    if (range < (1ull << 40) &&
        align_up((range + 2) * sizeof(uint32_t)) + radix::scan_ws_bytes<uint32_t>(range + 2) <= avail) {
      const int64_t r2 = (int64_t)range + 2;
      uint32_t* slot = reinterpret_cast<uint32_t*>(p);
      void* scan_ws = p + align_up(r2 * sizeof(uint32_t));
      hipLaunchKernelGGL(zero_u32_kernel, dim3(ew_grid(r2)), dim3(kT), 0, s, slot, r2);
      hipLaunchKernelGGL((dense_mark_kernel<K>), dim3(grid), dim3(kT), 0, s, keys, n, lo, slot);
      radix::scan<uint32_t>(slot, slot, r2, false, scan_ws, s);
      hipLaunchKernelGGL((dense_ids_kernel<K>), dim3(grid), dim3(kT), 0, s, keys, n, lo, (const uint32_t*)slot, ids);
      hipLaunchKernelGGL((dense_uniq_kernel<K>), dim3(ew_grid(r2 - 1)), dim3(kT), 0, s, (const uint32_t*)slot, r2 - 1,
                         lo, uniq);
      uint32_t count = 0;
      TFA_CHECK(hipMemcpyAsync(&count, slot + (r2 - 1), sizeof(count), hipMemcpyDeviceToHost, s) == hipSuccess,
                "factorize: D2H failed");
      TFA_CHECK(hipStreamSynchronize(s) == hipSuccess, "factorize: sync failed");
      return (int64_t)count;
    }
    if (range < (1ull << 32)) {
      narrow = true;
      nbits = bits_for(range);
    }
  }
  U* key = reinterpret_cast<U*>(p);
  p += align_up(n * sizeof(U));
  U* sorted = reinterpret_cast<U*>(p);
  p += align_up(n * sizeof(U));
  uint32_t* perm = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  uint32_t* seg = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  const size_t tmp = ws_size - static_cast<size_t>(p - base);
  if (narrow) {
    // key - lo fits 32 bits: the 32-bit buffers hold it
    uint32_t* k32 = reinterpret_cast<uint32_t*>(key);
    uint32_t* s32 = reinterpret_cast<uint32_t*>(sorted);
    hipLaunchKernelGGL((shift_kernel<K>), dim3(grid), dim3(kT), 0, s, keys, n, lo, k32);
    radix::sort_pairs<uint32_t, uint32_t>(k32, nullptr, s32, perm, n, nbits, p, tmp, s);
    hipLaunchKernelGGL((head_kernel<uint32_t>), dim3(grid), dim3(kT), 0, s, (const uint32_t*)s32, seg, n);
    radix::scan<uint32_t>(seg, seg, n, true, p, s);
    hipLaunchKernelGGL((scatter_ids_kernel<K, uint32_t, true>), dim3(grid), dim3(kT), 0, s, (const uint32_t*)s32,
                       (const uint32_t*)perm, (const uint32_t*)seg, ids, uniq, n, lo);
  } else {
    hipLaunchKernelGGL((sort_key_kernel<K>), dim3(grid), dim3(kT), 0, s, keys, n, key);
    radix::sort_pairs<U, uint32_t>(key, nullptr, sorted, perm, n, nbits, p, tmp, s);
    hipLaunchKernelGGL((head_kernel<U>), dim3(grid), dim3(kT), 0, s, (const U*)sorted, seg, n);
    radix::scan<uint32_t>(seg, seg, n, true, p, s);
    hipLaunchKernelGGL((scatter_ids_kernel<K, U, false>), dim3(grid), dim3(kT), 0, s, (const U*)sorted,
                       (const uint32_t*)perm, (const uint32_t*)seg, ids, uniq, n, 0ll);
  }
  uint32_t count = 0;
  TFA_CHECK(hipMemcpyAsync(&count, seg + (n - 1), sizeof(count), hipMemcpyDeviceToHost, s) == hipSuccess,
            "factorize: D2H failed");
  TFA_CHECK(hipStreamSynchronize(s) == hipSuccess, "factorize: sync failed");
  return (int64_t)count;
}

// idx[g * size + j] = perm[offs[g] + j]: the rows of G equal-size segments
__global__ __launch_bounds__(kT) void segment_rows_kernel(const int64_t* __restrict__ perm,
                                                          const int64_t* __restrict__ offs, int64_t G, int64_t size,
                                                          int64_t* __restrict__ idx) {
  const int64_t n = G * size;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t g = i / size;
    idx[i] = perm[offs[g] + (i - g * size)];
  }
}

// dst row idx[j] = src row j, rows of `words` W-sized words
template <typename W>
__global__ __launch_bounds__(kT) void scatter_rows_kernel(const W* __restrict__ src, const int64_t* __restrict__ idx,
                                                          W* __restrict__ dst, int64_t nidx, int64_t words) {
  const int64_t n = nidx * words;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t j = i / words, w = i - j * words;
    dst[idx[j] * words + w] = src[i];
  }
}

// Row packing for the keyed shuffle: the columns of a row, each in a
// word-aligned slot of one R-byte record, so ONE all-to-all moves them all.
template <typename W>
__global__ __launch_bounds__(kT) void pack_rows_kernel(PackCols pc, const int64_t* __restrict__ perm, int64_t nrows,
                                                       int64_t rwords, W* __restrict__ out) {
  const int64_t n = nrows * rwords;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t j = i / rwords, w = i - j * rwords;
    int c = 0;
    while (c + 1 < pc.n && w >= pc.off[c + 1] / (int64_t)sizeof(W)) ++c;
    const int64_t cw = w - pc.off[c] / (int64_t)sizeof(W), cwords = pc.row_bytes[c] / (int64_t)sizeof(W);
    const int64_t src_row = perm ? perm[j] : j;
    out[i] = cw < cwords ? static_cast<const W*>(pc.ptr[c])[src_row * cwords + cw] : W(0);
  }
}

template <typename W>
__global__ __launch_bounds__(kT) void unpack_rows_kernel(PackCols pc, const W* __restrict__ in, int64_t nrows,
                                                         int64_t rwords) {
  const int64_t n = nrows * rwords;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t j = i / rwords, w = i - j * rwords;
    int c = 0;
    while (c + 1 < pc.n && w >= pc.off[c + 1] / (int64_t)sizeof(W)) ++c;
    const int64_t cw = w - pc.off[c] / (int64_t)sizeof(W), cwords = pc.row_bytes[c] / (int64_t)sizeof(W);
    if (cw < cwords) static_cast<W*>(const_cast<void*>(pc.ptr[c]))[j * cwords + cw] = in[i];
  }
}

}  // namespace

size_t factorize_workspace_bytes(DType dt, int64_t n) {
  switch (dt) {
    case DType::I32: return fact_ws_bytes<int32_t>(n);
    case DType::I64: return fact_ws_bytes<int64_t>(n);
    case DType::F32: return fact_ws_bytes<float>(n);
    case DType::F64: return fact_ws_bytes<double>(n);
    default: TFA_CHECK(false, "factorize: unsupported key dtype ", dtype_name(dt));
  }
  return 0;
}

int64_t factorize(DType dt, const void* keys, int64_t n, int64_t* ids, void* uniq, void* ws, size_t ws_size,
                  hipStream_t s) {
  TFA_CHECK(n > 0, "factorize: empty key column");
  TFA_CHECK(n < (int64_t(1) << 31), "factorize: more than 2^31 keys in one block");
  TFA_CHECK(ws_size >= factorize_workspace_bytes(dt, n), "factorize: workspace too small");
  int64_t nseg = 0;
  switch (dt) {
    case DType::I32: nseg = factorize_typed<int32_t>((const int32_t*)keys, n, ids, (int32_t*)uniq, ws, ws_size, s); break;
    case DType::I64: nseg = factorize_typed<int64_t>((const int64_t*)keys, n, ids, (int64_t*)uniq, ws, ws_size, s); break;
    case DType::F32: nseg = factorize_typed<float>((const float*)keys, n, ids, (float*)uniq, ws, ws_size, s); break;
    case DType::F64: nseg = factorize_typed<double>((const double*)keys, n, ids, (double*)uniq, ws, ws_size, s); break;
    default: TFA_CHECK(false, "factorize: unsupported key dtype ", dtype_name(dt));
  }
  TFA_LAUNCH_CHECK("factorize");
  return nseg;
}

void key_hash(DType dt, const void* keys, int64_t n, uint64_t* h, bool accumulate, hipStream_t s) {
  if (n == 0) return;
  const int grid = ew_grid(n);
  const int acc = accumulate ? 1 : 0;
  switch (dt) {
    case DType::I32: hipLaunchKernelGGL((hash_kernel<int32_t>), dim3(grid), dim3(kT), 0, s, (const int32_t*)keys, n, h, acc); break;
    case DType::I64: hipLaunchKernelGGL((hash_kernel<int64_t>), dim3(grid), dim3(kT), 0, s, (const int64_t*)keys, n, h, acc); break;
    case DType::F32: hipLaunchKernelGGL((hash_kernel<float>), dim3(grid), dim3(kT), 0, s, (const float*)keys, n, h, acc); break;
    case DType::F64: hipLaunchKernelGGL((hash_kernel<double>), dim3(grid), dim3(kT), 0, s, (const double*)keys, n, h, acc); break;
    default: TFA_CHECK(false, "key_hash: unsupported key dtype ", dtype_name(dt));
  }
}

size_t segment_csr_workspace_bytes(int64_t n, int64_t nseg) {
  (void)nseg;
  return 2 * align_up(n * sizeof(uint32_t)) + radix::sort_ws_bytes<uint32_t, int64_t>(n);
}

void segment_csr(DType idt, const void* ids, int64_t n, int64_t nseg, int64_t* perm, int64_t* offsets, void* ws,
                 size_t ws_size, hipStream_t s) {
  TFA_CHECK(idt == DType::I32 || idt == DType::I64, "segment_csr: int32/int64 ids");
  TFA_CHECK(nseg + 2 < (int64_t(1) << 32), "segment_csr: too many segments");
  TFA_CHECK(ws_size >= segment_csr_workspace_bytes(n, nseg), "segment_csr: workspace too small");
  if (n == 0) {
    hipLaunchKernelGGL(zero_i64_kernel, dim3(ew_grid(nseg + 1)), dim3(kT), 0, s, offsets, nseg + 1);
    return;
  }
  char* p = static_cast<char*>(ws);
  uint32_t* key = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  uint32_t* sorted = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  const size_t tmp = ws_size - static_cast<size_t>(p - static_cast<char*>(ws));
  const int grid = ew_grid(n + 1);
  // key = clamp(id, -1, nseg) + 1: only the bits of [0, nseg + 1] are sorted
  if (idt == DType::I32)
    hipLaunchKernelGGL((seg_key_kernel<int32_t>), dim3(grid), dim3(kT), 0, s, static_cast<const int32_t*>(ids), key, n, nseg);
  else
    hipLaunchKernelGGL((seg_key_kernel<int64_t>), dim3(grid), dim3(kT), 0, s, static_cast<const int64_t*>(ids), key, n, nseg);
  radix::sort_pairs<uint32_t, int64_t>(key, nullptr, sorted, perm, n, bits_for((unsigned long long)nseg + 1), p, tmp, s);
  hipLaunchKernelGGL(offsets_u32_kernel, dim3(grid), dim3(kT), 0, s, (const uint32_t*)sorted, n, nseg, offsets);
  TFA_LAUNCH_CHECK("segment_csr");
}

void group_representatives(const int64_t* ids, int64_t n, int64_t* rep, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(rep_kernel, dim3(ew_grid(n)), dim3(kT), 0, s, ids, n, rep);
}

size_t partition_workspace_bytes(int64_t n) {
  return 2 * align_up(n * sizeof(uint32_t)) + radix::sort_ws_bytes<uint32_t, int64_t>(n);
}

void partition_rows(const int64_t* dest, int64_t n, int64_t world, int64_t* perm, int64_t* counts, void* ws,
                    size_t ws_size, hipStream_t s) {
  TFA_CHECK(world >= 1 && world <= 256, "partition_rows: world must be in [1, 256]");
  TFA_CHECK(ws_size >= partition_workspace_bytes(n), "partition_rows: workspace too small");
  hipLaunchKernelGGL(zero_i64_kernel, dim3(1), dim3(kT), 0, s, counts, world);
  if (n == 0) return;
  char* p = static_cast<char*>(ws);
  uint32_t* key = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  uint32_t* sorted = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * sizeof(uint32_t));
  const size_t tmp = ws_size - static_cast<size_t>(p - static_cast<char*>(ws));
  hipLaunchKernelGGL(dest_key_hist_kernel, dim3(std::min(ew_grid(n), 1024)), dim3(kT), 0, s, dest, n, world, key,
                     reinterpret_cast<unsigned long long*>(counts));
  // stable: rows keep their order within a destination
  radix::sort_pairs<uint32_t, int64_t>(key, nullptr, sorted, perm, n, bits_for((unsigned long long)world - 1), p, tmp, s);
  TFA_LAUNCH_CHECK("partition_rows");
}

void segment_rows(const int64_t* perm, const int64_t* offs, int64_t G, int64_t size, int64_t* idx, hipStream_t s) {
  if (G * size == 0) return;
  hipLaunchKernelGGL(segment_rows_kernel, dim3(ew_grid(G * size)), dim3(kT), 0, s, perm, offs, G, size, idx);
  TFA_LAUNCH_CHECK("segment_rows");
}

void scatter_rows(int64_t row_bytes, const void* src, const int64_t* idx, void* dst, int64_t nidx, hipStream_t s) {
  if (nidx * row_bytes == 0) return;
  const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst);
  if (row_bytes % 8 == 0 && al % 8 == 0)
    hipLaunchKernelGGL((scatter_rows_kernel<uint64_t>), dim3(ew_grid(nidx * row_bytes / 8)), dim3(kT), 0, s,
                       (const uint64_t*)src, idx, (uint64_t*)dst, nidx, row_bytes / 8);
  else if (row_bytes % 4 == 0 && al % 4 == 0)
    hipLaunchKernelGGL((scatter_rows_kernel<uint32_t>), dim3(ew_grid(nidx * row_bytes / 4)), dim3(kT), 0, s,
                       (const uint32_t*)src, idx, (uint32_t*)dst, nidx, row_bytes / 4);
  else
    hipLaunchKernelGGL((scatter_rows_kernel<uint8_t>), dim3(ew_grid(nidx * row_bytes)), dim3(kT), 0, s,
                       (const uint8_t*)src, idx, (uint8_t*)dst, nidx, row_bytes);
  TFA_LAUNCH_CHECK("scatter_rows");
}

static bool pack_words4(const PackCols& pc) {
  for (int c = 0; c < pc.n; ++c)
    if (pc.row_bytes[c] % 4 || pc.off[c] % 4 || reinterpret_cast<uintptr_t>(pc.ptr[c]) % 4) return false;
  return true;
}

void pack_rows(const PackCols& pc, const int64_t* perm, int64_t nrows, int64_t record_bytes, void* out,
               hipStream_t s) {
  TFA_CHECK(pc.n >= 1 && pc.n <= kMaxPackCols, "pack_rows: 1..", kMaxPackCols, " columns");
  if (nrows == 0) return;
  if (pack_words4(pc) && record_bytes % 4 == 0)
    hipLaunchKernelGGL((pack_rows_kernel<uint32_t>), dim3(ew_grid(nrows * record_bytes / 4)), dim3(kT), 0, s, pc, perm,
                       nrows, record_bytes / 4, (uint32_t*)out);
  else
    hipLaunchKernelGGL((pack_rows_kernel<uint8_t>), dim3(ew_grid(nrows * record_bytes)), dim3(kT), 0, s, pc, perm,
                       nrows, record_bytes, (uint8_t*)out);
  TFA_LAUNCH_CHECK("pack_rows");
}

void unpack_rows(const PackCols& pc, const void* in, int64_t nrows, int64_t record_bytes, hipStream_t s) {
  TFA_CHECK(pc.n >= 1 && pc.n <= kMaxPackCols, "unpack_rows: 1..", kMaxPackCols, " columns");
  if (nrows == 0) return;
  if (pack_words4(pc) && record_bytes % 4 == 0)
    hipLaunchKernelGGL((unpack_rows_kernel<uint32_t>), dim3(ew_grid(nrows * record_bytes / 4)), dim3(kT), 0, s, pc,
                       (const uint32_t*)in, nrows, record_bytes / 4);
  else
    hipLaunchKernelGGL((unpack_rows_kernel<uint8_t>), dim3(ew_grid(nrows * record_bytes)), dim3(kT), 0, s, pc,
                       (const uint8_t*)in, nrows, record_bytes);
  TFA_LAUNCH_CHECK("unpack_rows");
}

// ---- string keys: the bytes of every row packed into W big-endian 64-bit
// words (zero padded) with the sign bit flipped, plus the byte length. Signed
// comparison of (word 0, ..., word W-1, length) is then the lexicographic
// order of the byte strings, so the numeric groupBy kernels group string keys
// exactly (no hashing, no collisions) and in sorted order. One thread per
// (row, word); the output is column-major [W + 1][n] (contiguous key columns).
__global__ __launch_bounds__(kT) void string_words_kernel(const int64_t* __restrict__ offs,
                                                          const uint8_t* __restrict__ data, int64_t n, int W,
                                                          int64_t* __restrict__ out) {
  const int64_t total = n * (W + 1);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(t / n);
    const int64_t i = t - (int64_t)w * n;
    const int64_t a = offs[i], len = offs[i + 1] - a;
    if (w == W) {
      out[t] = len;
      continue;
    }
    uint64_t v = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int64_t j = (int64_t)w * 8 + b;
      const uint64_t byte = j < len ? data[a + j] : 0;
      v |= byte << (56 - 8 * b);
    }
    out[t] = (int64_t)(v ^ 0x8000000000000000ull);
  }
}

void string_words(const int64_t* offs, const uint8_t* data, int64_t n, int W, int64_t* out, hipStream_t s) {
  TFA_CHECK(W >= 1 && n >= 0, "string_words: bad shape");
  if (n == 0) return;
  hipLaunchKernelGGL(string_words_kernel, dim3(ew_grid(n * (W + 1))), dim3(kT), 0, s, offs, data, n, W, out);
  TFA_LAUNCH_CHECK("string_words");
}

// ---- bounded-width string keys: (word 0, tag) per row, 2 words whatever
// the longest key. tag = length for keys of <= 8 bytes (exact: word 0 holds
// all their bytes), 9 + a 62-bit hash of all the bytes (and the length) for
// longer ones, so a long key sorts after the short key that is its 8-byte
// prefix. Groups are verified against one representative row each
// (string_verify); only prefix ties among long keys need an exact re-order
// (ops/groupby.py).
__host__ __device__ inline uint64_t skey_hash(const uint8_t* p, int64_t len) {
  uint64_t h = 0x243F6A8885A308D3ull ^ (static_cast<uint64_t>(len) * 0x9E3779B97F4A7C15ull);
  for (int64_t j = 0; j < len; j += 8) {
    uint64_t k = 0;
    const int64_t m = len - j < 8 ? len - j : 8;
    for (int64_t b = 0; b < m; ++b) k |= static_cast<uint64_t>(p[j + b]) << (8 * b);
    h ^= k * 0xBF58476D1CE4E5B9ull;
    h = ((h << 27) | (h >> 37)) * 0x94D049BB133111EBull + 0x2545F4914F6CDD1Dull;
  }
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return (h >> 2) + 1;
}

__global__ __launch_bounds__(kT) void string_key_hash_kernel(const int64_t* __restrict__ offs,
                                                             const uint8_t* __restrict__ data, int64_t n,
                                                             int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = offs[i], len = offs[i + 1] - a;
    uint64_t v = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) v |= static_cast<uint64_t>(b < len ? data[a + b] : 0) << (56 - 8 * b);
    out[i] = static_cast<int64_t>(v ^ 0x8000000000000000ull);
    out[n + i] = len > 8 ? static_cast<int64_t>(skey_hash(data + a, len) + 9) : len;
  }
}

// flag <- 1 when a row's bytes differ from its group representative's (a
// hash collision); rows of <= 8 bytes are exact by construction
__global__ __launch_bounds__(kT) void string_verify_kernel(const int64_t* __restrict__ offs,
                                                           const uint8_t* __restrict__ data,
                                                           const int64_t* __restrict__ ids,
                                                           const int64_t* __restrict__ rep, int64_t n,
                                                           int* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = offs[i], len = offs[i + 1] - a;
    if (len <= 8) continue;
    const int64_t r = rep[ids[i]];
    if (r == i) continue;
    const int64_t ra = offs[r];
    bool diff = offs[r + 1] - ra != len;
    for (int64_t j = 8; j < len && !diff; ++j) diff = data[a + j] != data[ra + j];
    if (diff) flag[0] = 1;
  }
}

void string_key_hash(const int64_t* offs, const uint8_t* data, int64_t n, int64_t* out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(string_key_hash_kernel, dim3(ew_grid(n)), dim3(kT), 0, s, offs, data, n, out);
  TFA_LAUNCH_CHECK("string_key_hash");
}

void string_verify(const int64_t* offs, const uint8_t* data, const int64_t* ids, const int64_t* rep, int64_t n,
                   int* flag, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(string_verify_kernel, dim3(ew_grid(n)), dim3(kT), 0, s, offs, data, ids, rep, n, flag);
  TFA_LAUNCH_CHECK("string_verify");
}

uint64_t string_key_hash_host(const uint8_t* p, int64_t len) { return skey_hash(p, len); }

// rows idx of a string column: one block per output string (block-stride)
__global__ __launch_bounds__(kT) void gather_bytes_kernel(const uint8_t* __restrict__ data,
                                                          const int64_t* __restrict__ offs,
                                                          const int64_t* __restrict__ idx,
                                                          const int64_t* __restrict__ new_offs, int64_t n,
                                                          uint8_t* __restrict__ out) {
  for (int64_t g = blockIdx.x; g < n; g += gridDim.x) {
    const int64_t a = offs[idx[g]], len = offs[idx[g] + 1] - a, o = new_offs[g];
    for (int64_t j = threadIdx.x; j < len; j += blockDim.x) out[o + j] = data[a + j];
  }
}

__global__ __launch_bounds__(kT) void string_lens_kernel(const int64_t* __restrict__ offs,
                                                         const int64_t* __restrict__ idx, int64_t n,
                                                         int64_t* __restrict__ lens) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x)
    lens[g] = offs[idx[g] + 1] - offs[idx[g]];
}

void string_lens(const int64_t* offs, const int64_t* idx, int64_t n, int64_t* lens, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(string_lens_kernel, dim3(ew_grid(n)), dim3(kT), 0, s, offs, idx, n, lens);
  TFA_LAUNCH_CHECK("string_lens");
}

void gather_bytes(const uint8_t* data, const int64_t* offs, const int64_t* idx, const int64_t* new_offs, int64_t n,
                  uint8_t* out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(gather_bytes_kernel, dim3(static_cast<int>(std::min<int64_t>(n, 65536))), dim3(kT), 0, s, data,
                     offs, idx, new_offs, n, out);
  TFA_LAUNCH_CHECK("gather_bytes");
}


void hash_mod(const uint64_t* h, int64_t n, int64_t world, int64_t* dest, hipStream_t s) {
  if (n == 0) return;
  TFA_CHECK(world >= 1, "hash_mod: world must be >= 1");
  hipLaunchKernelGGL(mod_kernel, dim3(ew_grid(n)), dim3(kT), 0, s, h, n, world, dest);
}

}  // namespace k
}  // namespace tfa

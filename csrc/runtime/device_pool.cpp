// Engine-owned stream-ordered device memory (see device_pool.h).
//
// SURVEY C5(c) asks for a device tensor type with a stream-ordered allocator
// on HBM owned by the engine (the reference's libtensorflow owned its BFC
// allocator). Executor buffers (step outputs, GEMM/conv/reduce workspaces,
// pipeline rings, HIP-graph replay outputs) come from this caching pool:
// blocks of 4-per-octave size classes are hipMalloc'ed once and cached per
// (device, stream); a released block is reused by the next allocation on the
// SAME stream (stream order makes that safe with no event), and a block used
// on other streams (dev_record_stream: the pipeline's copy streams) waits in a
// pending list until events recorded on those streams complete. Memory stays
// cached (288 GB of HBM per GPU are the engine's); an allocation that fails
// frees the cache once and retries. The tensors are at::Tensor views
// (at::from_blob), so kernels, DLPack and test oracles see ordinary device
// tensors. (The driver's hipMemPool, tried first, cost ~40 us per
// allocate/free pair on this stack: 2x the K-Means iteration time.)
#include "device_pool.h"

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../common.h"

namespace tfa {
namespace {

// size classes: 4 per power of two (at most 25 % padding), 512 B minimum
size_t size_class(size_t bytes) {
  if (bytes <= 512) return 512;
  int lg = 63 - __builtin_clzll(bytes - 1);  // bytes in (2^lg, 2^(lg+1)]
  const size_t step = size_t(1) << (lg >= 2 ? lg - 2 : 0);
  return (bytes + step - 1) / step * step;
}

struct Block {
  void* p = nullptr;
  int device = 0;
  hipStream_t stream = nullptr;
  size_t size = 0;                 // class size (what hipMalloc returned)
  std::vector<hipStream_t> also;   // other streams the tensor was used on
};

struct Pending {
  Block* b;
  std::vector<hipEvent_t> events;
};

struct State {
  std::mutex mu;
  // cached blocks per (device, stream), by class size
  std::map<std::pair<int, hipStream_t>, std::multimap<size_t, Block*>> free;
  std::vector<Pending> pending;  // released, waiting for other streams
  std::unordered_map<void*, Block*> live;
  size_t cached = 0;
};

State& st() {
  static State* s = new State();  // never destroyed: tensors may die after static teardown
  return *s;
}
std::atomic<int64_t> g_allocs{0}, g_frees{0}, g_fallbacks{0}, g_live{0}, g_peak{0}, g_device_mallocs{0};
// allocations made while one of the engine's HIP graphs captures their stream:
// they belong to the graph (its private memory pool), not to this pool, and
// are counted apart from the fallbacks (pool disabled / out of memory)
std::atomic<int64_t> g_capture_allocs{0};

// streams being captured by the engine's own HIP graphs (HipGraph::begin /
// end report them): the common case, no capture anywhere, costs one atomic
// load instead of a runtime query per allocation
std::atomic<int> g_captures{0};
std::mutex g_cap_mu;
std::vector<hipStream_t>& cap_streams() {
  static auto* v = new std::vector<hipStream_t>();
  return *v;
}

bool capturing(hipStream_t s) {
  if (g_captures.load(std::memory_order_acquire) == 0) return false;
  std::lock_guard<std::mutex> lk(g_cap_mu);
  const auto& v = cap_streams();
  return std::find(v.begin(), v.end(), s) != v.end();
}

// caller holds the lock: move released blocks whose other-stream work is done
void drain_pending(State& S) {
  for (size_t i = 0; i < S.pending.size();) {
    bool done = true;
    for (hipEvent_t e : S.pending[i].events) {
      hipError_t q = hipEventQuery(e);
      if (q == hipErrorNotReady) {
        done = false;
        break;
      }
    }
    if (!done) {
      ++i;
      continue;
    }
    for (hipEvent_t e : S.pending[i].events) (void)hipEventDestroy(e);
    Block* b = S.pending[i].b;
    b->also.clear();
    S.free[{b->device, b->stream}].emplace(b->size, b);
    S.cached += b->size;
    S.pending[i] = S.pending.back();
    S.pending.pop_back();
  }
  (void)hipGetLastError();
}

// caller holds the lock: hipFree every cached block of `device` (after the
// device's queued work), to make room
void trim_device(State& S, int device) {
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != device) (void)hipSetDevice(device);
  (void)hipDeviceSynchronize();
  for (auto it = S.free.begin(); it != S.free.end(); ++it) {
    if (it->first.first != device) continue;
    for (auto& kv : it->second) {
      (void)hipFree(kv.second->p);
      S.cached -= kv.second->size;
      delete kv.second;
    }
    it->second.clear();
  }
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
}

// best fit: the smallest cached block of at least `want` bytes, if it wastes
// at most half of `want` (a neighbouring size class serves a request instead
// of a fresh hipMalloc: chunk tails and ragged batches vary in size)
Block* take_best_fit(State& S, int device, hipStream_t stream, size_t want) {
  auto fit = S.free.find({device, stream});
  if (fit == S.free.end()) return nullptr;
  auto it = fit->second.lower_bound(want);
  if (it == fit->second.end() || it->first > want + want / 2) return nullptr;
  Block* b = it->second;
  fit->second.erase(it);
  S.cached -= b->size;
  return b;
}

void release(Block* b) {
  State& S = st();
  std::lock_guard<std::mutex> lk(S.mu);
  S.live.erase(b->p);
  g_frees++;
  g_live -= static_cast<int64_t>(b->size);
  if (b->also.empty()) {
    // stream-ordered reuse: the next allocation on b->stream runs after every
    // use already queued there
    S.free[{b->device, b->stream}].emplace(b->size, b);
    S.cached += b->size;
    return;
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != b->device) (void)hipSetDevice(b->device);
  Pending pd{b, {}};
  for (hipStream_t s : b->also) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
      (void)hipEventRecord(e, s);
      pd.events.push_back(e);
    }
  }
  if (prev >= 0 && prev != b->device) (void)hipSetDevice(prev);
  S.pending.push_back(std::move(pd));
}

}  // namespace

bool dev_stream_capturing(hipStream_t s) { return capturing(s); }

void dev_capture_begin(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_cap_mu);
  cap_streams().push_back(s);
  g_captures.fetch_add(1, std::memory_order_release);
}

void dev_capture_end(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_cap_mu);
  auto& v = cap_streams();
  auto it = std::find(v.begin(), v.end(), s);
  if (it != v.end()) {
    v.erase(it);
    g_captures.fetch_sub(1, std::memory_order_release);
  }
}

bool dev_pool_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TFA_DEVICE_POOL");
    return !(e && e[0] == '0');
  }();
  return on;
}

at::Tensor dev_empty(at::IntArrayRef sizes, at::ScalarType dt, const at::Device& dev, hipStream_t stream) {
  auto opts = at::TensorOptions().dtype(dt).device(dev);
  if (dev.is_cuda() && dev_pool_enabled() && capturing(stream)) {
    g_capture_allocs++;
    return at::empty(sizes, opts);
  }
  if (!dev.is_cuda() || !dev_pool_enabled()) {
    if (dev.is_cuda()) g_fallbacks++;
    return at::empty(sizes, opts);
  }
  dev_pool_install_oom_hook();  // once; the framework allocator is initialised by now
  int64_t n = 1;
  for (int64_t s : sizes) n *= s;
  const size_t want = size_class(static_cast<size_t>(std::max<int64_t>(n, 1)) * c10::elementSize(dt));
  State& S = st();
  Block* b = nullptr;
  {
    std::unique_lock<std::mutex> lk(S.mu);
    if (!S.pending.empty()) drain_pending(S);
    b = take_best_fit(S, dev.index(), stream, want);
    if (!b) {
      void* p = nullptr;
      hipError_t e = hipMalloc(&p, want);
      if (e != hipSuccess) {
        // out of memory: give back our own cache, then the framework
        // allocator's (outside our lock: c10's OOM observer takes it), and
        // retry once
        (void)hipGetLastError();
        trim_device(S, dev.index());
        lk.unlock();
        c10::hip::HIPCachingAllocator::emptyCache();
        lk.lock();
        e = hipMalloc(&p, want);
      }
      if (e != hipSuccess || !p) {
        (void)hipGetLastError();
        g_fallbacks++;
        // out of device memory here: the framework allocator's turn. Drop our
        // lock first: if it is out of memory too, c10 runs the OOM observer
        // (dev_pool_install_oom_hook), which takes S.mu on this same thread,
        // and then raises OutOfMemoryError instead of deadlocking.
        lk.unlock();
        return at::empty(sizes, opts);
      }
      g_device_mallocs++;
      b = new Block{p, dev.index(), stream, want, {}};
    }
    S.live[b->p] = b;
  }
  g_allocs++;
  const int64_t now = (g_live += static_cast<int64_t>(b->size));
  int64_t pk = g_peak.load();
  while (now > pk && !g_peak.compare_exchange_weak(pk, now)) {
  }
  return at::from_blob(b->p, sizes, [b](void*) { release(b); }, opts);
}

at::Tensor dev_empty_like(const at::Tensor& t, hipStream_t stream) {
  return dev_empty(t.sizes(), t.scalar_type(), t.device(), stream);
}

void dev_record_stream(const at::Tensor& t, hipStream_t s) {
  void* p = t.storage().data_ptr().get();
  {
    State& S = st();
    std::lock_guard<std::mutex> lk(S.mu);
    auto it = S.live.find(p);
    if (it != S.live.end()) {
      Block* b = it->second;
      if (b->stream != s && std::find(b->also.begin(), b->also.end(), s) == b->also.end()) b->also.push_back(s);
      return;
    }
  }
  // an alias of a HIP graph's output buffer: the next replay waits for `s`
  if (replay_alias_record_stream(p, s)) return;
  // not ours: the framework allocator tracks it
  c10::hip::HIPCachingAllocator::recordStream(
      t.storage().data_ptr(), c10::hip::getStreamFromExternal(s, t.device().index()));
}

at::Tensor dev_clone(const at::Tensor& t, hipStream_t stream) {
  TFA_CHECK(t.is_cuda() && t.is_contiguous(), "dev_clone: contiguous device tensor expected");
  at::Tensor o = dev_empty(t.sizes(), t.scalar_type(), t.device(), stream);
  const size_t nb = t.numel() * t.element_size();
  if (nb) TFA_CHECK(hipMemcpyAsync(o.data_ptr(), t.data_ptr(), nb, hipMemcpyDeviceToDevice, stream) == hipSuccess,
                    "dev_clone: hipMemcpyAsync failed");
  return o;
}

at::Tensor pool_empty(at::IntArrayRef sizes, const at::TensorOptions& opts) {
  if (!opts.device().is_cuda()) return at::empty(sizes, opts);
  const int d = opts.device().has_index() ? opts.device().index() : c10::hip::current_device();
  at::Device dev(at::kCUDA, static_cast<c10::DeviceIndex>(d));
  return dev_empty(sizes, opts.dtype().toScalarType(), dev, c10::hip::getCurrentHIPStream(d).stream());
}

at::Tensor pool_empty_like(const at::Tensor& t) { return pool_empty(t.sizes(), t.options()); }

at::Tensor pool_zeros(at::IntArrayRef sizes, const at::TensorOptions& opts) {
  at::Tensor t = pool_empty(sizes, opts);
  if (t.is_cuda()) {
    const size_t nb = t.numel() * t.element_size();
    if (nb) TFA_CHECK(hipMemsetAsync(t.data_ptr(), 0, nb, c10::hip::getCurrentHIPStream(t.device().index()).stream()) ==
                          hipSuccess, "pool_zeros: hipMemsetAsync failed");
    return t;
  }
  return t.zero_();
}

void dev_pool_install_oom_hook() {
  static std::once_flag once;
  std::call_once(once, [] {
    // c10 calls observers before it raises OutOfMemoryError: hand our cached
    // blocks back so the caller's retry (or the next allocation) finds room
    c10::hip::HIPCachingAllocator::attachOutOfMemoryObserver(
        [](int64_t device, size_t, size_t, size_t) {
          State& S = st();
          std::lock_guard<std::mutex> lk(S.mu);
          trim_device(S, static_cast<int>(device));
        });
  });
}

DevPoolStats dev_pool_stats() {
  DevPoolStats s;
  s.allocs = g_allocs.load();
  s.frees = g_frees.load();
  s.fallbacks = g_fallbacks.load();
  s.capture_allocs = g_capture_allocs.load();
  s.live_bytes = g_live.load();
  s.peak_bytes = g_peak.load();
  s.device_mallocs = g_device_mallocs.load();
  {
    std::lock_guard<std::mutex> lk(st().mu);
    s.cached_bytes = static_cast<int64_t>(st().cached);
  }
  return s;
}

void dev_pool_trim() {
  State& S = st();
  std::lock_guard<std::mutex> lk(S.mu);
  int n = 0;
  (void)hipGetDeviceCount(&n);
  for (int d = 0; d < n; ++d) trim_device(S, d);
}

}  // namespace tfa

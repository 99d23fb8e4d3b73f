// Engine-owned device memory: a stream-ordered pool on HBM.
#pragma once

#include <torch/extension.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tfa {

// Uninitialised contiguous device tensor whose memory comes from the
// engine's own stream-ordered caching pool. Its lifetime is ordered on
// `stream`: when the last reference dies the block is reused by later
// allocations on `stream` (after the work already queued there), or, if it
// was recorded on other streams (dev_record_stream), only once their work
// queued so far has finished. During a HIP-graph capture on `stream` the
// tensor comes from the capture's private pool instead (graph-owned memory
// must outlive every replay).
at::Tensor dev_empty(at::IntArrayRef sizes, at::ScalarType dt, const at::Device& dev, hipStream_t stream);
at::Tensor dev_empty_like(const at::Tensor& t, hipStream_t stream);
// `t` (any device tensor) is also used on `s`: its memory is not reused
// before s's work queued so far has finished
void dev_record_stream(const at::Tensor& t, hipStream_t s);
// the executor's hook for memory it hands out that is neither the pool's nor
// c10's to recycle (aliases of a HIP graph's output buffers): returns true
// when `p` is such memory and the use on `s` was recorded (executor.cpp)
bool replay_alias_record_stream(const void* p, hipStream_t s);
// D2D copy of a contiguous tensor into fresh pool memory (hipMemcpyAsync)
at::Tensor dev_clone(const at::Tensor& t, hipStream_t stream);
// at::empty for op temporaries: device tensors come from the pool, ordered
// on the device's CURRENT HIP stream (where the calling op launches); host
// tensors from at::empty
at::Tensor pool_empty(at::IntArrayRef sizes, const at::TensorOptions& opts);
at::Tensor pool_empty_like(const at::Tensor& t);
at::Tensor pool_zeros(at::IntArrayRef sizes, const at::TensorOptions& opts);

struct DevPoolStats {
  int64_t allocs = 0, frees = 0, fallbacks = 0, device_mallocs = 0, capture_allocs = 0;
  int64_t live_bytes = 0, peak_bytes = 0, cached_bytes = 0;
};
DevPoolStats dev_pool_stats();
void dev_pool_trim();  // hipFree every cached block (after a device sync)
// hooks the framework allocator's out-of-memory path: when c10 runs out of
// device memory it first gets the pool's cached blocks back (idempotent)
void dev_pool_install_oom_hook();
// the engine's HIP-graph capture on `s` starts / ends: allocations on a
// capturing stream go to the capture's private (framework) pool
void dev_capture_begin(hipStream_t s);
void dev_capture_end(hipStream_t s);
bool dev_stream_capturing(hipStream_t s);  // inside the engine's own capture on `s`
bool dev_pool_enabled();  // TFA_DEVICE_POOL=0: every allocation goes to c10

}  // namespace tfa

// HIP graph capture / replay (see hip_graph.h).
#include "hip_graph.h"

#include <c10/hip/HIPCachingAllocator.h>

#include <atomic>

#include "../common.h"
#include "device_pool.h"

namespace tfa {
namespace {

// pool ids of our graphs: first element far above the ids the framework hands out
std::pair<unsigned long long, unsigned long long> next_pool() {
  static std::atomic<unsigned long long> k{0};
  return {(1ull << 62) + k.fetch_add(1), 0ull};
}

}  // namespace

void HipGraph::begin(hipStream_t stream, int device) {
  TFA_CHECK(!exec_ && !pool_open_, "HipGraph: already captured");
  stream_ = stream;
  device_ = device;
  pool_ = next_pool();
  // allocations made on the capturing stream go to the graph's private pool
  c10::hip::HIPCachingAllocator::get()->beginAllocateToPool(
      static_cast<c10::DeviceIndex>(device), pool_, [stream](hipStream_t s) { return s == stream; });
  pool_open_ = pool_owned_ = true;
  dev_capture_begin(stream);
  hipError_t e = hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    dev_capture_end(stream);
    c10::hip::HIPCachingAllocator::get()->endAllocateToPool(static_cast<c10::DeviceIndex>(device), pool_);
    pool_open_ = false;
    TFA_CHECK(false, "hipStreamBeginCapture failed: ", hipGetErrorString(e));
  }
}

void HipGraph::end() {
  hipError_t e = hipStreamEndCapture(stream_, &graph_);
  dev_capture_end(stream_);
  c10::hip::HIPCachingAllocator::get()->endAllocateToPool(static_cast<c10::DeviceIndex>(device_), pool_);
  pool_open_ = false;
  TFA_CHECK(e == hipSuccess && graph_ != nullptr, "hipStreamEndCapture failed: ", hipGetErrorString(e));
  e = hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0);
  TFA_CHECK(e == hipSuccess, "hipGraphInstantiate failed: ", hipGetErrorString(e));
}

void HipGraph::abort() {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (stream_ && hipStreamIsCapturing(stream_, &st) == hipSuccess && st != hipStreamCaptureStatusNone) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(stream_, &g);
    if (g) (void)hipGraphDestroy(g);
  }
  (void)hipGetLastError();  // clear the capture error
  if (stream_) dev_capture_end(stream_);
  if (pool_open_) {
    c10::hip::HIPCachingAllocator::get()->endAllocateToPool(static_cast<c10::DeviceIndex>(device_), pool_);
    pool_open_ = false;
  }
}

void HipGraph::replay(hipStream_t stream) {
  TFA_CHECK(exec_ != nullptr, "HipGraph: replay before capture");
  hipError_t e = hipGraphLaunch(exec_, stream);
  TFA_CHECK(e == hipSuccess, "hipGraphLaunch failed: ", hipGetErrorString(e));
}

HipGraph::~HipGraph() {
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
  if (pool_open_) c10::hip::HIPCachingAllocator::get()->endAllocateToPool(static_cast<c10::DeviceIndex>(device_), pool_);
  if (pool_owned_) c10::hip::HIPCachingAllocator::get()->releasePool(static_cast<c10::DeviceIndex>(device_), pool_);
}

}  // namespace tfa

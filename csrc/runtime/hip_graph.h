// HIP graph capture / replay of one plan's kernel sequence (runtime-owned:
// raw hipStreamBeginCapture / hipGraphInstantiate / hipGraphLaunch).
//
// Tensors allocated while a stream is being captured come from a private pool
// of the HIP caching allocator that lives as long as the graph, so the
// addresses baked into the captured kernels stay valid across replays.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

namespace tfa {

class HipGraph {
 public:
  HipGraph() = default;
  HipGraph(const HipGraph&) = delete;
  HipGraph& operator=(const HipGraph&) = delete;
  ~HipGraph();

  // Starts capturing `stream` (thread-local mode) on `device`.
  void begin(hipStream_t stream, int device);
  // Ends the capture and instantiates the executable graph.
  void end();
  // Abandons a capture after an error (the stream's capture is ended and discarded).
  void abort();
  // Launches the graph on `stream`.
  void replay(hipStream_t stream);
  bool ready() const { return exec_ != nullptr; }

 private:
  hipStream_t stream_ = nullptr;
  int device_ = -1;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  std::pair<unsigned long long, unsigned long long> pool_{0, 0};
  bool pool_open_ = false, pool_owned_ = false;
};

}  // namespace tfa

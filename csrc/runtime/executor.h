// Program = a graph pruned to (fetches, feeds) + a cache of concrete plans.
//
// Replaces the per-partition `withSession { runner.feed(..).fetch(..).run() }`
// of the reference (reference: src/main/scala/org/tensorframes/impl/DebugRowOps.scala:766-803,900-917).
// A plan is specialised to concrete feed shapes: shapes are inferred, every
// shape-only subgraph is folded on the host, MatMul/Conv2D + BiasAdd + Relu
// chains are fused into one kernel, and intermediate buffers are released at
// their last use (the HIP caching allocator then reuses them).
#pragma once

#include <ATen/ATen.h>
#include <hip/hip_runtime.h>

#include <map>
#include <tuple>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

#include "../ir/graph.h"

namespace tfa {

struct MonoidInfo {
  std::string fetch;
  std::string placeholder;
  std::string op;  // Sum / Min / Max / Prod
};

struct ExecStats {
  int64_t runs = 0;
  int64_t kernels = 0;
  int64_t plans_built = 0;
  int64_t plans_adopted = 0;  // plans taken over from a structurally equal program
  int64_t h2d_bytes = 0;
  int64_t d2h_bytes = 0;
  int64_t chunks = 0;
  double h2d_ms = 0, compute_ms = 0, d2h_ms = 0, wall_ms = 0;
  double plan_ms = 0;     // host time building plans (inference, fusion, kernel choice)
  double exec_ms = 0;     // host time issuing a plan's steps (launch overhead on a GPU)
  int64_t graphs_captured = 0, graph_replays = 0, graph_failures = 0, graphs_declined = 0;
  int64_t graph_busy = 0;  // pointer-keyed replays that copied their outputs out (the caller held the aliases)
};

class Program {
 public:
  Program(std::shared_ptr<Graph> g, const std::vector<std::string>& fetches,
          const std::vector<std::string>& feeds);
  ~Program();

  const std::vector<std::string>& fetch_names() const { return fetch_names_; }
  const std::vector<std::string>& feed_names() const { return feed_names_; }

  // Static analysis with optional hints (dtype/shape per feed).
  Graph::Infos analyze(const std::map<std::string, TensorInfo>& feed_infos) const;
  // Can the graph be evaluated on row chunks of the block independently?
  bool row_separable(const std::map<std::string, TensorInfo>& feed_infos) const;
  // Per-fetch monoid reduction `fetch = Op(placeholder, axis 0)` (empty if not all are).
  std::vector<MonoidInfo> monoids() const;

  // Plan reuse across rebuilt graphs of the same structure (Graph::structure_key):
  // take over `old`'s plans (step lists, fused kernels, HIP-graph captures and
  // device constant arenas) for this program's graph, whose parameter
  // constants may hold different values. Each arena is refreshed in place with
  // this graph's values by one asynchronous host->device copy before its next
  // run, so captured graphs stay valid. `old` keeps its own graph and plans
  // afresh if it runs again (a lazy frame built on it still sees its own
  // constants). False (nothing moved) when the structures differ.
  bool adopt(Program& old);
  // A program for this graph with new parameter-constant payloads
  // (Graph::with_values) that takes over this program's plans: the per-step
  // rebuild of an iterative workload without serialising or parsing a graph.
  std::shared_ptr<Program> rebind(const std::map<std::string, at::Tensor>& values);

  // Run on concrete inputs (all on one device: CPU or a GPU). Returns the fetches.
  std::vector<at::Tensor> run(const std::vector<at::Tensor>& inputs);

  // Independent runs over several input sets on one GPU (the device-resident
  // partitions of one map_blocks), forked onto up to `max_streams` engine side
  // streams after the caller's stream and joined back into it: a partition
  // whose chain of small kernels cannot fill the GPU runs beside the others.
  // The fork/join is a few event records and waits on the host (no Python
  // stream objects); outputs are ordered into the caller's stream.
  std::vector<std::vector<at::Tensor>> run_concurrent(const std::vector<std::vector<at::Tensor>>& inputs_list,
                                                      int max_streams = 4);

  // Pipelined host->device->host execution over row chunks of several segments.
  // seg_inputs[s][i]: pinned host tensor for feed i of segment s (leading dim = rows).
  // seg_outputs[s][j]: preallocated pinned host tensor for fetch j.
  //
  // The ring of device input slots and the per-slot events persist across
  // calls (one pipeline per program and device): a call continues the slot
  // rotation of the previous one, so its first H2D waits only for the compute
  // of the chunk that last used that slot, not for the whole previous call.
  // wait = false: return as soon as every copy and kernel is enqueued (no
  // synchronisation); the result is an event handle that completes when the
  // last D2H has landed (pipeline_wait). The caller keeps seg_inputs and
  // seg_outputs alive until then. wait = true: returns 0 after the drain.
  int64_t run_chunked(const std::vector<std::vector<at::Tensor>>& seg_inputs,
                      const std::vector<std::vector<at::Tensor>>& seg_outputs, int64_t chunk_rows,
                      int device, int depth, bool wait = true);

  void release_pipeline() {
    std::lock_guard<std::mutex> lk(pipe_mu_);
    drop_pipe(false);
  }

  // Pipelined host->device reduction over row chunks (reduce_blocks of host
  // partitions): every chunk's fetches are copied into slot c of a device
  // buffer [nchunks, *fetch shape] on the compute stream while the next chunk's
  // H2D runs on the copy stream; nothing comes back to the host. Returns the
  // stacked per-chunk partials (device), which the caller folds with the same
  // (associative) graph.
  std::vector<at::Tensor> run_chunked_reduce(const std::vector<std::vector<at::Tensor>>& seg_inputs,
                                             int64_t chunk_rows, int device, int depth);

  ExecStats stats() const;
  void reset_stats();
  // as_gpu: describe the plan a GPU run would use (fusion included), from host tensors
  std::string describe_plan(const std::vector<at::Tensor>& inputs, bool as_gpu = false);
  // generated sources of the fused regions of the GPU plan for these input shapes
  std::vector<std::string> fused_sources(const std::vector<at::Tensor>& inputs);

 private:
  std::string host_op_error_;  // set when a host-only op is reachable (analysis ok, running not)
  struct Step;
  struct Plan;
 public:
  // a captured replay whose output buffers are handed out as aliases: told
  // about every other stream a consumer queued reads of an alias on
  struct AliasUseSink {
    virtual ~AliasUseSink() = default;
    virtual void record_use(hipStream_t s) = 0;
  };

 private:
  std::shared_ptr<Plan> plan_for(const std::vector<at::Tensor>& inputs);
  std::shared_ptr<Plan> build_plan(const std::vector<at::Tensor>& inputs, bool force_gpu);
  std::vector<at::Tensor> execute(Plan& p, const std::vector<at::Tensor>& inputs, void* stream);
  at::Tensor device_const(Plan& p, int slot, const at::Device& dev, void* stream);
  void upload_consts(Plan& p, std::map<int, at::Tensor>& m, const at::Device& dev, void* stream);
  void wait_consts(const at::Device& dev, void* stream);
  void refresh_consts(Plan& p, int di, void* stream);
  bool graphable(const Plan& p) const;
  std::string graph_blocker(const Plan& p) const;
  std::vector<at::Tensor> run_graph(Plan& p, const std::vector<at::Tensor>& inputs);
  std::optional<std::vector<at::Tensor>> run_ptr_graph(Plan& p, const std::vector<at::Tensor>& inputs,
                                                       int64_t bytes);

  std::shared_ptr<Graph> g_;
  std::vector<std::string> fetch_names_, feed_names_;
  std::vector<TensorRef> fetches_;
  std::vector<int> feed_nodes_;
  std::vector<int> order_;
  std::mutex mu_;
  static constexpr size_t kMaxPlans = 256;
  std::map<std::string, std::shared_ptr<Plan>> plans_;
  std::mutex const_mu_;
  std::map<std::tuple<int, int, int>, at::Tensor> graph_consts_;  // (node, output, device) -> tensor
  // constants go up with an asynchronous copy on the stream of the run that
  // needs them first; a run on another stream waits for that copy's event
  std::map<std::pair<int, void*>, void*> const_events_;  // (device, upload stream) -> hipEvent_t
  ExecStats stats_;
  // persistent chunk pipeline of run_chunked (see there)
  struct Pipe {
    int device = -1, depth = 0;
    int64_t rows = 0;                          // ring capacity in rows
    std::vector<std::vector<int64_t>> shapes;  // per feed: row shape
    std::vector<at::ScalarType> dtypes;
    std::vector<std::vector<at::Tensor>> ring; // [slot][feed]
    std::vector<hipEvent_t> ev_comp, ev_d2h;   // per slot: last compute / D2H that used it
    std::vector<bool> used;
    int64_t next = 0;                          // chunk counter (slot = next % depth)
  };
  std::mutex pipe_mu_;
  std::unique_ptr<Pipe> pipe_;
  // caller holds pipe_mu_: free ring and events (draining the streams first
  // unless `synced`)
  void drop_pipe(bool synced);
};

// per-step device time of GPU plan runs while on (tools: the per-layer table
// of the plan that ran); read_step_timing waits for and drains the records
struct StepTiming {
  std::string node, op, label;
  double flops, bytes;  // bytes: operands in + outputs out, once each
  float ms;
};
void set_step_timing(bool on);
bool step_timing();
std::vector<StepTiming> read_step_timing();

// waits for (and releases) an event handle returned by run_chunked(wait=false)
void pipeline_wait(int64_t handle);

// pinned host memory (hipHostMalloc, exact size; freed with hipHostFree)
at::Tensor empty_pinned(const std::vector<int64_t>& sizes, at::ScalarType dt);
void trim_pinned_pool();
size_t pinned_pool_cached_bytes();
// {limit, cached (free) bytes, live bytes, peak live bytes} of the pinned pool
std::vector<size_t> pinned_pool_stats();
// page-lock an existing host tensor's memory in place (hipHostRegister)
void pin_host_tensor(const at::Tensor& t);
void unpin_host_tensor(const at::Tensor& t);
// the runtime's persistent copy streams: which = 0 host->device, 1 device->host
hipStream_t copy_stream(int device, int which);
// Config.debug_sync: synchronise + check after every kernel (read per launch)
void set_debug_sync(bool on);
bool get_debug_sync();

}  // namespace tfa

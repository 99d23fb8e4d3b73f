// Planner + executor (see executor.h).
#include "executor.h"

#include <optional>
#include "device_pool.h"


#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <unistd.h>
#include <cstdlib>
#include <set>
#include <unordered_map>
#include <sstream>

#include "../ir/ops_common.h"
#include "fusion.h"
#include "hip_graph.h"
#include "jit.h"

namespace tfa {


namespace {

#define HIP_OK(expr)                                                                  \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TFA_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ", #expr); \
  } while (0)

// -1: not set yet (TFA_DEBUG_SYNC decides on first use); set_debug_sync()
// (Config.debug_sync) overrides it at any time, read on every launch
std::atomic<int> g_debug_sync{-1};

bool debug_sync() {
  int v = g_debug_sync.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("TFA_DEBUG_SYNC");
    int want = (e && e[0] == '1') ? 1 : 0;
    g_debug_sync.compare_exchange_strong(v, want);
    v = g_debug_sync.load(std::memory_order_relaxed);
  }
  return v == 1;
}

struct RangeGuard {
  explicit RangeGuard(const std::string& name) { roctxRangePushA(name.c_str()); }
  ~RangeGuard() { roctxRangePop(); }
};

// Step timing (set_step_timing): a hipEvent pair around every step of every
// GPU plan run while it is on, read back (device ms, FLOPs, the step's label)
// by read_step_timing: the per-layer table of the plan that really ran
// (sibling-fused convs, Winograd or implicit GEMM), not of isolated layers.
std::atomic<bool> g_step_timing{false};
struct StepRec {
  std::string node, op, label;
  double flops = 0, bytes = 0;
  hipEvent_t a = nullptr, b = nullptr;
};
std::mutex g_step_mu;
std::vector<StepRec> g_step_recs;

// TFA_STAGE_TIMERS=0 turns off the per-chunk hipEvent stage timers of run_chunked
bool stage_timers_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TFA_STAGE_TIMERS");
    return !(e && e[0] == '0');
  }();
  return on;
}

// unary ops a GEMM/conv epilogue absorbs (k::Act code; ACT_NONE = not fusible)
int epilogue_act(const std::string& op) {
  static const std::map<std::string, int> m = {
      {"Relu", k::ACT_RELU},   {"Relu6", k::ACT_RELU6}, {"Sigmoid", k::ACT_SIGMOID}, {"Tanh", k::ACT_TANH},
      {"Elu", k::ACT_ELU},     {"Selu", k::ACT_SELU},   {"Softplus", k::ACT_SOFTPLUS}};
  auto it = m.find(op);
  return it == m.end() ? k::ACT_NONE : it->second;
}

const char* act_name(int act) {
  static const char* names[] = {"none", "relu", "relu6", "sigmoid", "tanh", "elu", "selu", "softplus"};
  return act >= 0 && act < 8 ? names[act] : "?";
}

// TFA_EPI_CHAIN=0: GEMM/conv epilogues absorb bias and one activation only
bool epi_chain_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TFA_EPI_CHAIN");
    return !(e && e[0] == '0');
  }();
  return on;
}

// TFA_SIBLING_FUSION=0: sibling convs (same input, same geometry) stay separate GEMMs
bool sibling_fusion_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TFA_SIBLING_FUSION");
    return !(e && e[0] == '0');
  }();
  return on;
}

// TFA_POOL_FUSION=0: pools keep their own BiasAdd/Relu steps and write
// their own outputs (no fused epilogue, no concat slice)
bool pool_fusion_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TFA_POOL_FUSION");
    return !(e && e[0] == '0');
  }();
  return on;
}

// TFA_PIPE_COMPUTE_STREAMS: compute streams of the chunk pipeline (1 or 2)
int pipe_compute_streams() {
  static const int n = [] {
    const char* e = std::getenv("TFA_PIPE_COMPUTE_STREAMS");
    return e && e[0] == '1' ? 1 : 2;
  }();
  return n;
}

// TFA_POOL_CONV_FUSION=0 (or set_pool_conv_fusion(false), for plans made
// after it): a 3x3 VALID MaxPool feeding only a 1x1 conv stays its own step.
// Fused (default), Inception-v3's MaxPool_3a -> Conv2d_3b takes 13.9 ms per
// 8 x 2048 images against 18.8 ms for the pool kernel + the 1x1 GEMM
// (the wave-specialised kernel, profiles/r6_poolconv/)
std::atomic<int>& pool_conv_fusion_state() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_POOL_CONV_FUSION");
    return (e && e[0] == '0') ? 0 : 1;
  }());
  return v;
}

}  // namespace

void set_pool_conv_fusion(bool on) { pool_conv_fusion_state().store(on ? 1 : 0); }

namespace {

// TFA_CONV_POOL_FUSION=0: a 2x2 / stride-2 MaxPool after a Winograd conv
// stays its own step (A/B of the pooled Winograd epilogue)
bool conv_pool_fusion_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TFA_CONV_POOL_FUSION");
    return !(e && e[0] == '0');
  }();
  return on;
}

// transposition flags of MatMul (transpose_a/b) and BatchMatMul (adj_x/y)
bool gemm_ta(const Node& nd) {
  return nd.op == "MatMul" ? nd.attr_b("transpose_a", false) : nd.attr_b("adj_x", false);
}
bool gemm_tb(const Node& nd) {
  return nd.op == "MatMul" ? nd.attr_b("transpose_b", false) : nd.attr_b("adj_y", false);
}

std::string strip0(const std::string& s) {
  if (s.size() > 2 && s.compare(s.size() - 2, 2, ":0") == 0) return s.substr(0, s.size() - 2);
  return s;
}

}  // namespace

void set_debug_sync(bool on) { g_debug_sync.store(on ? 1 : 0); }

// Persistent non-blocking copy streams, created on first use: [device][0 = H2D, 1 = D2H]
hipStream_t copy_stream(int device, int which) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, hipStream_t> streams;
  std::lock_guard<std::mutex> lk(mu);
  auto it = streams.find({device, which});
  if (it != streams.end()) return it->second;
  int cur = 0;
  TFA_CHECK(hipGetDevice(&cur) == hipSuccess, "hipGetDevice failed");
  TFA_CHECK(hipSetDevice(device) == hipSuccess, "hipSetDevice failed");
  hipStream_t st = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  (void)hipSetDevice(cur);
  TFA_CHECK(e == hipSuccess, "hipStreamCreate failed: ", hipGetErrorString(e));
  streams[{device, which}] = st;
  return st;
}
bool get_debug_sync() { return debug_sync(); }

struct Program::Step {
  enum Kind { OP, GEMM, CONV, FUSED } kind = OP;
  int fused = -1;        // FUSED: index into Plan::fused
  int node = -1;         // node whose op runs (for GEMM/CONV: the MatMul/Conv2D node)
  int out_node = -1;     // node whose outputs this step produces
  std::vector<int> in_slots;
  std::vector<int> out_slots;
  std::vector<TensorInfo> out_info;
  std::vector<const TensorInfo*> in_info;
  int bias_slot = -1;
  TensorRef bias_ref{-1, 0};  // planning: resolved to bias_slot when the step is placed
  int act = 0;
  // absorbed elementwise chain after bias/act (GEMM/CONV steps)
  struct Epi {
    int code, kind, act;
    double s;
    int slot;       // tensor operand slot (-1: none / constant scalar)
    TensorRef ref;  // planning: the operand, resolved to `slot` when the step is placed
  };
  std::vector<Epi> epi;
  Shape gemm_shape;  // GEMM/CONV: the MatMul/Conv2D's own output shape (out_info may be a view of it)
  std::vector<int> release;  // slots dropped after the step
  // write-into-slice (GPU): a GEMM/CONV step whose only consumer is a
  // last-axis ConcatV2 writes straight into its channel range of the concat
  // output (allocated by the first such producer); the concat then copies
  // only the remaining inputs
  int alias_slot = -1;           // producer: concat output slot
  int64_t alias_offset = 0;      // producer: first channel in the concat output
  const TensorInfo* alias_info = nullptr;  // producer: concat output info
  std::vector<char> preplaced;   // concat: per value input, already written in place
  // horizontally fused sibling convs (GPU plans): Conv2Ds that read the same
  // input with the same geometry run as ONE implicit GEMM over their
  // concatenated filters (wider N: more blocks, less tile padding); every
  // member writes its own output, or its concat slice
  struct Sib {
    int node;
    int64_t oc;
    int alias_slot;
    int64_t alias_offset;
    const TensorInfo* alias_info;
    int act;  // this member's epilogue activation (members may differ)
  };
  std::vector<Sib> sibs;
  // Winograd F(2x2,3x3) filter of this CONV step (plan-made constant slot, or
  // -1): 3x3 stride-1 convs whose filter is a constant (conv_wino.hip)
  int wino_slot = -1;
  bool pool2 = false;  // CONV: writes the 2x2 / stride-2 max pool of its output (planner-fused MaxPool)
  // CONV 1x1: reads the VALID max pool {kh, kw, sh, sw} of in_slots[0] (planner-fused MaxPool before it)
  int pool_in[4] = {0, 0, 0, 0};
};

struct Program::Plan {
  Graph::Infos infos;
  std::vector<Step> steps;
  int nslots = 0;
  std::vector<int> feed_slots;
  std::vector<std::pair<int, TensorRef>> const_slots;  // slot <- constant value of ref
  std::map<int, at::Tensor> synth_consts;               // slot <- plan-made constant (fused sibling filters)
  std::vector<int> fetch_slots;
  std::map<int, std::map<int, at::Tensor>> dev_consts;  // device index -> slot -> tensor
  std::map<int, TensorInfo> feed_infos;                  // what the plan was inferred with
  // the graph the plan was built from: infos values may view its constant
  // payloads, and adopt() carries the infos of unchanged nodes over from it
  std::shared_ptr<Graph> base_graph;
  // one device arena per device (upload_consts): the slots it holds, for an
  // in-place refresh after adopt()
  struct Arena {
    at::Tensor dev;
    std::vector<std::tuple<int, TensorRef, size_t, size_t>> items;  // slot, ref, offset, bytes
  };
  std::map<int, Arena> arenas;
  std::set<int> stale;                  // devices whose constants predate adopt()
  bool cap_reset = false;               // the capture reads constants that were replaced
  std::map<int, void*> last_stream;     // device -> stream of the last run
  // device -> every stream a run or replay of this plan was issued on (the
  // arena refresh waits for all of them: partitions may run concurrently)
  std::map<int, std::set<void*>> used_streams;
  int fused = 0;
  int fused_siblings = 0;  // convs folded into sibling-fused steps
  int wino_convs = 0;      // Winograd filters made (one per distinct 3x3 s1 filter)
  // fused elementwise regions (GPU plans): generated source + loaded kernel per device
  struct Fused {
    FusedRegion region;
    std::mutex mu;
    std::map<int, jit::Kernel> kernels;
  };
  std::vector<std::unique_ptr<Fused>> fused_regions;
  // HIP-graph replay of this plan (small, repeated launches): static input
  // buffers the inputs are copied into, the captured graph, its outputs
  // replays of one capture share its buffers: a replay on another stream
  // than the last one first waits for that stream (rare: concurrent
  // partitions; a per-replay event record cost 3 us of host time)
  struct ReplayOrder {
    hipStream_t last = nullptr;
    void before(hipStream_t cur) {
      if (last && last != cur) (void)hipStreamSynchronize(last);
    }
    void after(hipStream_t cur) { last = cur; }
    void drain() {
      if (last) (void)hipStreamSynchronize(last);
      last = nullptr;
    }
  };
  struct Captured {
    std::mutex mu;
    int64_t gpu_runs = 0;
    bool failed = false;
    // host time of warm eager runs vs replays: a replay (input copy + graph
    // launch + output clone) can cost more than launching a few kernels
    int64_t eager_ns = 0, eager_n = 0, replay_ns = 0, replay_n = 0;
    bool declined = false;
    int device = -1;
    hipStream_t stream = nullptr;  // our own capture stream (never shared)
    std::unique_ptr<HipGraph> graph;
    std::vector<at::Tensor> static_in, static_out;
    ReplayOrder order;
    ~Captured() {
      order.drain();
      graph.reset();
      if (stream) (void)hipStreamDestroy(stream);
    }
  } cap;
  // zero-copy replays for device inputs that come back at the same addresses
  // (device-cached partitions of an iterative workload): the graph is
  // captured on the caller's own input tensors, so a replay copies nothing in;
  // keyed by the input data pointers (same plan => same shapes and dtypes)
  // The outputs of the first instance of a pointer set are handed out as
  // aliases of the graph's own output buffers (no copy): it replays only once
  // the caller has dropped every output of its last replay (storage use
  // counts back at their values right after the capture). While they are
  // held, a second, `cloning` instance replays and copies its outputs out.
  // Uses of the aliases on other streams: a consumer that queued work reading
  // an alias on another stream and said so (engine.record_stream ->
  // dev_record_stream -> replay_alias_record_stream) gets an event recorded
  // there; the next replay waits for those events before it rewrites the
  // buffers, so dropping the host reference early is safe (ReplayOrder only
  // orders replays against each other).
  struct PtrCap : AliasUseSink {
    bool cloning = false;
    std::unique_ptr<HipGraph> graph;
    std::vector<at::Tensor> static_out;
    std::vector<long> base_uc;      // storage use count of each output after capture
    std::vector<bool> input_alias;  // output is (a view of) an input: never written
    hipStream_t stream = nullptr;
    int64_t last_use = 0;
    ReplayOrder order;
    std::mutex use_mu;
    std::vector<hipEvent_t> uses;   // events on consumer streams since the last replay
    bool outputs_free() const {
      for (size_t i = 0; i < static_out.size(); ++i)
        if (!input_alias[i] && static_out[i].storage().use_count() > base_uc[i]) return false;
      return true;
    }
    void record_use(hipStream_t s) override {
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipStreamSynchronize(s);  // no event: make the use complete now instead
        return;
      }
      (void)hipEventRecord(e, s);
      std::lock_guard<std::mutex> lk(use_mu);
      uses.push_back(e);
    }
    void wait_uses(hipStream_t cur) {
      std::lock_guard<std::mutex> lk(use_mu);
      for (hipEvent_t e : uses) {
        (void)hipStreamWaitEvent(cur, e, 0);
        (void)hipEventDestroy(e);  // destroyed after the wait is enqueued: HIP keeps it until then
      }
      uses.clear();
    }
    ~PtrCap() override;
  };
  std::mutex ptr_mu;
  std::map<std::vector<const void*>, int> ptr_seen;  // pointer set -> runs seen (bounded)
  std::map<std::vector<const void*>, std::vector<std::unique_ptr<PtrCap>>> ptr_caps;
  int64_t ptr_tick = 0;
  bool ptr_declined = false;
  int64_t ptr_eager_ns = 0, ptr_eager_n = 0, ptr_replay_ns = 0, ptr_replay_n = 0;
};

namespace {
// storage base of every aliased replay output -> its capture
std::mutex g_alias_mu;
std::unordered_map<const void*, Program::AliasUseSink*>& alias_registry() {
  static auto* m = new std::unordered_map<const void*, Program::AliasUseSink*>();
  return *m;
}
void register_aliases(Program::AliasUseSink* sink, const std::vector<const void*>& ptrs) {
  std::lock_guard<std::mutex> lk(g_alias_mu);
  for (const void* q : ptrs) alias_registry()[q] = sink;
}
void unregister_aliases(Program::AliasUseSink* sink, const std::vector<const void*>& ptrs) {
  std::lock_guard<std::mutex> lk(g_alias_mu);
  for (const void* q : ptrs) {
    auto it = alias_registry().find(q);
    if (it != alias_registry().end() && it->second == sink) alias_registry().erase(it);
  }
}
std::vector<const void*> alias_ptrs(const std::vector<at::Tensor>& outs, const std::vector<bool>& input_alias) {
  std::vector<const void*> v;
  for (size_t i = 0; i < outs.size(); ++i)
    if (!input_alias[i]) v.push_back(outs[i].storage().data_ptr().get());
  return v;
}
}  // namespace

Program::Plan::PtrCap::~PtrCap() {
  if (!cloning) unregister_aliases(this, alias_ptrs(static_out, input_alias));
  for (hipEvent_t e : uses) {
    (void)hipEventSynchronize(e);
    (void)hipEventDestroy(e);
  }
  order.drain();
  graph.reset();
  if (stream) (void)hipStreamDestroy(stream);
}

bool replay_alias_record_stream(const void* p, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_alias_mu);
  auto it = alias_registry().find(p);
  if (it == alias_registry().end()) return false;
  it->second->record_use(s);
  return true;
}

Program::Program(std::shared_ptr<Graph> g, const std::vector<std::string>& fetches,
                 const std::vector<std::string>& feeds)
    : g_(std::move(g)) {
  TFA_CHECK(!fetches.empty(), "no fetches given");
  std::set<std::string> seen;
  for (auto& f : fetches) {
    fetches_.push_back(g_->resolve(f));
    fetch_names_.push_back(strip0(f));
  }
  std::set<int> cut;
  for (auto& f : feeds) {
    TensorRef r = g_->resolve(f);
    TFA_CHECK(r.index == 0, "can only feed output 0 of node '", f, "'");
    feed_nodes_.push_back(r.node);
    feed_names_.push_back(strip0(f));
    cut.insert(r.node);
  }
  // closure with feed nodes as cut points
  std::vector<int> state(g_->nodes().size(), 0);
  std::vector<std::pair<int, size_t>> stack;
  for (auto& f : fetches_) {
    if (state[f.node]) continue;
    stack.push_back({f.node, 0});
    state[f.node] = 1;
    while (!stack.empty()) {
      auto& [n, k] = stack.back();
      const Node& nd = g_->node(n);
      size_t total = cut.count(n) ? 0 : nd.inputs.size() + nd.control.size();
      if (k < total) {
        int dep = k < nd.inputs.size() ? nd.inputs[k].node : nd.control[k - nd.inputs.size()];
        ++k;
        TFA_CHECK(state[dep] != 1, "cycle in graph at node '", g_->node(dep).name, "'");
        if (state[dep] == 0) {
          state[dep] = 1;
          stack.push_back({dep, 0});
        }
      } else {
        state[n] = 2;
        order_.push_back(n);
        stack.pop_back();
      }
    }
  }
  // feeds outside the fetch closure still get an (inferred) info slot
  {
    std::set<int> in_order(order_.begin(), order_.end());
    std::vector<int> extra;
    for (int f : feed_nodes_)
      if (!in_order.count(f)) extra.push_back(f);
    order_.insert(order_.begin(), extra.begin(), extra.end());
  }
  // every placeholder reached must be fed; host ops must be cut off (fed) to run
  for (int n : order_) {
    const Node& nd = g_->node(n);
    if (!cut.count(n) && host_op_error_.empty()) {
      const OpDef* od = OpRegistry::get().find(nd.op);
      if (od && od->host_only)
        host_op_error_ = str_cat(nd.op, " (node '", nd.name, "') is a host op: it is decoded on the host by "
                                 "the map_rows host stage; feed its output or use map_rows with a binary column");
    }
    if ((nd.op == "Placeholder" || nd.op == "PlaceholderV2") && !cut.count(n))
      TFA_CHECK(false, "placeholder '", nd.name, "' is needed by the fetches but is not fed");
  }
}

Graph::Infos Program::analyze(const std::map<std::string, TensorInfo>& feed_infos) const {
  std::map<int, TensorInfo> feeds;
  for (size_t i = 0; i < feed_nodes_.size(); ++i) {
    auto it = feed_infos.find(feed_names_[i]);
    if (it != feed_infos.end()) {
      TensorInfo ti = it->second;
      ti.row = RowClass::ROW;
      feeds[feed_nodes_[i]] = ti;
    } else {
      const Node& nd = g_->node(feed_nodes_[i]);
      if (nd.op != "Placeholder" && nd.op != "PlaceholderV2") {
        TensorInfo ti;
        ti.row = RowClass::ROW;
        feeds[feed_nodes_[i]] = ti;
      }
    }
  }
  return g_->infer(order_, feeds, false);
}

bool Program::row_separable(const std::map<std::string, TensorInfo>& feed_infos) const {
  Graph::Infos infos = analyze(feed_infos);
  for (auto& f : fetches_)
    if (infos[f.node][f.index].row != RowClass::ROW) return false;
  return true;
}

std::vector<MonoidInfo> Program::monoids() const {
  std::vector<MonoidInfo> out;
  for (size_t i = 0; i < fetches_.size(); ++i) {
    const Node& n = g_->node(fetches_[i].node);
    if (!(n.op == "Sum" || n.op == "Min" || n.op == "Max" || n.op == "Prod")) return {};
    if (n.inputs.size() != 2) return {};
    const Node& src = g_->node(n.inputs[0].node);
    if (!(src.op == "Placeholder" || src.op == "PlaceholderV2")) return {};
    const Node& ax = g_->node(n.inputs[1].node);
    if (ax.op != "Const") return {};
    at::Tensor v = host_tensor_to_at(ax.attr_tensor("value"));
    auto axes = to_int_vector(v);
    if (axes.size() != 1 || axes[0] != 0) return {};
    bool keep = n.has_attr("keep_dims") ? n.attr_b("keep_dims") : n.attr_b("keepdims", false);
    if (keep) return {};
    out.push_back({fetch_names_[i], src.name, n.op});
  }
  return out;
}

static std::string plan_key(const std::vector<at::Tensor>& inputs) {
  std::ostringstream os;
  for (auto& t : inputs) {
    os << static_cast<int>(t.scalar_type()) << ':' << (t.is_cuda() ? 1 : 0) << '[';
    for (auto d : t.sizes()) os << d << ',';
    os << ']';
  }
  return os.str();
}

std::shared_ptr<Program::Plan> Program::plan_for(const std::vector<at::Tensor>& inputs) {
  TFA_CHECK(inputs.size() == feed_nodes_.size(), "expected ", feed_nodes_.size(), " inputs, got ",
            inputs.size());
  std::string key = plan_key(inputs);
  std::lock_guard<std::mutex> lk(mu_);
  auto it = plans_.find(key);
  if (it != plans_.end()) return it->second;
  const auto tp = std::chrono::steady_clock::now();
  auto p = build_plan(inputs, false);
  stats_.plan_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
  if (plans_.size() >= kMaxPlans) plans_.erase(plans_.begin());  // bounded (e.g. many image sizes)
  plans_[key] = p;
  stats_.plans_built++;
  return p;
}

std::shared_ptr<Program::Plan> Program::build_plan(const std::vector<at::Tensor>& inputs, bool force_gpu) {
  auto p = std::make_shared<Plan>();
  p->base_graph = g_;
  const bool gpu_plan = force_gpu || (!inputs.empty() && inputs[0].is_cuda());
  std::map<int, TensorInfo> feeds;
  for (size_t i = 0; i < inputs.size(); ++i) {
    TensorInfo ti;
    ti.dtype = from_scalar_type(inputs[i].scalar_type());
    ti.shape = shape_of(inputs[i]);
    ti.row = RowClass::ROW;
    const Node& nd = g_->node(feed_nodes_[i]);
    if (nd.op == "Placeholder" || nd.op == "PlaceholderV2") {
      DType want = nd.attr_type("dtype");
      TFA_CHECK(want == ti.dtype, "placeholder '", nd.name, "' has dtype ", dtype_name(want),
                " but was fed ", dtype_name(ti.dtype), " (no implicit casting)");
      if (const AttrValue* a = nd.def->find_attr("shape")) {
        if (a->kind == AttrValue::SHAPE && !a->shape.unknown_rank) {
          const Shape& s = a->shape;
          bool ok = s.rank() == ti.shape.rank();
          for (int d = 0; ok && d < s.rank(); ++d) ok = s.dims[d] < 0 || s.dims[d] == ti.shape.dims[d];
          TFA_CHECK(ok, "placeholder '", nd.name, "' has shape ", s.str(), " but was fed ", ti.shape.str());
        }
      }
    }
    feeds[feed_nodes_[i]] = ti;
  }
  // TFA_PLAN_TIMING=1: host time of each planning phase on stderr
  static const bool plan_timing = [] {
    const char* e = std::getenv("TFA_PLAN_TIMING");
    return e && *e && std::string(e) != "0";
  }();
  auto tp0 = std::chrono::steady_clock::now();
  std::vector<std::pair<const char*, double>> phases;
  auto phase = [&](const char* name) {
    if (!plan_timing) return;
    auto t = std::chrono::steady_clock::now();
    phases.push_back({name, std::chrono::duration<double, std::micro>(t - tp0).count()});
    tp0 = t;
  };
  p->feed_infos = feeds;
  p->infos = g_->infer(order_, feeds, true);
  const Graph::Infos& infos = p->infos;
  phase("infer");

  // slots
  std::map<TensorRef, int> slot_of;
  auto new_slot = [&]() { return p->nslots++; };
  std::set<int> feed_set(feed_nodes_.begin(), feed_nodes_.end());
  for (size_t i = 0; i < feed_nodes_.size(); ++i) {
    int s = new_slot();
    slot_of[{feed_nodes_[i], 0}] = s;
    p->feed_slots.push_back(s);
  }
  auto is_const = [&](const TensorRef& r) { return static_cast<bool>(infos[r.node][r.index].value); };
  auto slot_for = [&](const TensorRef& r) -> int {
    auto it = slot_of.find(r);
    if (it != slot_of.end()) return it->second;
    TFA_CHECK(is_const(r), "internal: tensor '", g_->node(r.node).name, ":", r.index, "' has no producer");
    int s = new_slot();
    slot_of[r] = s;
    p->const_slots.push_back({s, r});
    return s;
  };

  // consumer counts (runtime consumers + fetches)
  std::map<TensorRef, int> uses;
  std::set<TensorRef> fetched(fetches_.begin(), fetches_.end());
  std::vector<int> runtime;
  for (int n : order_) {
    if (feed_set.count(n)) continue;
    const Node& nd = g_->node(n);
    bool all_const = true;
    for (auto& o : infos[n]) all_const = all_const && (o.value.has_value() || o.dtype == DType::STRING);
    if (all_const || nd.num_outputs == 0) continue;
    runtime.push_back(n);
    for (auto& r : nd.inputs) uses[r]++;
  }
  for (auto& f : fetches_) uses[f]++;

  std::map<int, int> consumer;  // node -> its single runtime consumer node (if exactly one use)
  for (int n : runtime)
    for (auto& r : g_->node(n).inputs)
      if (uses[r] == 1) consumer[r.node] = n;

  const OpRegistry& reg = OpRegistry::get();
  std::set<int> absorbed;
  // a fused GEMM/CONV step is placed at its LAST absorbed node: the operands of
  // its bias / epilogue chain may be produced by nodes that come after the
  // MatMul in topological order (they all come before the chain's last op)
  auto place = [&](Step& st) {
    if (st.bias_ref.node >= 0) st.bias_slot = slot_for(st.bias_ref);
    for (auto& e : st.epi)
      if (e.ref.node >= 0) e.slot = slot_for(e.ref);
    const Node& nd = g_->node(st.node);
    const OpDef* od = reg.find(nd.op);
    TFA_CHECK(od && od->compute, "op '", nd.op, "' has no compute function");
    for (auto& r : nd.inputs) {
      st.in_slots.push_back(slot_for(r));
      st.in_info.push_back(&infos[r.node][r.index]);
    }
    st.out_info = infos[st.out_node];
    for (size_t k = 0; k < infos[st.out_node].size(); ++k) {
      int s = new_slot();
      slot_of[{st.out_node, static_cast<int>(k)}] = s;
      st.out_slots.push_back(s);
    }
    p->steps.push_back(std::move(st));
  };
  std::map<int, Step> deferred;  // out_node -> fused step waiting for its placement
  for (int n : runtime) {
    auto dit = deferred.find(n);
    if (dit != deferred.end()) {
      place(dit->second);
      deferred.erase(dit);
      continue;
    }
    if (absorbed.count(n)) continue;
    const Node& nd = g_->node(n);
    Step st;
    st.node = n;
    st.out_node = n;
    // ---- fusion: MatMul/Conv2D -> (BiasAdd | Add const-vector) -> (Relu | Relu6),
    // looking through single-consumer view ops (Reshape/Squeeze/ExpandDims/
    // Identity: same elements, same order) between them, e.g. the lifted
    // row-wise MatMul of map_rows: [B*1,k]x[k,n] -> Reshape [B,1,n] -> Squeeze -> Relu
    bool gemm = (nd.op == "MatMul" || nd.op == "BatchMatMul" || nd.op == "BatchMatMulV2") &&
                (infos[n][0].dtype == DType::F32 || infos[n][0].dtype == DType::F64);
    bool conv = nd.op == "Conv2D" && infos[n][0].dtype == DType::F32;
    if (gemm || conv) {
      st.kind = gemm ? Step::GEMM : Step::CONV;
      int cur = n;
      int64_t ncols = infos[n][0].shape.dims.back();
      // the only consumer node of output 0 (it may read it twice: x * x)
      auto single = [&](int node) -> int {
        TensorRef r{node, 0};
        if (fetched.count(r)) return -1;
        if (uses[r] == 1 && consumer.count(node)) return consumer[node];
        if (uses[r] == 2) {
          for (int m : runtime) {
            const auto& ins = g_->node(m).inputs;
            if (std::count(ins.begin(), ins.end(), r) == 2) return m;
          }
        }
        return -1;
      };
      auto is_view = [&](int node) {
        const std::string& op = g_->node(node).op;
        return (op == "Reshape" || op == "Squeeze" || op == "ExpandDims" || op == "Identity") &&
               g_->node(node).inputs.size() >= 1 && infos[node][0].shape.fully_known() &&
               !infos[node][0].shape.dims.empty() && infos[node][0].shape.dims.back() == ncols;
      };
      // follows views from `from`; returns the first non-view single consumer (or -1)
      // and the last view passed (== from when none)
      auto next_op = [&](int from, int* last_view) -> int {
        int at = from;
        for (int guard = 0; guard < 8; ++guard) {
          int c = single(at);
          if (c < 0) { *last_view = at; return -1; }
          if (is_view(c) && g_->node(c).inputs[0] == TensorRef{at, 0}) { at = c; continue; }
          *last_view = at;
          return c;
        }
        *last_view = at;
        return -1;
      };
      int lv = cur;
      int c1 = next_op(cur, &lv);
      if (c1 >= 0) {
        const TensorRef cur_ref{lv, 0};
        const Node& cn = g_->node(c1);
        int other = -1;
        if (cn.op == "BiasAdd" && cn.inputs[0] == cur_ref &&
            cn.attr_s("data_format", std::string("NHWC")) != "NCHW")
          other = 1;
        else if ((cn.op == "Add" || cn.op == "AddV2") && cn.inputs.size() == 2)
          other = cn.inputs[0] == cur_ref ? 1 : (cn.inputs[1] == cur_ref ? 0 : -1);
        if (other >= 0) {
          const TensorRef& br = cn.inputs[other];
          const TensorInfo& bi = infos[br.node][br.index];
          bool ok = bi.shape.rank() == 1 && bi.shape.dims[0] == ncols && bi.dtype == infos[n][0].dtype &&
                    infos[c1][0].shape == infos[lv][0].shape;
          if (ok) {
            st.bias_ref = br;
            for (int v = lv; v != cur; v = g_->node(v).inputs[0].node) absorbed.insert(v);
            absorbed.insert(c1);
            cur = c1;
          }
        }
      }
      int lv2 = cur;
      int c2 = next_op(cur, &lv2);
      if (c2 >= 0) {
        const Node& cn = g_->node(c2);
        const int act = epilogue_act(cn.op);
        if (act != k::ACT_NONE && cn.inputs[0] == TensorRef{lv2, 0}) {
          st.act = act;
          for (int v = lv2; v != cur; v = g_->node(v).inputs[0].node) absorbed.insert(v);
          absorbed.insert(c2);
          cur = c2;
        }
      }
      // ---- absorbed elementwise chain: ops that follow the product (and its
      // bias / activation) one by one, each with a scalar, per-column [N],
      // per-row or same-shaped operand, become the epilogue's program
      const DType gdt = infos[n][0].dtype;
      const bool batched = gemm && infos[n][0].shape.rank() > 2;
      for (int k = 0; k < (epi_chain_enabled() ? k::kMaxEpi : 0); ++k) {
        int lvk = cur;
        int ck = next_op(cur, &lvk);
        if (ck < 0) break;
        const Node& cn = g_->node(ck);
        const TensorRef cref{lvk, 0};
        const TensorInfo& vin = infos[lvk][0];
        const TensorInfo& oinf = infos[ck][0];
        if (oinf.dtype != gdt || !oinf.shape.fully_known() || !(oinf.shape == vin.shape)) break;
        Step::Epi e{k::EPI_ADD, k::EPO_NONE, k::ACT_NONE, 0.0, -1, TensorRef{-1, 0}};
        const int uact = epilogue_act(cn.op);
        static const std::map<std::string, int> unary = {{"Neg", k::EPI_NEG}, {"Square", k::EPI_SQUARE},
                                                         {"Abs", k::EPI_ABS}};
        static const std::map<std::string, std::pair<int, int>> binary = {
            {"Add", {k::EPI_ADD, k::EPI_ADD}},     {"AddV2", {k::EPI_ADD, k::EPI_ADD}},
            {"Sub", {k::EPI_SUB, k::EPI_RSUB}},    {"Mul", {k::EPI_MUL, k::EPI_MUL}},
            {"RealDiv", {k::EPI_DIV, k::EPI_RDIV}}, {"Div", {k::EPI_DIV, k::EPI_RDIV}},
            {"Maximum", {k::EPI_MAX, k::EPI_MAX}}, {"Minimum", {k::EPI_MIN, k::EPI_MIN}}};
        if (uact != k::ACT_NONE || unary.count(cn.op)) {
          if (cn.inputs.empty() || !(cn.inputs[0] == cref)) break;
          e.code = uact != k::ACT_NONE ? k::EPI_ACT : unary.at(cn.op);
          e.act = uact;
        } else if (binary.count(cn.op) && cn.inputs.size() == 2) {
          const bool first = cn.inputs[0] == cref, second = cn.inputs[1] == cref;
          if (first && second) {
            if (cn.op != "Mul") break;
            e.code = k::EPI_SQUARE;
          } else if (first || second) {
            e.code = first ? binary.at(cn.op).first : binary.at(cn.op).second;
            const TensorRef& oref = cn.inputs[first ? 1 : 0];
            const TensorInfo& oi = infos[oref.node][oref.index];
            if (oi.dtype != gdt || !oi.shape.fully_known()) break;
            const auto& od = oi.shape.dims;
            const auto& vd = vin.shape.dims;
            int64_t numel = 1;
            for (int64_t d : od) numel *= d;
            bool col = !od.empty() && od.back() == ncols && numel == ncols;
            bool row = !batched && od.size() == vd.size() && !od.empty() && od.back() == 1 &&
                       std::equal(od.begin(), od.end() - 1, vd.begin());
            if (numel == 1) {
              if (oi.value) {
                e.kind = k::EPO_SCALAR;
                e.s = oi.value->to(at::kDouble).reshape({}).item<double>();
              } else {
                e.kind = k::EPO_SCALAR_PTR;
              }
            } else if (col) {
              e.kind = k::EPO_COL;
            } else if (row) {
              e.kind = k::EPO_ROW;
            } else if (oi.shape == vin.shape) {
              // a full-size operand that the elementwise fusion would compute
              // on the fly (a Tile/broadcast/elementwise producer) stays
              // there: reading it here would materialise it in HBM
              const std::string& pop = g_->node(oref.node).op;
              if (gpu_plan && fusion_enabled() && fusible_op(pop) && pop != "Identity") break;
              e.kind = k::EPO_FULL;
            } else {
              break;
            }
            if (e.kind != k::EPO_SCALAR) e.ref = oref;
          } else {
            break;
          }
        } else {
          break;
        }
        st.epi.push_back(e);
        for (int v = lvk; v != cur; v = g_->node(v).inputs[0].node) absorbed.insert(v);
        absorbed.insert(ck);
        cur = ck;
      }
      st.out_node = cur;
      st.gemm_shape = infos[n][0].shape;
      if (cur != n) p->fused++;
    }
    // ---- fusion (GPU): MaxPool/AvgPool -> BiasAdd [C] -> (Relu | Relu6) in
    // the pool kernel (Inception's reordered pool branch: 1x1 conv, pool,
    // bias, relu), so the pooled tensor is written once
    const bool pool = gpu_plan && pool_fusion_enabled() && (nd.op == "AvgPool" || nd.op == "MaxPool") &&
                      infos[n][0].dtype == DType::F32 && infos[n][0].shape.fully_known() &&
                      infos[n][0].shape.rank() == 4 && nd.attr_s("data_format", std::string("NHWC")) == "NHWC";
    if (pool) {
      const int64_t ch = infos[n][0].shape.dims.back();
      auto only = [&](int node) -> int {
        TensorRef r{node, 0};
        if (fetched.count(r) || uses[r] != 1 || !consumer.count(node)) return -1;
        return consumer[node];
      };
      int cur = n;
      int c1 = only(cur);
      if (c1 >= 0) {
        const Node& cn = g_->node(c1);
        if (cn.op == "BiasAdd" && cn.inputs[0] == TensorRef{cur, 0} &&
            cn.attr_s("data_format", std::string("NHWC")) != "NCHW") {
          const TensorRef& br = cn.inputs[1];
          const TensorInfo& bi = infos[br.node][br.index];
          if (bi.shape.rank() == 1 && bi.shape.dims[0] == ch && bi.dtype == DType::F32 &&
              infos[c1][0].shape == infos[n][0].shape) {
            st.bias_ref = br;
            absorbed.insert(c1);
            cur = c1;
          }
        }
      }
      int c2 = only(cur);
      if (c2 >= 0) {
        const Node& cn = g_->node(c2);
        const int act = epilogue_act(cn.op);
        if ((act == k::ACT_RELU || act == k::ACT_RELU6) && cn.inputs[0] == TensorRef{cur, 0}) {
          st.act = act;
          absorbed.insert(c2);
          cur = c2;
        }
      }
      st.out_node = cur;
      st.gemm_shape = infos[n][0].shape;
      if (cur != n) p->fused++;
    }
    if (st.out_node != n) {
      deferred.emplace(st.out_node, std::move(st));
      continue;
    }
    place(st);
  }
  TFA_CHECK(deferred.empty(), "internal: a fused step was never placed");
  phase("steps+epilogue_chains");
  // ---- elementwise-region fusion (GPU plans): regions replace their member steps
  if (gpu_plan && fusion_enabled()) {
    FusionInput fi;
    fi.g = g_.get();
    fi.infos = &p->infos;
    fi.runtime = runtime;
    fi.fetched = fetched;
    fi.excluded = absorbed;
    for (auto& st : p->steps)
      if (st.kind != Step::OP) fi.excluded.insert(st.node);
    for (int n : runtime)
      for (auto& r : g_->node(n).inputs) fi.consumers[r.node].push_back(n);
    std::vector<FusedRegion> regions = find_fused_regions(fi);
    if (!regions.empty()) {
      std::map<int, int> first_out;  // first output node -> region index
      std::set<int> covered;         // prologue members and outputs: their steps are replaced
      for (size_t i = 0; i < regions.size(); ++i) {
        first_out[regions[i].outputs.front()] = static_cast<int>(i);
        covered.insert(regions[i].nodes.begin(), regions[i].nodes.end());
        covered.insert(regions[i].outputs.begin(), regions[i].outputs.end());
      }
      std::map<int, const Step*> step_of;
      for (auto& st : p->steps)
        if (st.kind == Step::OP) step_of[st.node] = &st;
      std::vector<Step> steps;
      for (auto& st : p->steps) {
        if (st.kind != Step::OP || !covered.count(st.node)) {
          steps.push_back(std::move(st));
          continue;
        }
        auto rit = first_out.find(st.node);
        if (rit == first_out.end()) continue;  // evaluated inside a region's kernel
        const FusedRegion& rg = regions[rit->second];
        Step fs;
        fs.kind = Step::FUSED;
        fs.node = fs.out_node = st.node;
        fs.fused = static_cast<int>(p->fused_regions.size());
        for (auto& l : rg.leaves) {
          fs.in_slots.push_back(slot_for(l.ref));
          fs.in_info.push_back(&infos[l.ref.node][l.ref.index]);
        }
        for (int o : rg.outputs) {
          const Step* os = step_of.at(o);
          TFA_CHECK(os->out_slots.size() == 1, "internal: fused output with several outputs");
          fs.out_slots.push_back(os->out_slots[0]);
          fs.out_info.push_back(os->out_info[0]);
        }
        auto fe = std::make_unique<Plan::Fused>();
        fe->region = rg;
        p->fused_regions.push_back(std::move(fe));
        steps.push_back(std::move(fs));
      }
      p->steps = std::move(steps);
    }
  }
  for (auto& f : fetches_) p->fetch_slots.push_back(slot_for(f));

  // write-into-slice for last-axis ConcatV2 of f32 GEMM/CONV outputs
  {
    std::map<int, size_t> step_of_out;  // slot -> producing step
    for (size_t i = 0; i < p->steps.size(); ++i)
      for (int s : p->steps[i].out_slots) step_of_out[s] = i;
    for (size_t ci = 0; ci < p->steps.size(); ++ci) {
      Step& cs = p->steps[ci];
      const Node& cn = g_->node(cs.node);
      if (cs.kind != Step::OP || cn.op != "ConcatV2" || cs.in_slots.size() < 3) continue;
      const TensorInfo& oi = cs.out_info[0];
      const int nv = static_cast<int>(cs.in_slots.size()) - 1;
      const TensorInfo* ax = cs.in_info[nv];
      if (!ax->value || oi.dtype != DType::F32 || !oi.shape.fully_known() || oi.shape.rank() < 2) continue;
      const int64_t axis = to_int_vector(*ax->value)[0];
      if (axis != -1 && axis != oi.shape.rank() - 1) continue;
      cs.preplaced.assign(nv, 0);
      int64_t off = 0;
      for (int v = 0; v < nv; ++v) {
        const int slot = cs.in_slots[v];
        const TensorInfo* vi = cs.in_info[v];
        const int64_t len = vi->shape.dims.back();
        auto it = step_of_out.find(slot);
        if (it != step_of_out.end()) {
          Step& ps = p->steps[it->second];
          const TensorRef out_ref{ps.out_node, 0};
          const bool single_use = uses[out_ref] == 1 && !fetched.count(out_ref);
          const bool pool_step = ps.kind == Step::OP && gpu_plan && pool_fusion_enabled() &&
                                 (g_->node(ps.node).op == "AvgPool" || g_->node(ps.node).op == "MaxPool") &&
                                 ps.gemm_shape.rank() == 4;
          if ((ps.kind == Step::CONV || ps.kind == Step::GEMM || pool_step) && single_use && ps.alias_slot < 0 &&
              ps.out_info[0].dtype == DType::F32 && ps.out_info[0].shape == ps.gemm_shape) {
            ps.alias_slot = cs.out_slots[0];
            ps.alias_offset = off;
            ps.alias_info = &cs.out_info[0];
            cs.preplaced[v] = 1;
          } else if (ps.kind == Step::OP && g_->node(ps.node).op == "ConcatV2" && single_use &&
                     ps.alias_slot < 0 && !ps.preplaced.empty() &&
                     std::all_of(ps.preplaced.begin(), ps.preplaced.end(), [](char c) { return c != 0; }) &&
                     ps.out_info[0].dtype == DType::F32 && ps.out_info[0].shape.rank() == oi.shape.rank()) {
            // a nested concat whose inputs were all written in place: its
            // producers write straight into the outer concat (offset by this
            // slice), and the inner concat's output is that slice (no copy)
            const int inner = ps.out_slots[0];
            for (auto& q : p->steps)
              if (q.alias_slot == inner) {
                q.alias_slot = cs.out_slots[0];
                q.alias_offset += off;
                q.alias_info = &cs.out_info[0];
              }
            ps.alias_slot = cs.out_slots[0];
            ps.alias_offset = off;
            ps.alias_info = &cs.out_info[0];
            cs.preplaced[v] = 1;
          }
        }
        off += len;
      }
      bool any = false;
      for (char c : cs.preplaced) any = any || c;
      if (!any) cs.preplaced.clear();
    }
  }

  phase("elementwise_regions");
  // ---- horizontal fusion of sibling convs (GPU plans): CONV steps with the
  // same input slot, the same geometry and activation, constant filters (and
  // biases) and no epilogue chain become one step over the filters
  // concatenated along OC (at most kMaxOutSegs members per step). The merged
  // step runs where the first member ran: the others depend only on the same
  // input and on constants.
  if (gpu_plan && sibling_fusion_enabled()) {
    std::map<int, TensorRef> const_ref;
    for (auto& cs : p->const_slots) const_ref[cs.first] = cs.second;
    auto const_val = [&](int slot) -> const at::Tensor* {
      auto it = const_ref.find(slot);
      if (it == const_ref.end()) return nullptr;
      const auto& v = infos[it->second.node][it->second.index].value;
      return v ? &*v : nullptr;
    };
    std::map<std::pair<int, std::string>, std::vector<size_t>> groups;
    for (size_t i = 0; i < p->steps.size(); ++i) {
      const Step& st = p->steps[i];
      if (st.kind != Step::CONV || !st.epi.empty() || st.in_slots.size() != 2 || !st.sibs.empty()) continue;
      if (!(st.out_info[0].shape == st.gemm_shape) || !st.out_info[0].shape.fully_known()) continue;
      const Node& nd = g_->node(st.node);
      if (nd.op != "Conv2D" || nd.attr_s("data_format", std::string("NHWC")) != "NHWC") continue;
      const std::string pad = nd.attr_s("padding", std::string("VALID"));
      if (pad != "SAME" && pad != "VALID") continue;
      const at::Tensor* w = const_val(st.in_slots[1]);
      if (!w || w->dim() != 4 || w->scalar_type() != at::kFloat) continue;
      const at::Tensor* b = st.bias_slot >= 0 ? const_val(st.bias_slot) : nullptr;
      if (st.bias_slot >= 0 && (!b || b->scalar_type() != at::kFloat)) continue;
      std::string sig = pad;
      for (int64_t v : nd.attr_ilist("strides", {1, 1, 1, 1})) sig += "," + std::to_string(v);
      for (int64_t v : nd.attr_ilist("dilations", {1, 1, 1, 1})) sig += "," + std::to_string(v);
      for (int d = 0; d < 3; ++d) sig += "," + std::to_string(w->size(d));
      groups[{st.in_slots[0], sig}].push_back(i);
    }
    std::map<size_t, Step> merged_at;
    std::set<size_t> dropped;
    for (auto& kv : groups) {
      const auto& idx = kv.second;
      for (size_t g0 = 0; g0 + 1 < idx.size(); g0 += k::kMaxOutSegs) {
        const size_t g1 = std::min(idx.size(), g0 + k::kMaxOutSegs);
        if (g1 - g0 < 2) break;
        Step ms = p->steps[idx[g0]];
        ms.out_slots.clear();
        ms.out_info.clear();
        ms.alias_slot = -1;
        ms.act = 0;
        std::vector<at::Tensor> ws, bs;
        bool any_bias = false;
        for (size_t q = g0; q < g1; ++q) any_bias = any_bias || p->steps[idx[q]].bias_slot >= 0;
        for (size_t q = g0; q < g1; ++q) {
          const Step& m = p->steps[idx[q]];
          const at::Tensor* w = const_val(m.in_slots[1]);
          ws.push_back(*w);
          // members without a bias add zeros (e.g. the pool branch's conv, whose
          // bias follows the moved AvgPool: graph/rewrite.py)
          if (any_bias) bs.push_back(m.bias_slot >= 0 ? *const_val(m.bias_slot) : at::zeros({w->size(3)}, w->options()));
          ms.sibs.push_back({m.node, w->size(3), m.alias_slot, m.alias_offset, m.alias_info, m.act});
          ms.act = std::max(ms.act, m.act);  // > RELU6 selects the general epilogue
          ms.out_slots.push_back(m.out_slots[0]);
          ms.out_info.push_back(m.out_info[0]);
          if (q > g0) dropped.insert(idx[q]);
        }
        const int wslot = p->nslots++;
        p->synth_consts[wslot] = at::cat(ws, 3).contiguous();
        ms.in_slots[1] = wslot;
        ms.bias_slot = -1;
        if (any_bias) {
          const int bslot = p->nslots++;
          p->synth_consts[bslot] = at::cat(bs, 0).contiguous();
          ms.bias_slot = bslot;
        }
        merged_at[idx[g0]] = std::move(ms);
        p->fused_siblings += static_cast<int>(g1 - g0);
      }
    }
    if (!merged_at.empty()) {
      std::vector<Step> steps;
      for (size_t i = 0; i < p->steps.size(); ++i) {
        if (dropped.count(i)) continue;
        auto it = merged_at.find(i);
        steps.push_back(it != merged_at.end() ? std::move(it->second) : std::move(p->steps[i]));
      }
      p->steps = std::move(steps);
    }
  }

  // ---- Winograd filters (GPU plans): every 3x3 / 1x7 / 7x1 stride-1 CONV
  // step with a constant f32 filter and a cheap epilogue gets its F(2x2,3x3)
  // or F(2,7) transform
  // (fp64 on the host, once per plan) as a plan-made constant; the kernel
  // layer runs conv_wino.hip with it unless TFA_CONV_ALGO=direct
  if (gpu_plan && k::conv_wino_enabled()) {
    std::map<int, TensorRef> const_ref;
    for (auto& cs : p->const_slots) const_ref[cs.first] = cs.second;
    auto filt = [&](int slot) -> const at::Tensor* {
      auto sc = p->synth_consts.find(slot);
      if (sc != p->synth_consts.end()) return &sc->second;
      auto it = const_ref.find(slot);
      if (it == const_ref.end()) return nullptr;
      const auto& v = infos[it->second.node][it->second.index].value;
      return v ? &*v : nullptr;
    };
    std::map<int, int> made;  // filter slot -> Winograd slot (convs sharing a filter share it)
    for (auto& st : p->steps) {
      if (st.kind != Step::CONV || !st.epi.empty() || st.in_slots.size() != 2 || st.act > k::ACT_RELU6) continue;
      bool acts_ok = true;
      for (const auto& sb : st.sibs) acts_ok = acts_ok && sb.act <= k::ACT_RELU6;
      if (!acts_ok) continue;
      const Node& nd = g_->node(st.node);
      if (nd.op != "Conv2D" || nd.attr_s("data_format", std::string("NHWC")) != "NHWC") continue;
      const std::vector<int64_t> one{1, 1, 1, 1};
      const auto strides = nd.attr_ilist("strides", one), dil = nd.attr_ilist("dilations", one);
      if (strides != one || !(dil == one || dil.empty())) continue;
      const at::Tensor* w = filt(st.in_slots[1]);
      if (!w || w->dim() != 4 || w->scalar_type() != at::kFloat) continue;
      const int kind = k::conv_wino_kind(w->size(0), w->size(1), 1, 1, 1, 1, w->size(2), w->size(3));
      if (kind == 0) continue;
      auto hit = made.find(st.in_slots[1]);
      if (hit != made.end()) {
        st.wino_slot = hit->second;
        continue;
      }
      const at::Tensor wc = w->contiguous();
      at::Tensor u = at::empty({k::conv_wino_filter_elems(kind, wc.size(2), wc.size(3))}, wc.options());
      k::conv_wino_filter(kind, wc.data_ptr<float>(), wc.size(2), wc.size(3), u.data_ptr<float>());
      const int slot = p->nslots++;
      p->synth_consts[slot] = u;
      made[st.in_slots[1]] = slot;
      st.wino_slot = slot;
      ++p->wino_convs;
    }
  }
  phase("winograd");

  // ---- 2x2 / stride-2 VALID MaxPool after a Winograd 3x3 conv (VGG's
  // conv -> bias -> relu -> pool): the F(2x2,3x3) epilogue pools its own 2x2
  // output tiles and writes only the pooled tensor (the full-size activation
  // and the pool's read of it never reach HBM). The pool step goes away.
  if (gpu_plan && k::conv_wino_enabled() && conv_pool_fusion_enabled()) {
    std::map<int, size_t> reader;  // slot -> the only step reading it (or SIZE_MAX when several)
    for (size_t i = 0; i < p->steps.size(); ++i) {
      const Step& st = p->steps[i];
      std::vector<int> rd = st.in_slots;
      if (st.bias_slot >= 0) rd.push_back(st.bias_slot);
      for (auto& e : st.epi)
        if (e.slot >= 0) rd.push_back(e.slot);
      for (int sl : rd) {
        auto it = reader.find(sl);
        if (it == reader.end()) reader[sl] = i;
        else if (it->second != i) it->second = SIZE_MAX;
      }
    }
    std::set<int> fetch_set(p->fetch_slots.begin(), p->fetch_slots.end());
    std::set<size_t> gone;
    for (size_t i = 0; i < p->steps.size(); ++i) {
      Step& st = p->steps[i];
      if (st.kind != Step::CONV || st.wino_slot < 0 || !st.sibs.empty() || !st.epi.empty() || st.alias_slot >= 0 ||
          st.out_slots.size() != 1 || !(st.out_info[0].shape == st.gemm_shape))
        continue;
      const Shape& cs = st.out_info[0].shape;
      if (cs.rank() != 4 || !cs.fully_known() || cs.dims[1] % 2 || cs.dims[2] % 2) continue;
      const int oslot = st.out_slots[0];
      auto rit = reader.find(oslot);
      if (fetch_set.count(oslot) || rit == reader.end() || rit->second == SIZE_MAX || gone.count(rit->second)) continue;
      Step& ps = p->steps[rit->second];
      const Node& pn = g_->node(ps.node);
      const std::vector<int64_t> two{1, 2, 2, 1};
      if (ps.kind != Step::OP || pn.op != "MaxPool" || ps.in_slots.size() != 1 || ps.in_slots[0] != oslot ||
          ps.bias_slot >= 0 || ps.act != 0 || !ps.epi.empty() || ps.out_slots.size() != 1 ||
          pn.attr_ilist("ksize") != two || pn.attr_ilist("strides") != two ||
          pn.attr_s("padding", std::string("VALID")) != "VALID" ||
          pn.attr_s("data_format", std::string("NHWC")) != "NHWC")
        continue;
      const at::Tensor* w = nullptr;
      {
        auto sc = p->synth_consts.find(st.in_slots[1]);
        if (sc != p->synth_consts.end()) w = &sc->second;
        for (auto& cs2 : p->const_slots)
          if (!w && cs2.first == st.in_slots[1]) {
            const auto& v = infos[cs2.second.node][cs2.second.index].value;
            if (v) w = &*v;
          }
      }
      if (!w || w->dim() != 4 || w->size(0) != 3 || w->size(1) != 3) continue;
      st.pool2 = true;
      st.out_slots = ps.out_slots;
      st.out_info = ps.out_info;
      st.out_node = ps.out_node;
      st.gemm_shape = ps.out_info[0].shape;
      st.alias_slot = ps.alias_slot;
      st.alias_offset = ps.alias_offset;
      st.alias_info = ps.alias_info;
      gone.insert(rit->second);
      ++p->fused;
    }
    if (!gone.empty()) {
      std::vector<Step> steps;
      for (size_t i = 0; i < p->steps.size(); ++i)
        if (!gone.count(i)) steps.push_back(std::move(p->steps[i]));
      p->steps = std::move(steps);
    }
  }
  phase("conv_pool");

  // ---- 3x3 VALID MaxPool feeding only a 1x1 stride-1 conv (Inception-v3
  // MaxPool_3a -> Conv2d_3b): the conv reads the pool window maxima straight
  // from the pool's input (kernels/conv_smallc.hip pool_conv1x1), the pooled
  // tensor is never written. The pool step goes away.
  if (gpu_plan && pool_conv_fusion_state().load()) {
    std::map<int, size_t> reader, producer;
    for (size_t i = 0; i < p->steps.size(); ++i) {
      const Step& st = p->steps[i];
      std::vector<int> rd = st.in_slots;
      if (st.bias_slot >= 0) rd.push_back(st.bias_slot);
      for (auto& e : st.epi)
        if (e.slot >= 0) rd.push_back(e.slot);
      for (int sl : rd) {
        auto it = reader.find(sl);
        if (it == reader.end()) reader[sl] = i;
        else if (it->second != i) it->second = SIZE_MAX;
      }
      for (int sl : st.out_slots) producer[sl] = i;
    }
    std::set<int> fetch_set(p->fetch_slots.begin(), p->fetch_slots.end());
    std::set<size_t> gone;
    const std::vector<int64_t> one{1, 1, 1, 1};
    for (size_t i = 0; i < p->steps.size(); ++i) {
      Step& st = p->steps[i];
      if (st.kind != Step::CONV || st.wino_slot >= 0 || st.pool2 || !st.sibs.empty() || !st.epi.empty() ||
          st.in_slots.size() != 2 || st.out_slots.size() != 1 || st.act > k::ACT_RELU6)
        continue;
      const Node& nd = g_->node(st.node);
      if (nd.op != "Conv2D" || nd.attr_s("data_format", std::string("NHWC")) != "NHWC") continue;
      const auto dil = nd.attr_ilist("dilations", one);
      if (nd.attr_ilist("strides", one) != one || !(dil == one || dil.empty())) continue;
      const int xs = st.in_slots[0];
      auto pit = producer.find(xs);
      auto rit = reader.find(xs);
      if (pit == producer.end() || rit == reader.end() || rit->second != i || fetch_set.count(xs) ||
          gone.count(pit->second))
        continue;
      const at::Tensor* w = nullptr;
      for (auto& cs2 : p->const_slots)
        if (!w && cs2.first == st.in_slots[1]) {
          const auto& v = infos[cs2.second.node][cs2.second.index].value;
          if (v) w = &*v;
        }
      if (!w || w->dim() != 4 || w->size(0) != 1 || w->size(1) != 1 || w->scalar_type() != at::kFloat) continue;
      const int64_t C = w->size(2), OC = w->size(3);
      if (!(C == 16 || C == 32 || C == 64) || OC > 96) continue;
      Step& ps = p->steps[pit->second];
      const Node& pn = g_->node(ps.node);
      if (ps.kind != Step::OP || pn.op != "MaxPool" || ps.in_slots.size() != 1 || ps.bias_slot >= 0 ||
          ps.act != 0 || !ps.epi.empty() || ps.out_slots.size() != 1 || ps.alias_slot >= 0 ||
          pn.attr_s("padding", std::string("VALID")) != "VALID" ||
          pn.attr_s("data_format", std::string("NHWC")) != "NHWC")
        continue;
      const auto ks = pn.attr_ilist("ksize", one), ss = pn.attr_ilist("strides", one);
      if (ks.size() != 4 || ss.size() != 4 || ks[0] != 1 || ks[3] != 1 || ss[0] != 1 || ss[3] != 1 || ks[1] != 3 ||
          ks[2] != 3)
        continue;
      st.in_slots[0] = ps.in_slots[0];
      st.pool_in[0] = (int)ks[1];
      st.pool_in[1] = (int)ks[2];
      st.pool_in[2] = (int)ss[1];
      st.pool_in[3] = (int)ss[2];
      gone.insert(pit->second);
      ++p->fused;
    }
    if (!gone.empty()) {
      std::vector<Step> steps;
      for (size_t i = 0; i < p->steps.size(); ++i)
        if (!gone.count(i)) steps.push_back(std::move(p->steps[i]));
      p->steps = std::move(steps);
    }
  }
  phase("pool_conv");

  // liveness: release each slot after its last reading step (fetches/consts are kept)
  std::vector<int> last(p->nslots, -1);
  for (size_t i = 0; i < p->steps.size(); ++i) {
    for (int s : p->steps[i].in_slots) last[s] = static_cast<int>(i);
    if (p->steps[i].bias_slot >= 0) last[p->steps[i].bias_slot] = static_cast<int>(i);
    if (p->steps[i].wino_slot >= 0) last[p->steps[i].wino_slot] = static_cast<int>(i);
    for (auto& e : p->steps[i].epi)
      if (e.slot >= 0) last[e.slot] = static_cast<int>(i);
  }
  std::set<int> keep(p->fetch_slots.begin(), p->fetch_slots.end());
  for (auto& cs : p->const_slots) keep.insert(cs.first);
  for (auto& sc : p->synth_consts) keep.insert(sc.first);
  for (int s = 0; s < p->nslots; ++s)
    if (last[s] >= 0 && !keep.count(s)) p->steps[last[s]].release.push_back(s);
  phase("siblings+liveness");
  if (plan_timing) {
    std::string line = "[tfa plan]";
    for (auto& ph : phases) line += str_cat(" ", ph.first, "=", static_cast<int>(ph.second), "us");
    std::fprintf(stderr, "%s steps=%zu\n", line.c_str(), p->steps.size());
  }
  return p;
}

at::Tensor Program::device_const(Plan& p, int slot, const at::Device& dev, void* stream) {
  int di = dev.is_cuda() ? dev.index() : -1;
  std::lock_guard<std::mutex> lk(const_mu_);
  auto& m = p.dev_consts[di];
  auto it = m.find(slot);
  if (it != m.end()) return it->second;
  if (dev.is_cuda() && m.empty()) {
    upload_consts(p, m, dev, stream);
    it = m.find(slot);
    if (it != m.end()) return it->second;
  }
  TensorRef r{};
  for (auto& cs : p.const_slots)
    if (cs.first == slot) r = cs.second;
  // graph Const values are the same in every plan: one device copy per program
  // (plans differ per input shape, e.g. per image size in map_rows; the weights do not)
  const bool graph_const = g_->node(r.node).op == "Const";
  auto gkey = std::make_tuple(r.node, r.index, di);
  if (graph_const) {
    auto git = graph_consts_.find(gkey);
    if (git != graph_consts_.end()) {
      m[slot] = git->second;
      return git->second;
    }
  }
  const at::Tensor& v = *p.infos[r.node][r.index].value;
  // always a copy: constant values may be views of the GraphDef's bytes
  at::Tensor t = dev.is_cuda() ? v.contiguous().to(dev, /*non_blocking=*/false) : v.clone();
  m[slot] = t;
  if (graph_const) graph_consts_[gkey] = t;
  return t;
}

// All constants of a plan that are not already on the device go up in ONE
// host->device copy: they are packed (256-byte aligned) into a pinned staging
// buffer and the device arena is sliced into typed views. A program built per
// iteration (K-Means rebuilds its graph with new centres) then pays one
// transfer instead of one synchronous copy per constant, and the copy is
// asynchronous on the run's own stream (the host does not wait for the GPU to
// drain before every new program's first run); runs on other streams wait
// for its event (wait_consts).
void Program::upload_consts(Plan& p, std::map<int, at::Tensor>& m, const at::Device& dev, void* stream) {
  const int di = dev.index();
  struct Item {
    int slot;
    at::Tensor v;
    size_t off;
    bool graph_const;
    std::tuple<int, int, int> gkey;
  };
  std::vector<Item> items;
  size_t total = 0;
  for (auto& cs : p.const_slots) {
    const TensorRef& r = cs.second;
    const bool graph_const = g_->node(r.node).op == "Const";
    auto gkey = std::make_tuple(r.node, r.index, di);
    if (graph_const) {
      auto git = graph_consts_.find(gkey);
      if (git != graph_consts_.end()) {
        m[cs.first] = git->second;
        continue;
      }
    }
    const at::Tensor& v = *p.infos[r.node][r.index].value;
    if (v.numel() == 0) continue;  // the per-slot path makes the empty tensor
    at::Tensor c = v.contiguous();
    const size_t off = (total + 255) & ~size_t(255);
    total = off + c.nbytes();
    items.push_back({cs.first, c, off, graph_const, gkey});
  }
  if (items.empty()) return;
  at::Tensor host = at::empty({static_cast<int64_t>(total)},
                              at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  auto* hp = static_cast<uint8_t*>(host.data_ptr());
  for (auto& it : items) std::memcpy(hp + it.off, it.v.data_ptr(), it.v.nbytes());
  hipStream_t s = static_cast<hipStream_t>(stream);
  at::Tensor arena;
  {
    // copy_ on `s` records the staging block's use there (the pinned caching
    // host allocator keeps it until the copy has run)
    c10::hip::HIPStreamGuard sg(c10::hip::getStreamFromExternal(s, static_cast<c10::DeviceIndex>(di)));
    arena = at::empty({static_cast<int64_t>(total)}, at::TensorOptions().dtype(at::kByte).device(dev));
    arena.copy_(host, /*non_blocking=*/true);
  }
  void*& ev = const_events_[{di, stream}];
  if (!ev) {
    hipEvent_t e;
    TFA_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
    ev = e;
  }
  (void)hipEventRecord(static_cast<hipEvent_t>(ev), s);
  Plan::Arena ar;
  ar.dev = arena;
  for (auto& it : items) {
    at::Tensor t = arena.narrow(0, static_cast<int64_t>(it.off), static_cast<int64_t>(it.v.nbytes()))
                       .view(it.v.scalar_type())
                       .view(it.v.sizes());
    m[it.slot] = t;
    if (it.graph_const) graph_consts_[it.gkey] = t;
    TensorRef r{};
    for (auto& cs : p.const_slots)
      if (cs.first == it.slot) r = cs.second;
    ar.items.emplace_back(it.slot, r, it.off, it.v.nbytes());
  }
  p.arenas[di] = std::move(ar);
}

// caller holds const_mu_. Rewrites a plan's device constants with the values
// of its (adopted) graph: the arena is repacked in pinned memory and copied
// over itself asynchronously on `stream`, so every pointer into it (captured
// HIP graphs included) stays valid. A plan whose constants on this device do
// not all live in its own arena (some came from another plan's upload) drops
// them, and its capture, and uploads afresh.
void Program::refresh_consts(Plan& p, int di, void* stream) {
  p.stale.erase(di);
  auto& m = p.dev_consts[di];
  if (m.empty()) return;
  auto drop = [&]() {
    m.clear();
    p.arenas.erase(di);
    p.cap_reset = true;  // its capture read the old arena: run() discards it
  };
  if (di < 0) {  // host plan: the slots are clones, rebuilt from the new values
    m.clear();
    return;
  }
  auto ait = p.arenas.find(di);
  if (ait == p.arenas.end()) return drop();
  Plan::Arena& ar = ait->second;
  std::set<int> in_arena;
  for (auto& it : ar.items) in_arena.insert(std::get<0>(it));
  for (auto& kv : m)
    if (!in_arena.count(kv.first) && kv.second.numel() > 0) return drop();
  at::Tensor host = at::empty({ar.dev.numel()}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  auto* hp = static_cast<uint8_t*>(host.data_ptr());
  for (auto& it : ar.items) {
    const TensorRef& r = std::get<1>(it);
    const auto& v = p.infos[r.node][r.index].value;
    if (!v) return drop();
    at::Tensor c = v->contiguous();
    if (static_cast<size_t>(c.nbytes()) != std::get<3>(it)) return drop();
    std::memcpy(hp + std::get<2>(it), c.data_ptr(), c.nbytes());
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  // the previous runs and replays may still read the arena: the same stream
  // is ordered, every other stream they used is waited for
  for (void* us : p.used_streams[di])
    if (us && us != stream) (void)hipStreamSynchronize(static_cast<hipStream_t>(us));
  {
    c10::hip::HIPStreamGuard sg(c10::hip::getStreamFromExternal(s, static_cast<c10::DeviceIndex>(di)));
    ar.dev.copy_(host, /*non_blocking=*/true);
  }
  void*& ev = const_events_[{di, stream}];
  if (!ev) {
    hipEvent_t e;
    TFA_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
    ev = e;
  }
  (void)hipEventRecord(static_cast<hipEvent_t>(ev), s);
}

std::shared_ptr<Program> Program::rebind(const std::map<std::string, at::Tensor>& values) {
  static const bool timing = [] {
    const char* e = std::getenv("TFA_PLAN_TIMING");
    return e && std::string(e) == "3";
  }();
  const auto t0 = std::chrono::steady_clock::now();
  auto g = g_->with_values(values);
  const auto t1 = std::chrono::steady_clock::now();
  auto p = std::make_shared<Program>(std::move(g), fetch_names_, feed_names_);
  const auto t2 = std::chrono::steady_clock::now();
  p->adopt(*this);
  if (timing) {
    const auto t3 = std::chrono::steady_clock::now();
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    std::fprintf(stderr, "[tfa rebind] with_values %.1fus program %.1fus adopt %.1fus\n", us(t0, t1), us(t1, t2),
                 us(t2, t3));
  }
  return p;
}

bool Program::adopt(Program& old) {
  if (&old == this) return false;
  if (g_->structure_key() != old.g_->structure_key() || g_->nodes().size() != old.g_->nodes().size())
    return false;
  if (fetch_names_ != old.fetch_names_ || feed_names_ != old.feed_names_ || order_ != old.order_) return false;
  if (!host_op_error_.empty() || !old.host_op_error_.empty()) return false;
  std::scoped_lock lk(mu_, old.mu_, const_mu_, old.const_mu_);
  if (!plans_.empty()) return false;
  for (auto& kv : old.plans_) {
    if (!kv.second->synth_consts.empty()) return false;  // plan-made constants derive from the weights
    // a run of the old program still holds this plan (in flight, or about to
    // execute on another thread): its constants must not change under it.
    // Under old.mu_ no new reference can be handed out, so a count of one
    // means the map's is the only one.
    if (kv.second.use_count() != 1) return false;
  }
  // new values of every constant slot (the same nodes: equal structure);
  // shapes and dtypes must match (the parameter rule guarantees it)
  std::vector<std::pair<std::shared_ptr<Plan>, Graph::Infos>> fresh;
  // only the nodes the (changed) parameter constants reach are re-inferred;
  // every other node's info is the old plan's (same structure)
  const std::vector<char>& prm = g_->parameter_consts();
  std::vector<char> redo(g_->nodes().size(), 0);
  for (int n : order_) {
    char t = prm[n];
    for (auto& r : g_->node(n).inputs) t = t || redo[r.node];
    redo[n] = t;
  }
  for (auto& kv : old.plans_) {
    Plan& p = *kv.second;
    Graph::Infos ni = p.infos.size() == g_->nodes().size() ? g_->infer_update(order_, p.infos, redo, true)
                                                           : g_->infer(order_, p.feed_infos, true);
    for (auto& cs : p.const_slots) {
      const TensorRef& r = cs.second;
      const TensorInfo& a = p.infos[r.node][r.index];
      const TensorInfo& b = ni[r.node][r.index];
      if (a.dtype != b.dtype || a.shape.dims != b.shape.dims || !b.value || !a.value ||
          a.value->sizes() != b.value->sizes())
        return false;
    }
    fresh.emplace_back(kv.second, std::move(ni));
  }
  for (auto& [pp, ni] : fresh) {
    Plan& p = *pp;
    for (auto& cs : p.const_slots) {  // in place: steps hold pointers into p.infos
      const TensorRef& r = cs.second;
      p.infos[r.node][r.index].value = ni[r.node][r.index].value;
    }
    // every node the parameters reach takes the new values (the next adopt
    // starts from them); the others keep their base-graph values
    for (size_t n = 0; n < redo.size() && n < p.infos.size(); ++n)
      if (redo[n])
        for (size_t k = 0; k < p.infos[n].size() && k < ni[n].size(); ++k) p.infos[n][k].value = ni[n][k].value;
    for (auto& kv : p.dev_consts)
      if (!kv.second.empty()) p.stale.insert(kv.first);
  }
  plans_ = std::move(old.plans_);
  old.plans_.clear();
  old.graph_consts_.clear();  // its arenas belong to the moved plans now
  for (auto& kv : old.const_events_) {
    void*& ev = const_events_[kv.first];
    if (ev) (void)hipEventDestroy(static_cast<hipEvent_t>(ev));
    ev = kv.second;
  }
  old.const_events_.clear();
  stats_.plans_adopted += static_cast<int64_t>(plans_.size());
  return true;
}

// a run on `stream` reads constants uploaded on other streams: order it after
// those copies (completed uploads are forgotten, so steady state costs a map
// lookup). Inside the engine's own capture the capture stream already waits
// for the eager warm-up runs that uploaded everything.
void Program::wait_consts(const at::Device& dev, void* stream) {
  std::lock_guard<std::mutex> lk(const_mu_);
  if (const_events_.empty()) return;
  const int di = dev.index();
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (auto it = const_events_.begin(); it != const_events_.end();) {
    hipEvent_t e = static_cast<hipEvent_t>(it->second);
    if (it->first.first != di) {
      ++it;
      continue;
    }
    if (hipEventQuery(e) == hipSuccess) {
      (void)hipEventDestroy(e);
      it = const_events_.erase(it);
      continue;
    }
    if (it->first.second != stream && !dev_stream_capturing(s)) (void)hipStreamWaitEvent(s, e, 0);
    ++it;
  }
}

Program::~Program() {
  {
    std::lock_guard<std::mutex> lk(pipe_mu_);
    drop_pipe(false);
  }
  for (auto& kv : const_events_) (void)hipEventDestroy(static_cast<hipEvent_t>(kv.second));
}

std::vector<at::Tensor> Program::execute(Plan& p, const std::vector<at::Tensor>& inputs, void* stream) {
  const auto t_exec = std::chrono::steady_clock::now();
  // operands of a step's absorbed epilogue chain (contiguous, on the step's device)
  auto epi_steps = [](const Step& st, const std::vector<at::Tensor>& slots) {
    std::vector<EpiStep> ep;
    for (const auto& e : st.epi) {
      EpiStep x;
      x.code = e.code;
      x.kind = e.kind;
      x.act = e.act;
      x.s = e.s;
      if (e.slot >= 0) x.t = slots[e.slot].contiguous();
      ep.push_back(std::move(x));
    }
    return ep;
  };
  const OpRegistry& reg = OpRegistry::get();
  at::Device dev = inputs.empty() ? at::Device(at::kCPU) : inputs[0].device();
  bool gpu = dev.is_cuda();
  for (auto& t : inputs)
    TFA_CHECK(t.device() == dev, "all inputs must live on the same device");
  std::vector<at::Tensor> slots(p.nslots);
  for (size_t i = 0; i < inputs.size(); ++i) slots[p.feed_slots[i]] = inputs[i].contiguous();
  if (!p.stale.empty()) {
    std::lock_guard<std::mutex> lk(const_mu_);
    const int di = gpu ? dev.index() : -1;
    if (p.stale.count(di)) refresh_consts(p, di, stream);
  }
  for (auto& cs : p.const_slots) slots[cs.first] = device_const(p, cs.first, dev, stream);
  if (gpu) {
    wait_consts(dev, stream);
    std::lock_guard<std::mutex> lk(const_mu_);
    p.last_stream[dev.index()] = stream;
    if (!dev_stream_capturing(static_cast<hipStream_t>(stream))) p.used_streams[dev.index()].insert(stream);
  }
  for (auto& sc : p.synth_consts) {
    std::lock_guard<std::mutex> lk(const_mu_);
    auto& m = p.dev_consts[dev.is_cuda() ? dev.index() : -1];
    auto it = m.find(sc.first);
    if (it == m.end()) it = m.emplace(sc.first, dev.is_cuda() ? sc.second.to(dev) : sc.second).first;
    slots[sc.first] = it->second;
  }
  const bool timing = gpu && g_step_timing.load(std::memory_order_relaxed) &&
                      !dev_stream_capturing(static_cast<hipStream_t>(stream));
  for (auto& st : p.steps) {
    const Node& nd = g_->node(st.node);
    ExecCtx c{nd, {}, {}, &st.out_info, &st.in_info, gpu, stream};
    for (int s : st.in_slots) c.in.push_back(slots[s]);
    c.out.resize(st.out_info.size());
    StepRec rec;
    if (timing) {
      TFA_CHECK(hipEventCreate(&rec.a) == hipSuccess, "hipEventCreate failed");
      TFA_CHECK(hipEventCreate(&rec.b) == hipSuccess, "hipEventCreate failed");
      TFA_CHECK(hipEventRecord(rec.a, static_cast<hipStream_t>(stream)) == hipSuccess, "hipEventRecord failed");
    }
    {
      std::unique_ptr<RangeGuard> rg;
      if (gpu) rg = std::make_unique<RangeGuard>(nd.op + ":" + nd.name);
      try {
        if (st.kind == Step::FUSED) {
          TFA_CHECK(gpu, "internal: fused step in a host plan");
          Plan::Fused& fe = *p.fused_regions[st.fused];
          const int di = dev.index();
          jit::Kernel kern;
          {
            std::lock_guard<std::mutex> lk(fe.mu);
            auto kit = fe.kernels.find(di);
            if (kit == fe.kernels.end()) {
              hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
              (void)hipStreamIsCapturing(static_cast<hipStream_t>(stream), &cs);
              TFA_CHECK(cs == hipStreamCaptureStatusNone, "fused kernel not loaded before graph capture");
              kit = fe.kernels.emplace(di, jit::get(fe.region.source, fe.region.entry)).first;
            }
            kern = kit->second;
          }
          std::vector<void*> outs;
          for (size_t k = 0; k < st.out_slots.size(); ++k) {
            c.out[k] = c.alloc_out(static_cast<int>(k));
            outs.push_back(c.out[k].data_ptr());
          }
          std::vector<const void*> ptrs;
          for (size_t k = 0; k < c.in.size(); ++k) {
            if (!c.in[k].is_contiguous()) c.in[k] = materialize(c, c.in[k]);
            ptrs.push_back(c.in[k].data_ptr());
          }
          std::vector<int64_t> w = fused_args(fe.region, ptrs, outs);
          TFA_CHECK(fe.region.grid >= 1 && fe.region.grid < (int64_t(1) << 31), "fused kernel: grid out of range");
          jit::launch(kern, static_cast<unsigned>(fe.region.grid), fe.region.block, w.data(),
                      w.size() * sizeof(int64_t), static_cast<hipStream_t>(stream));
        } else if (st.kind == Step::OP && gpu && !st.preplaced.empty()) {
          // concat whose producers wrote in place: copy only the other inputs
          // (a nested concat's output is itself a slice of the outer concat)
          if (st.alias_slot >= 0) {
            at::Tensor& whole = slots[st.alias_slot];
            if (!whole.defined())
              whole = dev_empty(dims_or_throw(st.alias_info->shape, "concat output"), at::kFloat, dev,
                                static_cast<hipStream_t>(stream));
            slots[st.out_slots[0]] = whole.narrow(whole.dim() - 1, st.alias_offset, st.out_info[0].shape.dims.back());
          }
          at::Tensor& out = slots[st.out_slots[0]];
          TFA_CHECK(out.defined(), "internal: concat output not allocated by its producers");
          int64_t off = 0;
          const int64_t ax = out.dim() - 1;
          for (size_t v = 0; v < st.preplaced.size(); ++v) {
            const int64_t len = c.in[v].size(ax);
            if (!st.preplaced[v] && len > 0) gpu_copy(c.in[v], out.narrow(ax, off, len), stream_of(c));
            off += len;
          }
          c.out[0] = out;
        } else if (st.kind == Step::OP && gpu && (st.bias_slot >= 0 || st.act || st.alias_slot >= 0) &&
                   (nd.op == "AvgPool" || nd.op == "MaxPool")) {
          at::Tensor out;
          if (st.alias_slot >= 0) {
            at::Tensor& whole = slots[st.alias_slot];
            if (!whole.defined())
              whole = dev_empty(dims_or_throw(st.alias_info->shape, "concat output"), at::kFloat, dev,
                                static_cast<hipStream_t>(stream));
            out = whole.narrow(whole.dim() - 1, st.alias_offset, st.out_info[0].shape.dims.back());
          } else {
            out = c.alloc_out(0);
          }
          at::Tensor bias;
          if (st.bias_slot >= 0) bias = slots[st.bias_slot].contiguous();
          run_pool_fused(c, nd.op == "MaxPool", c.in[0], st.bias_slot >= 0 ? &bias : nullptr, st.act, out);
          c.out[0] = out;
        } else if (st.kind == Step::OP) {
          reg.find(nd.op)->compute(c);
        } else if (!st.sibs.empty()) {
          TFA_CHECK(gpu, "internal: sibling-fused conv in a host plan");
          std::vector<at::Tensor> outs;
          for (size_t k = 0; k < st.sibs.size(); ++k) {
            const Step::Sib& sb = st.sibs[k];
            if (sb.alias_slot >= 0) {
              at::Tensor& whole = slots[sb.alias_slot];
              if (!whole.defined())
                whole = dev_empty(dims_or_throw(sb.alias_info->shape, "concat output"), at::kFloat, dev,
                                  static_cast<hipStream_t>(stream));
              outs.push_back(whole.narrow(whole.dim() - 1, sb.alias_offset, sb.oc));
            } else {
              outs.push_back(c.alloc_out(static_cast<int>(k)));
            }
          }
          at::Tensor bias;
          if (st.bias_slot >= 0) bias = slots[st.bias_slot];
          std::vector<int> acts;
          for (const auto& sb : st.sibs) acts.push_back(sb.act);
          run_conv2d_siblings(c, c.in[0], c.in[1], st.bias_slot >= 0 ? &bias : nullptr, st.act, outs, acts,
                              st.wino_slot >= 0 ? &slots[st.wino_slot] : nullptr);
          for (size_t k = 0; k < outs.size(); ++k) c.out[k] = outs[k];
        } else if (gpu && st.alias_slot >= 0) {
          at::Tensor& whole = slots[st.alias_slot];
          if (!whole.defined())
            whole = dev_empty(dims_or_throw(st.alias_info->shape, "concat output"), at::kFloat, dev,
                              static_cast<hipStream_t>(stream));
          at::Tensor out = whole.narrow(whole.dim() - 1, st.alias_offset, st.out_info[0].shape.dims.back());
          at::Tensor bias;
          if (st.bias_slot >= 0) bias = slots[st.bias_slot];
          const at::Tensor* bp = st.bias_slot >= 0 ? &bias : nullptr;
          std::vector<EpiStep> ep = epi_steps(st, slots);
          const std::vector<EpiStep>* epp = ep.empty() ? nullptr : &ep;
          if (st.kind == Step::GEMM)
            run_gemm(c, c.in[0], c.in[1], gemm_ta(nd), gemm_tb(nd), bp, st.act, out,
                     epp);
          else
            run_conv2d(c, c.in[0], c.in[1], bp, st.act, out, epp, st.wino_slot >= 0 ? &slots[st.wino_slot] : nullptr,
                       st.pool2, st.pool_in[0] ? st.pool_in : nullptr);
          c.out[0] = out;
        } else {
          at::Tensor out = gpu ? c.alloc_out(0) : at::Tensor();
          // absorbed views: the kernel writes the MatMul/Conv2D shape, the step
          // hands out the same elements in the view's shape
          const bool viewed = !(st.out_info[0].shape == st.gemm_shape);
          at::Tensor kout = (gpu && viewed) ? out.view(st.gemm_shape.dims) : out;
          at::Tensor bias;
          if (st.bias_slot >= 0) bias = slots[st.bias_slot];
          const at::Tensor* bp = st.bias_slot >= 0 ? &bias : nullptr;
          std::vector<EpiStep> ep = epi_steps(st, slots);
          const std::vector<EpiStep>* epp = ep.empty() ? nullptr : &ep;
          if (st.kind == Step::GEMM)
            run_gemm(c, c.in[0], c.in[1], gemm_ta(nd), gemm_tb(nd), bp, st.act,
                     kout, epp);
          else
            run_conv2d(c, c.in[0], c.in[1], bp, st.act, kout, epp, st.wino_slot >= 0 ? &slots[st.wino_slot] : nullptr,
                       st.pool2, st.pool_in[0] ? st.pool_in : nullptr);
          c.out[0] = viewed ? kout.reshape(st.out_info[0].shape.dims) : kout;
        }
      } catch (const GraphError& e) {
        throw GraphError(str_cat("while executing node '", nd.name, "' (", nd.op, "): ", e.what()));
      }
    }
    if (gpu) {
      // launch errors are reported with the node that caused them (a HIP fault
      // is sticky: the caller must not retry in this process); debug_sync also
      // waits for the kernel so asynchronous faults are attributed too
      hipError_t le = hipGetLastError();
      if (le == hipSuccess && debug_sync()) {
        le = hipStreamSynchronize(static_cast<hipStream_t>(stream));
        if (le == hipSuccess) le = hipGetLastError();
      }
      TFA_CHECK(le == hipSuccess, "HIP error ", hipGetErrorString(le), " (", hipGetErrorName(le),
                ") in node '", nd.name, "' (", nd.op, ")");
    }
    for (size_t k = 0; k < st.out_slots.size(); ++k) {
      at::Tensor& o = c.out[k];
      TFA_CHECK(o.defined(), "internal: node '", nd.name, "' produced no output ", k);
      const Shape& want = st.out_info[k].shape;
      TFA_CHECK(want.fully_known() && o.sizes().vec() == want.dims, "internal: node '", nd.name,
                "' produced shape ", shape_of(o).str(), " but inference said ", want.str());
      slots[st.out_slots[k]] = o;
    }
    if (timing) {
      TFA_CHECK(hipEventRecord(rec.b, static_cast<hipStream_t>(stream)) == hipSuccess, "hipEventRecord failed");
      rec.node = g_->node(st.out_node >= 0 ? st.out_node : st.node).name;
      rec.op = nd.op;
      // the least HBM traffic the step can do: its operands once in, its outputs once out
      for (auto& t : c.in)
        if (t.defined()) rec.bytes += static_cast<double>(t.numel()) * t.element_size();
      for (auto& t : c.out)
        if (t.defined()) rec.bytes += static_cast<double>(t.numel()) * t.element_size();
      if (st.kind == Step::CONV || st.kind == Step::GEMM) {
        // 2 * output elements * reduction length, summed over sibling outputs
        int64_t outs_n = 0;
        for (auto& o : c.out) outs_n += o.numel();
        if (st.pool2) outs_n *= 4;  // the conv's own outputs, before the fused pool
        int64_t red = 0;
        if (st.kind == Step::CONV) {
          const at::Tensor& f = c.in[1];
          red = f.dim() == 4 ? f.size(0) * f.size(1) * f.size(2) : 0;
        } else {
          const at::Tensor& a = c.in[0];
          red = a.dim() >= 2 ? (gemm_ta(nd) ? a.size(a.dim() - 2) : a.size(a.dim() - 1)) : 0;
        }
        rec.flops = 2.0 * static_cast<double>(outs_n) * static_cast<double>(red);
        rec.label = st.kind == Step::GEMM ? std::string("gemm") + k::last_f32_tile() : std::string(k::last_conv_algo());
        if (!st.sibs.empty()) rec.label += str_cat("+siblings", st.sibs.size());
      } else {
        rec.label = st.kind == Step::FUSED ? "fused" : "op";
      }
      std::lock_guard<std::mutex> lk(g_step_mu);
      g_step_recs.push_back(std::move(rec));
    }
    for (int s : st.release) slots[s] = at::Tensor();
    stats_.kernels++;
  }
  std::vector<at::Tensor> outs;
  for (int s : p.fetch_slots) outs.push_back(slots[s]);
  stats_.exec_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_exec).count();
  return outs;
}

// HIP graphs: a plan that keeps being run with small inputs is launch-bound;
// after kGraphWarmRuns ordinary runs its kernel sequence is captured once and
// replayed (inputs copied into static buffers, outputs cloned out). A replay
// has a fixed cost (input copy, graph launch, output clone: ~80-150 us on
// MI355X, scripts/map_rows_overhead.py), so only plans of at least
// kGraphMinSteps kernels are captured: a 5-kernel image-preprocessing plan
// runs in 25 us eager vs 85-160 us replayed, a 40-op elementwise chain in
// 440 us eager vs 190 us replayed. The first kGraphProbeRuns replays are also
// timed (host side) against the warm eager runs and the graph is dropped when
// replaying costs more. TFA_HIP_GRAPHS: 1 (default) adaptive, 2 always
// replay (any size), 0 never. Inputs up to TFA_HIP_GRAPH_MAX_BYTES.
namespace {
constexpr int64_t kGraphWarmRuns = 3;
constexpr int64_t kGraphProbeRuns = 5;
constexpr size_t kGraphMinSteps = 16;
int hip_graphs_mode() {
  static const int mode = [] {
    const char* e = std::getenv("TFA_HIP_GRAPHS");
    if (!e) return 1;
    const std::string v(e);
    return v == "0" ? 0 : (v == "2" ? 2 : 1);
  }();
  return (debug_sync() || g_step_timing.load()) ? 0 : mode;  // step timing needs the eager path
}
bool hip_graphs_enabled() { return hip_graphs_mode() != 0; }
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
int64_t hip_graph_max_bytes() {
  static const int64_t v = env_positive("TFA_HIP_GRAPH_MAX_BYTES", int64_t(16) << 20);
  return v;
}
}  // namespace

bool Program::graphable(const Plan& p) const { return graph_blocker(p).empty(); }

void set_step_timing(bool on) { g_step_timing.store(on); }
bool step_timing() { return g_step_timing.load(); }

std::vector<StepTiming> read_step_timing() {
  std::vector<StepRec> recs;
  {
    std::lock_guard<std::mutex> lk(g_step_mu);
    recs.swap(g_step_recs);
  }
  std::vector<StepTiming> out;
  for (auto& r : recs) {
    float ms = 0;
    TFA_CHECK(hipEventSynchronize(r.b) == hipSuccess, "hipEventSynchronize failed");
    TFA_CHECK(hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess, "hipEventElapsedTime failed");
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
    out.push_back({r.node, r.op, r.label, r.flops, r.bytes, ms});
  }
  return out;
}

// why a plan cannot be captured into a HIP graph ("" = it can)
std::string Program::graph_blocker(const Plan& p) const {
  // every plan-time (host) input must be a known constant: a data-dependent
  // one would need a device->host sync, which a capture cannot contain
  static const std::set<std::string> kRuntimeHostCopies = {
      "FusedBatchNorm", "FusedBatchNormV2", "FusedBatchNormV3", "Shape", "Size", "Rank"};
  const OpRegistry& reg = OpRegistry::get();
  for (auto& st : p.steps) {
    const std::string& op = g_->node(st.node).op;
    const std::string& nm = g_->node(st.node).name;
    if (kRuntimeHostCopies.count(op)) return str_cat(op, " '", nm, "' copies host data at run time");
    // a fused region / GEMM / conv step launches generated or fixed kernels
    // on device operands only: its op's host inputs were consumed at plan time
    if (st.kind != Step::OP) continue;
    const OpDef* od = reg.find(op);
    if (!od) return str_cat(op, " '", nm, "' has no registered op");
    for (int hi : od->host_inputs) {
      if (hi < 0 || hi >= static_cast<int>(st.in_info.size())) continue;
      if (!st.in_info[hi]->value) return str_cat(op, " '", nm, "': host input ", hi, " is not a plan-time constant");
    }
    // scalar operands read on the host at run time when not constant
    if (op == "Fill" && st.in_info.size() > 1 && !st.in_info[1]->value)
      return str_cat("Fill '", nm, "': value read on the host");
  }
  return p.steps.empty() ? "no steps" : "";
}

namespace {
// the outputs of a replay leave the graph's static buffers in ONE batched-copy
// launch into one pool buffer (the outputs are views of it) instead of one
// DMA call per output: a K-Means partition run returns 4 small outputs
std::vector<at::Tensor> clone_outputs(const std::vector<at::Tensor>& outs, hipStream_t s) {
  std::vector<at::Tensor> r;
  r.reserve(outs.size());
  if (outs.size() < 2 || outs.size() > static_cast<size_t>(k::kMaxCopyPieces)) {
    for (auto& o : outs) r.push_back(dev_clone(o.contiguous(), s));
    return r;
  }
  std::vector<at::Tensor> src;
  std::vector<int64_t> off;
  int64_t total = 0;
  for (auto& o : outs) {
    src.push_back(o.contiguous());
    off.push_back(total);
    total += (src.back().numel() * src.back().element_size() + 255) / 256 * 256;
  }
  at::Tensor buf = dev_empty({std::max<int64_t>(total, 1)}, at::kByte, outs[0].device(), s);
  k::CopyPieces pc;
  for (size_t i = 0; i < src.size(); ++i) {
    const int64_t nb = src[i].numel() * src[i].element_size();
    if (!nb) continue;
    pc.src[pc.n] = src[i].data_ptr();
    pc.dst_off[pc.n] = off[i];
    pc.bytes[pc.n] = nb;
    pc.n++;
  }
  k::batched_copy(pc, buf.data_ptr(), s);
  for (size_t i = 0; i < src.size(); ++i) {
    const int64_t nb = src[i].numel() * src[i].element_size();
    r.push_back(buf.narrow(0, off[i], nb).view(src[i].scalar_type()).view(src[i].sizes()));
  }
  return r;
}
}  // namespace

std::vector<at::Tensor> Program::run_graph(Plan& p, const std::vector<at::Tensor>& inputs) {
  auto& c = p.cap;  // caller holds c.mu
  const int dev = inputs[0].device().index();
  hipStream_t cur = c10::hip::getCurrentHIPStream(dev).stream();
  if (!c.graph) {
    c.device = dev;
    TFA_CHECK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) == hipSuccess, "hipStreamCreate failed");
    auto side = c10::hip::getStreamFromExternal(c.stream, dev);
    for (auto& t : inputs) c.static_in.push_back(at::empty_like(t, at::MemoryFormat::Contiguous));
    // static inputs hold valid data before the capture stream reads them
    {
      c10::hip::HIPStreamGuard sg(c10::hip::getCurrentHIPStream(dev));
      for (size_t i = 0; i < inputs.size(); ++i) c.static_in[i].copy_(inputs[i], true);
    }
    hipEvent_t ev;
    TFA_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
    (void)hipEventRecord(ev, cur);
    (void)hipStreamWaitEvent(c.stream, ev, 0);
    (void)hipEventDestroy(ev);
    auto g = std::make_unique<HipGraph>();
    try {
      c10::hip::HIPStreamGuard sg(side);
      g->begin(c.stream, dev);
      c.static_out = execute(p, c.static_in, c.stream);
      g->end();
    } catch (const std::exception& e) {
      // the capture is discarded and the plan runs eagerly from now on
      g->abort();
      c.failed = true;
      c.static_in.clear();
      c.static_out.clear();
      g.release();  // its pool may still back tensors of the failed capture; leak it
      stats_.graph_failures++;
      return execute(p, inputs, cur);
    }
    c.graph = std::move(g);
    // the capture stream's work (none executed yet) is ordered before replays on `cur`
    stats_.graphs_captured++;
  }
  c.order.before(cur);  // the last replay (maybe on another stream) is done with the buffers
  for (size_t i = 0; i < inputs.size(); ++i) c.static_in[i].copy_(inputs[i], true);
  wait_consts(inputs[0].device(), cur);
  {
    std::lock_guard<std::mutex> cl(const_mu_);
    p.used_streams[dev].insert(cur);
  }
  // the replay is ordered after the input copies on the caller's stream
  c.graph->replay(cur);
  // replay outputs are copied out of the graph's static buffers
  std::vector<at::Tensor> outs = clone_outputs(c.static_out, cur);
  c.order.after(cur);
  stats_.graph_replays++;
  return outs;
}

namespace {
constexpr int kPtrWarmRuns = 2;       // eager runs of a pointer set before it is captured
constexpr size_t kPtrMinSteps = 3;    // no input copies: worth it from a few kernels on
constexpr size_t kPtrMaxCaps = 8;     // captures per plan (each owns its intermediates)
constexpr size_t kPtrMaxSeen = 32;
int64_t ptr_graph_max_bytes() {
  static const int64_t v = env_positive("TFA_HIP_GRAPH_PTR_MAX_BYTES", int64_t(256) << 20);
  return v;
}
}  // namespace

std::optional<std::vector<at::Tensor>> Program::run_ptr_graph(Plan& p, const std::vector<at::Tensor>& inputs,
                                                               int64_t bytes) {
  if (hip_graphs_mode() != 1 || p.ptr_declined || p.cap_reset || bytes > ptr_graph_max_bytes() ||
      p.steps.size() < kPtrMinSteps || inputs.empty())
    return std::nullopt;
  for (auto& t : inputs)
    if (!t.is_cuda() || !t.is_contiguous()) return std::nullopt;
  std::vector<const void*> key;
  key.reserve(inputs.size());
  for (auto& t : inputs) key.push_back(t.data_ptr());
  std::lock_guard<std::mutex> lk(p.ptr_mu);
  const int dev = inputs[0].device().index();
  hipStream_t cur = c10::hip::getCurrentHIPStream(dev).stream();
  auto it = p.ptr_caps.find(key);
  Plan::PtrCap* use = nullptr;
  if (it != p.ptr_caps.end()) {
    for (auto& c : it->second)
      if (!c->cloning && c->outputs_free()) use = c.get();
    if (!use)
      for (auto& c : it->second)
        if (c->cloning) use = c.get();
  }
  const bool cloning = it != p.ptr_caps.end() && (use ? use->cloning : true);
  if (!use) {
    if (it == p.ptr_caps.end()) {
      int& seen = p.ptr_seen[key];
      if (p.ptr_seen.size() > kPtrMaxSeen) {  // a stream of fresh pointers: not an iterative workload
        p.ptr_seen.clear();
        return std::nullopt;
      }
      if (++seen <= kPtrWarmRuns || !graphable(p)) {
        if (seen > 1) {  // warm eager run: the baseline a replay must beat
          const int64_t t0 = now_ns();
          auto outs = execute(p, inputs, cur);
          p.ptr_eager_ns += now_ns() - t0;
          p.ptr_eager_n++;
          return outs;
        }
        return std::nullopt;
      }
    }
    // capture on a private stream, on the caller's own tensors
    size_t total = 0;
    for (auto& kv : p.ptr_caps) total += kv.second.size();
    if (total >= kPtrMaxCaps) {  // evict the least recently used instance
      std::vector<std::unique_ptr<Plan::PtrCap>>* lv = nullptr;
      size_t li = 0;
      int64_t best = INT64_MAX;
      for (auto& kv : p.ptr_caps)
        for (size_t i = 0; i < kv.second.size(); ++i)
          if (kv.second[i]->last_use < best) {
            best = kv.second[i]->last_use;
            lv = &kv.second;
            li = i;
          }
      if (lv) {
        auto& victim = (*lv)[li];
        if (victim->stream) (void)hipStreamSynchronize(victim->stream);
        victim->order.drain();  // its replays are done before its pool goes
        lv->erase(lv->begin() + static_cast<long>(li));
        for (auto j = p.ptr_caps.begin(); j != p.ptr_caps.end();)
          j = j->second.empty() ? p.ptr_caps.erase(j) : std::next(j);
      }
    }
    auto pc = std::make_unique<Plan::PtrCap>();
    TFA_CHECK(hipStreamCreateWithFlags(&pc->stream, hipStreamNonBlocking) == hipSuccess, "hipStreamCreate failed");
    hipEvent_t ev;
    TFA_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
    (void)hipEventRecord(ev, cur);
    (void)hipStreamWaitEvent(pc->stream, ev, 0);
    (void)hipEventDestroy(ev);
    auto g = std::make_unique<HipGraph>();
    try {
      c10::hip::HIPStreamGuard sg(c10::hip::getStreamFromExternal(pc->stream, dev));
      g->begin(pc->stream, dev);
      pc->static_out = execute(p, inputs, pc->stream);
      g->end();
    } catch (const std::exception&) {
      g->abort();
      g.release();  // its pool may back tensors of the failed capture; leak it
      p.ptr_declined = true;
      stats_.graph_failures++;
      return std::nullopt;
    }
    pc->graph = std::move(g);
    pc->cloning = cloning;
    for (auto& o : pc->static_out) {
      bool in_alias = false;
      for (auto& t : inputs) in_alias = in_alias || o.storage().is_alias_of(t.storage());
      pc->input_alias.push_back(in_alias);
      pc->base_uc.push_back(o.storage().use_count());
    }
    stats_.graphs_captured++;
    use = pc.get();
    if (!pc->cloning) register_aliases(pc.get(), alias_ptrs(pc->static_out, pc->input_alias));
    p.ptr_caps[key].push_back(std::move(pc));
    p.ptr_seen.erase(key);
  }
  use->last_use = ++p.ptr_tick;
  const int64_t t0 = now_ns();
  wait_consts(inputs[0].device(), cur);  // a refresh on another stream lands first
  {
    std::lock_guard<std::mutex> cl(const_mu_);
    p.used_streams[dev].insert(cur);
  }
  use->order.before(cur);
  use->wait_uses(cur);  // readers of the previous aliases on other streams
  use->graph->replay(cur);
  use->order.after(cur);
  std::vector<at::Tensor> outs;
  if (use->cloning) {
    outs = clone_outputs(use->static_out, cur);
    stats_.graph_busy++;
  } else {
    outs.reserve(use->static_out.size());
    for (auto& o : use->static_out) outs.push_back(o.alias());  // no copy: see PtrCap
  }
  stats_.graph_replays++;
  // the first replays are timed against the warm eager runs; a plan whose
  // replays cost more host time than launching its kernels keeps running eagerly
  if (p.ptr_eager_n > 0 && p.ptr_replay_n < kGraphProbeRuns) {
    p.ptr_replay_ns += now_ns() - t0;
    if (++p.ptr_replay_n == kGraphProbeRuns && p.ptr_replay_ns * p.ptr_eager_n > p.ptr_eager_ns * p.ptr_replay_n) {
      p.ptr_declined = true;
      stats_.graphs_declined++;
    }
  }
  return outs;
}

namespace {
// engine side streams and fork/join events per device (created once, never
// destroyed: runs may outlive static teardown)
struct SideStreams {
  std::mutex mu;
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> events;  // [0]: fork; [1]: previous caller; [2 + i]: join of stream i
  hipStream_t last_caller = nullptr;
};
SideStreams& side_streams(int dev) {
  static std::mutex m;
  static std::map<int, SideStreams*> all;
  std::lock_guard<std::mutex> lk(m);
  auto& p = all[dev];
  if (!p) p = new SideStreams();
  return *p;
}
}  // namespace

std::vector<std::vector<at::Tensor>> Program::run_concurrent(
    const std::vector<std::vector<at::Tensor>>& inputs_list, int max_streams) {
  std::vector<std::vector<at::Tensor>> outs;
  if (inputs_list.empty()) return outs;
  TFA_CHECK(!inputs_list[0].empty() && inputs_list[0][0].is_cuda(), "run_concurrent: device inputs expected");
  const int dev = inputs_list[0][0].device().index();
  for (auto& ins : inputs_list)
    for (auto& t : ins)
      TFA_CHECK(t.is_cuda() && t.device().index() == dev, "run_concurrent: all inputs on one device");
  const int k = std::max(1, std::min<int>(max_streams, static_cast<int>(inputs_list.size())));
  c10::hip::HIPGuard guard(dev);
  const hipStream_t caller = c10::hip::getCurrentHIPStream(dev).stream();
  SideStreams& ss = side_streams(dev);
  std::lock_guard<std::mutex> lk(ss.mu);  // one fork/join at a time per device (events are shared)
  while (static_cast<int>(ss.streams.size()) < k) {
    hipStream_t st;
    TFA_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess, "run_concurrent: hipStreamCreate");
    ss.streams.push_back(st);
  }
  while (ss.events.size() < ss.streams.size() + 2) {
    hipEvent_t e;
    TFA_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "run_concurrent: hipEventCreate");
    ss.events.push_back(e);
  }
  // Fork: every side stream waits for the caller's work so far. Outputs made
  // on side stream i go back to ITS free list in the pool when the caller
  // drops them; only these private streams allocate from those lists, and
  // only after such a fork, so a reuse is ordered after every read the caller
  // queued before dropping them -- no per-block stream records (an event per
  // freed block cost more host time than the overlap saved). A call from a
  // different caller stream also waits for the previous caller's work.
  TFA_CHECK(hipEventRecord(ss.events[0], caller) == hipSuccess, "run_concurrent: hipEventRecord");
  const bool other_caller = ss.last_caller && ss.last_caller != caller;
  if (other_caller)
    TFA_CHECK(hipEventRecord(ss.events[1], ss.last_caller) == hipSuccess, "run_concurrent: hipEventRecord");
  for (int i = 0; i < k; ++i) {
    TFA_CHECK(hipStreamWaitEvent(ss.streams[i], ss.events[0], 0) == hipSuccess, "run_concurrent: hipStreamWaitEvent");
    if (other_caller)
      TFA_CHECK(hipStreamWaitEvent(ss.streams[i], ss.events[1], 0) == hipSuccess, "run_concurrent: hipStreamWaitEvent");
  }
  ss.last_caller = caller;
  outs.reserve(inputs_list.size());
  for (size_t i = 0; i < inputs_list.size(); ++i) {
    // partition i always runs on side stream i % k: its zero-copy replay
    // instance keeps one stream across calls (no cross-stream drain)
    const hipStream_t st = ss.streams[i % k];
    c10::hip::HIPStreamGuard sg(c10::hip::getStreamFromExternal(st, static_cast<c10::DeviceIndex>(dev)));
    outs.push_back(run(inputs_list[i]));
  }
  // Join: the caller's stream waits for every side stream (its later
  // allocations, which may reuse the inputs' blocks, and its reads of the
  // outputs are ordered after the side-stream work)
  for (int i = 0; i < k; ++i) {
    TFA_CHECK(hipEventRecord(ss.events[2 + i], ss.streams[i]) == hipSuccess, "run_concurrent: hipEventRecord");
    TFA_CHECK(hipStreamWaitEvent(caller, ss.events[2 + i], 0) == hipSuccess, "run_concurrent: hipStreamWaitEvent");
  }
  return outs;
}

std::vector<at::Tensor> Program::run(const std::vector<at::Tensor>& inputs) {
  TFA_CHECK(host_op_error_.empty(), host_op_error_);
  auto p = plan_for(inputs);
  bool gpu = !inputs.empty() && inputs[0].is_cuda();
  void* stream = nullptr;
  std::optional<c10::hip::HIPGuard> guard;
  if (gpu) {
    guard.emplace(inputs[0].device().index());
    stream = c10::hip::getCurrentHIPStream(inputs[0].device().index()).stream();
    if (!p->stale.empty()) {  // before a replay, which reads the arena without execute()
      std::lock_guard<std::mutex> lk(const_mu_);
      if (p->stale.count(inputs[0].device().index())) refresh_consts(*p, inputs[0].device().index(), stream);
    }
    if (hip_graphs_enabled()) {
      int64_t bytes = 0;
      for (auto& t : inputs) bytes += t.numel() * t.element_size();
      if (auto outs = run_ptr_graph(*p, inputs, bytes)) {
        stats_.runs++;
        return std::move(*outs);
      }
      auto& c = p->cap;
      std::lock_guard<std::mutex> lk(c.mu);
      if (p->cap_reset) {
        p->cap_reset = false;
        {
          std::lock_guard<std::mutex> pl(p->ptr_mu);
          for (auto& kv : p->ptr_caps)
            for (auto& pc : kv.second)
              if (pc->stream) (void)hipStreamSynchronize(pc->stream);
          p->ptr_caps.clear();
          p->ptr_seen.clear();
        }
        if (c.graph) {
          if (c.stream) (void)hipStreamSynchronize(c.stream);
          c.order.drain();
          c.graph.reset();
          c.static_in.clear();
          c.static_out.clear();
        }
        c.gpu_runs = 0;
        c.eager_ns = c.eager_n = c.replay_ns = c.replay_n = 0;
      }
      const bool same_dev = c.device < 0 || c.device == inputs[0].device().index();
      const bool big_enough = hip_graphs_mode() == 2 || p->steps.size() >= kGraphMinSteps;
      if (!c.failed && !c.declined && same_dev && big_enough && bytes <= hip_graph_max_bytes() && graphable(*p)) {
        if (++c.gpu_runs > kGraphWarmRuns) {
          const bool captured = c.graph != nullptr;
          const int64_t t0 = now_ns();
          auto outs = run_graph(*p, inputs);
          if (captured && c.graph && hip_graphs_mode() == 1 && c.eager_n > 0) {
            c.replay_ns += now_ns() - t0;
            if (++c.replay_n == kGraphProbeRuns && c.replay_ns * c.eager_n > c.eager_ns * c.replay_n) {
              c.declined = true;  // eager launches are cheaper for this plan
              stats_.graphs_declined++;
            }
          }
          stats_.runs++;
          return outs;
        }
        if (c.gpu_runs > 1) {  // warm eager runs (the first one uploads constants)
          const int64_t t0 = now_ns();
          auto outs = execute(*p, inputs, stream);
          c.eager_ns += now_ns() - t0;
          c.eager_n++;
          stats_.runs++;
          return outs;
        }
      }
    }
  }
  auto outs = execute(*p, inputs, stream);
  stats_.runs++;
  return outs;
}

// The pipeline rings come from pool blocks cached for the compute stream:
// compute-stream work queued before this call (an earlier partition's last
// chunk) may still read them. The copy stream's first writes wait for it.
static void order_copy_after_compute(hipStream_t copy, hipStream_t compute) {
  hipEvent_t e;
  HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipEventRecord(e, compute));
  HIP_OK(hipStreamWaitEvent(copy, e, 0));
  HIP_OK(hipEventDestroy(e));
}

void Program::drop_pipe(bool synced) {
  if (!pipe_) return;
  if (pipe_->device >= 0) {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(pipe_->device));
    if (!synced) {
      (void)hipStreamSynchronize(copy_stream(pipe_->device, 0));
      (void)hipStreamSynchronize(copy_stream(pipe_->device, 1));
      (void)hipDeviceSynchronize();  // the compute streams that read the ring
    }
    for (hipEvent_t e : pipe_->ev_comp) (void)hipEventDestroy(e);
    for (hipEvent_t e : pipe_->ev_d2h) (void)hipEventDestroy(e);
  }
  pipe_.reset();
}

void pipeline_wait(int64_t handle) {
  if (!handle) return;
  hipEvent_t e = reinterpret_cast<hipEvent_t>(handle);
  HIP_OK(hipEventSynchronize(e));
  HIP_OK(hipEventDestroy(e));
}

int64_t Program::run_chunked(const std::vector<std::vector<at::Tensor>>& seg_inputs,
                             const std::vector<std::vector<at::Tensor>>& seg_outputs,
                             int64_t chunk_rows, int device, int depth, bool wait) {
  TFA_CHECK(host_op_error_.empty(), host_op_error_);
  TFA_CHECK(seg_inputs.size() == seg_outputs.size(), "segments mismatch");
  TFA_CHECK(chunk_rows > 0, "chunk_rows must be > 0");
  depth = std::max(2, std::min(depth, 4));
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  at::Device dev(at::kCUDA, static_cast<c10::DeviceIndex>(device));
  auto compute = c10::hip::getCurrentHIPStream(device);
  // the runtime's own copy streams (one per direction per device): the DMA
  // engines run both directions concurrently, overlapped with compute
  auto h2d = c10::hip::getStreamFromExternal(copy_stream(device, 0), static_cast<c10::DeviceIndex>(device));
  auto d2h = c10::hip::getStreamFromExternal(copy_stream(device, 1), static_cast<c10::DeviceIndex>(device));
  auto t0 = std::chrono::steady_clock::now();

  struct Chunk {
    size_t seg;
    int64_t start, rows;
  };
  std::vector<Chunk> chunks;
  for (size_t s = 0; s < seg_inputs.size(); ++s) {
    TFA_CHECK(seg_inputs[s].size() == feed_nodes_.size(), "segment ", s, ": expected ",
              feed_nodes_.size(), " inputs");
    TFA_CHECK(seg_outputs[s].size() == fetches_.size(), "segment ", s, ": expected ",
              fetches_.size(), " outputs");
    int64_t rows = seg_inputs[s].empty() ? 0 : seg_inputs[s][0].size(0);
    for (auto& t : seg_inputs[s]) {
      TFA_CHECK(t.size(0) == rows, "segment inputs disagree on rows");
      TFA_CHECK(!t.is_cuda() && t.is_contiguous(), "run_chunked inputs must be contiguous host tensors");
    }
    for (auto& t : seg_outputs[s])
      TFA_CHECK(!t.is_cuda() && t.is_contiguous() && t.size(0) == rows,
                "run_chunked outputs must be contiguous host tensors with ", rows, " rows");
    for (int64_t st = 0; st < rows; st += chunk_rows) chunks.push_back({s, st, std::min(chunk_rows, rows - st)});
  }
  if (chunks.empty()) return 0;
  std::lock_guard<std::mutex> plk(pipe_mu_);
  // the persistent device input ring: reused while device, depth, feed dtypes
  // and row shapes match and it holds chunk_rows rows; rebuilt (after a
  // drain) otherwise
  size_t nin = feed_nodes_.size();
  {
    std::vector<std::vector<int64_t>> shapes;
    std::vector<at::ScalarType> dts;
    for (size_t i = 0; i < nin; ++i) {
      auto sz = seg_inputs[chunks[0].seg][i].sizes().vec();
      sz.erase(sz.begin());
      shapes.push_back(sz);
      dts.push_back(seg_inputs[chunks[0].seg][i].scalar_type());
    }
    const bool fits = pipe_ && pipe_->device == device && pipe_->depth == depth && pipe_->shapes == shapes &&
                      pipe_->dtypes == dts && pipe_->rows >= chunk_rows;
    if (!fits) {
      drop_pipe(false);
      pipe_ = std::make_unique<Pipe>();
      pipe_->device = device;
      pipe_->depth = depth;
      pipe_->rows = chunk_rows;
      pipe_->shapes = shapes;
      pipe_->dtypes = dts;
      pipe_->ring.resize(depth);
      for (int d = 0; d < depth; ++d)
        for (size_t i = 0; i < nin; ++i) {
          std::vector<int64_t> sz = shapes[i];
          sz.insert(sz.begin(), chunk_rows);
          pipe_->ring[d].push_back(dev_empty(sz, dts[i], dev, compute.stream()));
        }
      // fresh pool blocks of the compute stream: work queued there earlier may
      // still read them; the first H2D writes wait for it
      order_copy_after_compute(h2d.stream(), compute.stream());
      pipe_->ev_comp.resize(depth);
      pipe_->ev_d2h.resize(depth);
      for (int d = 0; d < depth; ++d) {
        HIP_OK(hipEventCreateWithFlags(&pipe_->ev_comp[d], hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&pipe_->ev_d2h[d], hipEventDisableTiming));
      }
      pipe_->used.assign(depth, false);
    }
  }
  Pipe& P = *pipe_;
  for (size_t s = 0; s < seg_inputs.size(); ++s)
    for (size_t i = 0; i < nin; ++i) {
      auto sz = seg_inputs[s][i].sizes().vec();
      sz.erase(sz.begin());
      TFA_CHECK(sz == P.shapes[i] && seg_inputs[s][i].scalar_type() == P.dtypes[i],
                "run_chunked: segments disagree on the row shape / dtype of feed ", i);
    }
  std::vector<hipEvent_t> ev_h2d(depth);
  for (int d = 0; d < depth; ++d) HIP_OK(hipEventCreateWithFlags(&ev_h2d[d], hipEventDisableTiming));
  int64_t h2d_bytes = 0, d2h_bytes = 0;
  // per-stage device time (hipEvent pairs bracketing each chunk's H2D, compute
  // and D2H on their streams; read once after the final synchronisation)
  const bool timed = stage_timers_enabled() && wait;
  std::vector<std::array<hipEvent_t, 6>> tev;
  auto stamp = [&](size_t ci, int k, hipStream_t s) {
    if (!timed) return;
    HIP_OK(hipEventCreate(&tev[ci][k]));
    HIP_OK(hipEventRecord(tev[ci][k], s));
  };
  if (timed) tev.assign(chunks.size(), std::array<hipEvent_t, 6>{});
  // chunks alternate between the caller's compute stream and a second,
  // persistent one (TFA_PIPE_COMPUTE_STREAMS=1: one): a GPU-bound chunk's
  // kernel tails are filled by the next chunk's kernels. The second stream
  // forks from the caller's stream here and joins it at the end.
  const int ncomp = (pipe_compute_streams() > 1 && chunks.size() > 1) ? 2 : 1;
  hipStream_t cstr[2] = {compute.stream(), ncomp > 1 ? copy_stream(device, 2) : compute.stream()};
  hipEvent_t fork_ev = nullptr;
  if (ncomp > 1) {
    HIP_OK(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
    HIP_OK(hipEventRecord(fork_ev, compute.stream()));
    HIP_OK(hipStreamWaitEvent(cstr[1], fork_ev, 0));
  }
  for (size_t ci = 0; ci < chunks.size(); ++ci) {
    const hipStream_t cs = cstr[ci % ncomp];
    const Chunk& ch = chunks[ci];
    const int slot = static_cast<int>(P.next++ % depth);
    // H2D: wait until the compute (and any D2H of outputs aliasing the ring)
    // of the chunk that last used this slot finished (maybe in an earlier call)
    if (P.used[slot]) {
      HIP_OK(hipStreamWaitEvent(h2d.stream(), P.ev_comp[slot], 0));
      HIP_OK(hipStreamWaitEvent(h2d.stream(), P.ev_d2h[slot], 0));
    }
    std::vector<at::Tensor> dev_in;
    stamp(ci, 0, h2d.stream());
    for (size_t i = 0; i < nin; ++i) {
      const at::Tensor& src = seg_inputs[ch.seg][i];
      int64_t row_bytes = src.numel() / std::max<int64_t>(src.size(0), 1) * src.element_size();
      at::Tensor dst = P.ring[slot][i].narrow(0, 0, ch.rows);
      const char* sp = static_cast<const char*>(src.data_ptr()) + ch.start * row_bytes;
      if (ch.rows * row_bytes)
        HIP_OK(hipMemcpyAsync(dst.data_ptr(), sp, ch.rows * row_bytes, hipMemcpyHostToDevice, h2d.stream()));
      h2d_bytes += ch.rows * row_bytes;
      dev_in.push_back(dst);
    }
    stamp(ci, 1, h2d.stream());
    HIP_OK(hipEventRecord(ev_h2d[slot], h2d.stream()));
    // compute
    HIP_OK(hipStreamWaitEvent(cs, ev_h2d[slot], 0));
    std::vector<at::Tensor> outs;
    stamp(ci, 2, cs);
    {
      RangeGuard rg("chunk_compute");
      auto p = plan_for(dev_in);
      outs = execute(*p, dev_in, cs);
    }
    stamp(ci, 3, cs);
    HIP_OK(hipEventRecord(P.ev_comp[slot], cs));
    // D2H
    HIP_OK(hipStreamWaitEvent(d2h.stream(), P.ev_comp[slot], 0));
    stamp(ci, 4, d2h.stream());
    for (size_t j = 0; j < outs.size(); ++j) {
      at::Tensor o = outs[j];
      const at::Tensor& dst = seg_outputs[ch.seg][j];
      int64_t row_bytes = dst.numel() / std::max<int64_t>(dst.size(0), 1) * dst.element_size();
      TFA_CHECK(o.size(0) == ch.rows && o.numel() * o.element_size() == ch.rows * row_bytes,
                "fetch '", fetch_names_[j], "' produced ", o.size(0), " rows for a chunk of ", ch.rows);
      if (!o.is_cuda()) o = o.to(dev);  // constant fetch
      char* dp = static_cast<char*>(dst.data_ptr()) + ch.start * row_bytes;
      if (ch.rows * row_bytes)
        HIP_OK(hipMemcpyAsync(dp, o.data_ptr(), ch.rows * row_bytes, hipMemcpyDeviceToHost, d2h.stream()));
      dev_record_stream(o, d2h.stream());
      d2h_bytes += ch.rows * row_bytes;
    }
    stamp(ci, 5, d2h.stream());
    HIP_OK(hipEventRecord(P.ev_d2h[slot], d2h.stream()));
    P.used[slot] = true;
    stats_.chunks++;
  }
  if (ncomp > 1) {  // join: later work on the caller's stream follows every chunk
    HIP_OK(hipEventRecord(fork_ev, cstr[1]));
    HIP_OK(hipStreamWaitEvent(compute.stream(), fork_ev, 0));
    HIP_OK(hipEventDestroy(fork_ev));
  }
  int64_t handle = 0;
  if (wait) {
    HIP_OK(hipStreamSynchronize(h2d.stream()));
    HIP_OK(hipStreamSynchronize(compute.stream()));
    HIP_OK(hipStreamSynchronize(d2h.stream()));
    // drained: the ring goes back to the pool (only a deferred sequence of
    // calls keeps it, to continue the slot rotation)
    drop_pipe(true);
  } else {
    // completion of this call = its last D2H (which waited for the last
    // compute, which waited for the last H2D)
    hipEvent_t done;
    HIP_OK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    HIP_OK(hipEventRecord(done, d2h.stream()));
    handle = reinterpret_cast<int64_t>(done);
  }
  // ev_h2d: compute already waits on them; destroying a recorded event is safe
  for (int d = 0; d < depth; ++d) hipEventDestroy(ev_h2d[d]);
  double stage_ms[3] = {0, 0, 0};
  for (auto& e : tev) {
    for (int k = 0; k < 3; ++k) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, e[2 * k], e[2 * k + 1]) == hipSuccess) stage_ms[k] += ms;
    }
    for (hipEvent_t ev : e) hipEventDestroy(ev);
  }
  auto t1 = std::chrono::steady_clock::now();
  stats_.runs++;
  stats_.h2d_bytes += h2d_bytes;
  stats_.d2h_bytes += d2h_bytes;
  stats_.wall_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
  stats_.h2d_ms += stage_ms[0];
  stats_.compute_ms += stage_ms[1];
  stats_.d2h_ms += stage_ms[2];
  return handle;
}

std::vector<at::Tensor> Program::run_chunked_reduce(const std::vector<std::vector<at::Tensor>>& seg_inputs,
                                                    int64_t chunk_rows, int device, int depth) {
  TFA_CHECK(host_op_error_.empty(), host_op_error_);
  TFA_CHECK(chunk_rows > 0, "chunk_rows must be > 0");
  depth = std::max(2, std::min(depth, 4));
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  at::Device dev(at::kCUDA, static_cast<c10::DeviceIndex>(device));
  auto compute = c10::hip::getCurrentHIPStream(device);
  auto h2d = c10::hip::getStreamFromExternal(copy_stream(device, 0), static_cast<c10::DeviceIndex>(device));
  auto t0 = std::chrono::steady_clock::now();
  struct Chunk {
    size_t seg;
    int64_t start, rows;
  };
  std::vector<Chunk> chunks;
  for (size_t s = 0; s < seg_inputs.size(); ++s) {
    TFA_CHECK(seg_inputs[s].size() == feed_nodes_.size(), "segment ", s, ": expected ", feed_nodes_.size(), " inputs");
    const int64_t rows = seg_inputs[s].empty() ? 0 : seg_inputs[s][0].size(0);
    for (auto& t : seg_inputs[s]) {
      TFA_CHECK(t.size(0) == rows, "segment inputs disagree on rows");
      TFA_CHECK(!t.is_cuda() && t.is_contiguous(), "run_chunked_reduce inputs must be contiguous host tensors");
    }
    for (int64_t st = 0; st < rows; st += chunk_rows) chunks.push_back({s, st, std::min(chunk_rows, rows - st)});
  }
  TFA_CHECK(!chunks.empty(), "run_chunked_reduce: no rows");
  const size_t nin = feed_nodes_.size();
  std::vector<std::vector<at::Tensor>> ring(depth);
  for (int d = 0; d < depth; ++d)
    for (size_t i = 0; i < nin; ++i) {
      auto sz = seg_inputs[0][i].sizes().vec();
      sz[0] = chunk_rows;
      ring[d].push_back(dev_empty(sz, seg_inputs[0][i].scalar_type(), dev, compute.stream()));
    }
  order_copy_after_compute(h2d.stream(), compute.stream());
  std::vector<hipEvent_t> ev_h2d(depth), ev_comp(depth);
  for (int d = 0; d < depth; ++d) {
    HIP_OK(hipEventCreateWithFlags(&ev_h2d[d], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_comp[d], hipEventDisableTiming));
  }
  std::vector<bool> used(depth, false);
  std::vector<at::Tensor> acc;  // [nchunks, *fetch shape] per fetch, on the device
  int64_t h2d_bytes = 0;
  for (size_t ci = 0; ci < chunks.size(); ++ci) {
    const Chunk& ch = chunks[ci];
    const int slot = static_cast<int>(ci % depth);
    if (used[slot]) HIP_OK(hipStreamWaitEvent(h2d.stream(), ev_comp[slot], 0));
    std::vector<at::Tensor> dev_in;
    for (size_t i = 0; i < nin; ++i) {
      const at::Tensor& src = seg_inputs[ch.seg][i];
      const int64_t row_bytes = src.numel() / std::max<int64_t>(src.size(0), 1) * src.element_size();
      at::Tensor dst = ring[slot][i].narrow(0, 0, ch.rows);
      const char* sp = static_cast<const char*>(src.data_ptr()) + ch.start * row_bytes;
      if (ch.rows * row_bytes)
        HIP_OK(hipMemcpyAsync(dst.data_ptr(), sp, ch.rows * row_bytes, hipMemcpyHostToDevice, h2d.stream()));
      h2d_bytes += ch.rows * row_bytes;
      dev_in.push_back(dst);
    }
    HIP_OK(hipEventRecord(ev_h2d[slot], h2d.stream()));
    HIP_OK(hipStreamWaitEvent(compute.stream(), ev_h2d[slot], 0));
    std::vector<at::Tensor> outs;
    {
      RangeGuard rg("chunk_reduce");
      auto p = plan_for(dev_in);
      outs = execute(*p, dev_in, compute.stream());
    }
    if (acc.empty()) {
      for (auto& o : outs) {
        auto sz = o.sizes().vec();
        sz.insert(sz.begin(), static_cast<int64_t>(chunks.size()));
        acc.push_back(dev_empty(sz, o.scalar_type(), dev, compute.stream()));
      }
    }
    for (size_t j = 0; j < outs.size(); ++j) {
      at::Tensor o = outs[j].is_cuda() ? outs[j].contiguous() : outs[j].to(dev);
      at::Tensor dst = acc[j].select(0, static_cast<int64_t>(ci));
      TFA_CHECK(o.numel() == dst.numel(), "fetch '", fetch_names_[j], "' changed shape between chunks");
      const int64_t nb = o.numel() * o.element_size();
      if (nb) HIP_OK(hipMemcpyAsync(dst.data_ptr(), o.data_ptr(), nb, hipMemcpyDeviceToDevice, compute.stream()));
    }
    HIP_OK(hipEventRecord(ev_comp[slot], compute.stream()));
    used[slot] = true;
    stats_.chunks++;
  }
  // the ring's last readers are on the compute stream: the caller's stream
  // orders every later use of acc; the copy stream must finish before the
  // ring is freed
  HIP_OK(hipStreamSynchronize(h2d.stream()));
  for (int d = 0; d < depth; ++d) {
    hipEventDestroy(ev_h2d[d]);
    hipEventDestroy(ev_comp[d]);
  }
  auto t1 = std::chrono::steady_clock::now();
  stats_.runs++;
  stats_.h2d_bytes += h2d_bytes;
  stats_.wall_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
  return acc;
}

std::vector<std::string> Program::fused_sources(const std::vector<at::Tensor>& inputs) {
  auto p = build_plan(inputs, true);
  std::vector<std::string> out;
  for (auto& f : p->fused_regions) out.push_back(f->region.source);
  return out;
}

ExecStats Program::stats() const { return stats_; }
void Program::reset_stats() { stats_ = ExecStats(); }

std::string Program::describe_plan(const std::vector<at::Tensor>& inputs, bool as_gpu) {
  auto p = as_gpu ? build_plan(inputs, true) : plan_for(inputs);
  std::ostringstream os;
  os << "plan: " << p->steps.size() << " steps, " << p->const_slots.size() << " constants, "
     << p->fused << " fused epilogues, " << p->fused_regions.size() << " fused regions";
  if (p->fused_siblings) os << ", " << p->fused_siblings << " sibling convs fused";
  if (p->wino_convs) os << ", " << p->wino_convs << " Winograd filters";
  {
    const std::string why = graph_blocker(*p);
    os << (why.empty() ? ", graphable" : ", not graphable (" + why + ")");
  }
  os << "\n";
  for (auto& st : p->steps) {
    const Node& nd = g_->node(st.node);
    if (st.kind == Step::FUSED) {
      const FusedRegion& rg = p->fused_regions[st.fused]->region;
      os << "  FUSED" << (rg.kind == 1 ? "-ROWRED " : " ") << nd.name << " [" << rg.expr << "] "
         << rg.leaves.size() << " inputs " << rg.outputs.size() << " outputs " << st.out_info[0].shape.str() << '\n';
      continue;
    }
    os << "  " << (st.kind == Step::GEMM ? "GEMM" : st.kind == Step::CONV ? "CONV" : "OP  ") << ' '
       << nd.op << ' ' << nd.name;
    if (st.out_node != st.node) os << " -> " << g_->node(st.out_node).name;
    if (st.bias_slot >= 0) os << " +bias";
    if (st.act) os << " +" << act_name(st.act);
    if (!st.epi.empty()) {
      static const char* codes[] = {"add", "sub", "rsub", "mul", "div", "rdiv", "max", "min", "act", "neg", "square", "abs"};
      static const char* kinds[] = {"", "scalar", "scalar", "col", "row", "full"};
      os << " +epi[";
      for (size_t k = 0; k < st.epi.size(); ++k) {
        const auto& e = st.epi[k];
        os << (k ? "," : "") << (e.code == k::EPI_ACT ? act_name(e.act) : codes[e.code]);
        if (e.kind != k::EPO_NONE) os << ":" << kinds[e.kind];
      }
      os << "]";
    }
    if (st.alias_slot >= 0) os << " ->concat-slice@" << st.alias_offset;
    if (st.wino_slot >= 0) os << " +winograd";
    if (st.pool2) os << " +maxpool2x2";
    if (st.pool_in[0]) os << " +maxpool" << st.pool_in[0] << "x" << st.pool_in[1] << "/" << st.pool_in[2] << "-in";
    if (!st.sibs.empty()) {
      os << " siblings[";
      for (size_t k = 0; k < st.sibs.size(); ++k) {
        const auto& sb = st.sibs[k];
        os << (k ? "," : "") << g_->node(sb.node).name << ":" << sb.oc;
        if (sb.act) os << "+" << act_name(sb.act);
        if (sb.alias_slot >= 0) os << "->concat-slice@" << sb.alias_offset;
      }
      os << "]";
    }
    if (!st.preplaced.empty()) {
      int n = 0;
      for (char c : st.preplaced) n += c;
      os << " (" << n << " inputs written in place)";
    }
    os << ' ' << st.out_info[0].shape.str() << '\n';
  }
  return os.str();
}

// ------------------------------------------------------------------ pinned memory
// Page-locking is expensive (hipHostMalloc of 512 MB takes ~100 ms), so
// pinned blocks are cached by 2 MiB-rounded size and handed out again when a
// tensor using them dies. Bounded by TFA_PINNED_POOL_MB (default 64 GiB).
namespace {
class PinnedPool {
 public:
  static PinnedPool& get() {
    static PinnedPool* p = new PinnedPool();
    return *p;
  }
  void* alloc(size_t bytes, size_t* rounded) {
    size_t r = (bytes + kGran - 1) / kGran * kGran;
    *rounded = r;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = free_.find(r);
      if (it != free_.end()) {
        void* p = it->second;
        free_.erase(it);
        cached_ -= r;
        return p;
      }
    }
    // page-locked memory cannot be swapped: beyond the cap, cached blocks
    // are released before new ones are locked
    if (live_.load() + cached_ + r > limit_) trim(limit_ > live_.load() + r ? limit_ - live_.load() - r : 0);
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, r, hipHostMallocDefault);
    if (e != hipSuccess) {
      trim(0);  // release cached blocks and retry once
      HIP_OK(hipHostMalloc(&p, r, hipHostMallocDefault));
    }
    return p;
  }
  void note_live(size_t r, bool add) {
    const size_t now = add ? (live_ += r) : (live_ -= r);
    size_t pk = peak_.load();
    while (now > pk && !peak_.compare_exchange_weak(pk, now)) {
    }
  }
  void release(void* p, size_t r) {
    std::lock_guard<std::mutex> lk(mu_);
    free_.emplace(r, p);
    cached_ += r;
    while (cached_ > limit_ && !free_.empty()) {
      auto it = std::prev(free_.end());
      cached_ -= it->first;
      hipHostFree(it->second);
      free_.erase(it);
    }
  }
  void trim(size_t keep) {
    std::lock_guard<std::mutex> lk(mu_);
    while (cached_ > keep && !free_.empty()) {
      auto it = free_.begin();
      cached_ -= it->first;
      hipHostFree(it->second);
      free_.erase(it);
    }
  }
  size_t cached() const { return cached_; }
  size_t live() const { return live_.load(); }
  size_t peak() const { return peak_.load(); }
  size_t limit() const { return limit_; }

 private:
  PinnedPool() { limit_ = default_limit(); }
  // TFA_PINNED_POOL_MB, else half of this process's share of host RAM (one
  // rank per GPU: RAM / LOCAL_WORLD_SIZE), at most 64 GiB: eight ranks of a
  // node must not lock more memory than the machine has
  static size_t default_limit() {
    if (const char* e = std::getenv("TFA_PINNED_POOL_MB"))
      if (std::atoll(e) > 0) return static_cast<size_t>(std::atoll(e)) << 20;
    const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGE_SIZE);
    size_t ram = pages > 0 && psz > 0 ? static_cast<size_t>(pages) * static_cast<size_t>(psz) : (size_t(64) << 30);
    int local = 1;
    if (const char* lw = std::getenv("LOCAL_WORLD_SIZE")) local = std::max(1, std::atoi(lw));
    return std::min(size_t(64) << 30, ram / static_cast<size_t>(local) / 2);
  }
  static constexpr size_t kGran = size_t(2) << 20;
  std::mutex mu_;
  std::multimap<size_t, void*> free_;
  size_t cached_ = 0;
  std::atomic<size_t> live_{0}, peak_{0};
  size_t limit_;
};
}  // namespace

at::Tensor empty_pinned(const std::vector<int64_t>& sizes, at::ScalarType dt) {
  int64_t n = 1;
  for (auto s : sizes) n *= s;
  size_t bytes = static_cast<size_t>(std::max<int64_t>(n, 1)) * c10::elementSize(dt);
  size_t r = 0;
  void* p = PinnedPool::get().alloc(bytes, &r);
  PinnedPool::get().note_live(r, true);
  return at::from_blob(p, sizes,
                       [r](void* q) {
                         PinnedPool::get().note_live(r, false);
                         PinnedPool::get().release(q, r);
                       },
                       at::TensorOptions().dtype(dt));
}

void trim_pinned_pool() { PinnedPool::get().trim(0); }
size_t pinned_pool_cached_bytes() { return PinnedPool::get().cached(); }
std::vector<size_t> pinned_pool_stats() {
  auto& p = PinnedPool::get();
  return {p.limit(), p.cached(), p.live(), p.peak()};
}

void pin_host_tensor(const at::Tensor& t) {
  TFA_CHECK(!t.is_cuda(), "pin_host_tensor needs a host tensor");
  size_t bytes = t.numel() * t.element_size();
  if (!bytes) return;
  HIP_OK(hipHostRegister(t.data_ptr(), bytes, hipHostRegisterDefault));
}

void unpin_host_tensor(const at::Tensor& t) {
  if (t.numel()) hipHostUnregister(t.data_ptr());
}

}  // namespace tfa

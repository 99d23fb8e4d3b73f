// Engine-owned communicators: FakeComm (threads), RcclComm (RCCL), OneShotComm
// (IPC single-hop all-reduce), ShmComm (host tensors over shared memory). See comm.h.
#include "comm.h"

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "../ir/graph.h"
#include "../runtime/device_pool.h"

namespace tfa {
namespace comm {

k::RedOp parse_op(const std::string& op) {
  if (op == "Sum") return k::RedOp::SUM;
  if (op == "Min") return k::RedOp::MIN;
  if (op == "Max") return k::RedOp::MAX;
  if (op == "Prod") return k::RedOp::PROD;
  TFA_CHECK(false, "collective op must be Sum, Min, Max or Prod, got '", op, "'");
  return k::RedOp::SUM;
}

namespace {

at::Tensor fold(const at::Tensor& a, const at::Tensor& b, k::RedOp op) {
  switch (op) {
    case k::RedOp::SUM: return a + b;
    case k::RedOp::PROD: return a * b;
    case k::RedOp::MIN: return at::minimum(a, b);
    default: return at::maximum(a, b);
  }
}

void check_rows(const at::Tensor& x, const std::vector<int64_t>& send_rows, int world) {
  TFA_CHECK(static_cast<int>(send_rows.size()) == world, "all_to_all_v: ", send_rows.size(),
            " send counts for a world of ", world);
  int64_t tot = 0;
  for (int64_t r : send_rows) {
    TFA_CHECK(r >= 0, "all_to_all_v: negative row count");
    tot += r;
  }
  TFA_CHECK(x.dim() >= 1 && x.size(0) == tot, "all_to_all_v: input has ", x.dim() ? x.size(0) : 0,
            " rows, send counts sum to ", tot);
}

}  // namespace

// ---------------------------------------------------------------- FakeWorld
FakeWorld::FakeWorld(int n) : n_(n), slots_(n), meta_(n) { TFA_CHECK(n >= 1, "FakeWorld: n must be >= 1"); }

void FakeWorld::barrier() {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t g = gen_;
  if (++arrived_ == n_) {
    arrived_ = 0;
    ++gen_;
    cv_.notify_all();
    return;
  }
  // a rank that never arrives is a test bug: fail instead of hanging
  if (!cv_.wait_for(lk, std::chrono::seconds(120), [&] { return gen_ != g; }))
    TFA_CHECK(false, "FakeComm: barrier timed out (a rank did not join the collective)");
}

const std::vector<at::Tensor>& FakeWorld::exchange(int rank, const at::Tensor& t, const std::vector<int64_t>& meta,
                                                   std::vector<std::vector<int64_t>>* metas) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    slots_[rank] = t;
    meta_[rank] = meta;
  }
  barrier();
  if (metas) *metas = meta_;
  return slots_;
}

FakeComm::FakeComm(std::shared_ptr<FakeWorld> w, int rank) : w_(std::move(w)), rank_(rank) {
  TFA_CHECK(rank >= 0 && rank < w_->size(), "FakeComm: rank ", rank, " outside a world of ", w_->size());
}

void FakeComm::all_reduce(at::Tensor& t, k::RedOp op) {
  ++calls_;
  const auto& v = w_->exchange(rank_, t.contiguous().clone(), {}, nullptr);
  at::Tensor acc = v[0].clone();
  for (int r = 1; r < w_->size(); ++r) {
    TFA_CHECK(v[r].sizes() == acc.sizes() && v[r].scalar_type() == acc.scalar_type(),
              "all_reduce: ranks disagree on the tensor");
    acc = fold(acc, v[r], op);
  }
  w_->release();
  t.copy_(acc);
}

at::Tensor FakeComm::all_gather(const at::Tensor& t) {
  ++calls_;
  const auto& v = w_->exchange(rank_, t.contiguous(), {}, nullptr);
  at::Tensor out = at::stack(v, 0);
  w_->release();
  return out;
}

at::Tensor FakeComm::all_to_all_v(const at::Tensor& x, const std::vector<int64_t>& send_rows,
                                  const std::vector<int64_t>& recv_rows) {
  ++calls_;
  const int W = w_->size();
  check_rows(x, send_rows, W);
  std::vector<std::vector<int64_t>> metas;
  const auto& v = w_->exchange(rank_, x.contiguous(), send_rows, &metas);
  std::vector<at::Tensor> parts;
  std::string err;
  for (int s = 0; s < W && err.empty(); ++s) {
    int64_t off = 0;
    for (int r = 0; r < rank_; ++r) off += metas[s][r];
    const int64_t n = metas[s][rank_];
    if (static_cast<int>(recv_rows.size()) != W || n != recv_rows[s])
      err = str_cat("all_to_all_v: rank ", s, " sends ", n, " rows, ",
                    static_cast<int>(recv_rows.size()) == W ? recv_rows[s] : -1, " expected");
    else
      parts.push_back(v[s].narrow(0, off, n).clone());
  }
  w_->release();  // every rank leaves the collective, also the one that raises
  TFA_CHECK(err.empty(), err);
  return at::cat(parts, 0);
}

void FakeComm::broadcast(at::Tensor& t, int root) {
  ++calls_;
  const auto& v = w_->exchange(rank_, t.contiguous(), {}, nullptr);
  at::Tensor src = v.at(root).clone();
  w_->release();
  if (rank_ != root) t.copy_(src);
}

// ---------------------------------------------------------------- RCCL
namespace {

#define TFA_NCCL(call)                                                                      \
  do {                                                                                      \
    ncclResult_t r_ = (call);                                                               \
    TFA_CHECK(r_ == ncclSuccess, "RCCL ", #call, " failed: ", ncclGetErrorString(r_));      \
  } while (0)

ncclDataType_t nccl_dtype(at::ScalarType st) {
  switch (st) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    default: TFA_CHECK(false, "RCCL: unsupported dtype ", c10::toString(st));
  }
  return ncclFloat32;
}

ncclRedOp_t nccl_op(k::RedOp op) {
  switch (op) {
    case k::RedOp::SUM: return ncclSum;
    case k::RedOp::PROD: return ncclProd;
    case k::RedOp::MIN: return ncclMin;
    default: return ncclMax;
  }
}

hipStream_t cur_stream(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

}  // namespace

std::string rccl_unique_id() {
  ncclUniqueId id;
  TFA_NCCL(ncclGetUniqueId(&id));
  return std::string(id.internal, sizeof(id.internal));
}

RcclComm::RcclComm(const std::string& unique_id, int rank, int size, int device)
    : rank_(rank), size_(size), device_(device) {
  TFA_CHECK(unique_id.size() == sizeof(ncclUniqueId), "RcclComm: unique id must be ", sizeof(ncclUniqueId), " bytes");
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), sizeof(id.internal));
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  ncclComm_t c = nullptr;
  TFA_NCCL(ncclCommInitRank(&c, size, id, rank));
  comm_ = c;
  wd_ = std::thread([this] { watchdog(); });
}

RcclComm::~RcclComm() {
  stop_ = true;
  wcv_.notify_all();
  if (wd_.joinable()) wd_.join();
  if (comm_) {
    // a failed communicator may have a collective that never completes:
    // destroy would wait for it, abort does not
    if (failed_) (void)ncclCommAbort(static_cast<ncclComm_t>(comm_));
    else (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
  }
  for (auto& f : inflight_) {
    (void)hipEventDestroy(f.ev);
    if (f.start) (void)hipEventDestroy(f.start);
  }
  for (hipEvent_t e : free_events_) (void)hipEventDestroy(e);
  (void)hipGetLastError();
}

void RcclComm::set_timeout(double seconds, bool exit_on_timeout) {
  std::lock_guard<std::mutex> lk(wmu_);
  timeout_s_ = seconds;
  exit_on_timeout_ = exit_on_timeout;
}

hipEvent_t RcclComm::take_event() {
  hipEvent_t e = nullptr;
  {
    std::lock_guard<std::mutex> lk(wmu_);
    if (!free_events_.empty()) {
      e = free_events_.back();
      free_events_.pop_back();
    }
  }
  if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return e;
}

hipEvent_t RcclComm::begin(hipStream_t s) {
  hipEvent_t e = take_event();
  if (e) (void)hipEventRecord(e, s);
  return e;
}

void RcclComm::track(hipStream_t s, hipEvent_t start) {
  hipEvent_t e = take_event();
  if (!e) {  // no event: this collective is not watched (never fails the call)
    if (start) {
      std::lock_guard<std::mutex> lk(wmu_);
      free_events_.push_back(start);
    }
    return;
  }
  (void)hipEventRecord(e, s);
  {
    std::lock_guard<std::mutex> lk(wmu_);
    inflight_.push_back({e, start, std::chrono::steady_clock::now(), start == nullptr});
  }
  wcv_.notify_one();
}

double RcclComm::front_age() {
  if (inflight_.empty()) return 0;
  Inflight& f = inflight_.front();
  const auto now = std::chrono::steady_clock::now();
  if (!f.started) {
    if (hipEventQuery(f.start) == hipErrorNotReady) return 0;
    f.started = true;
    f.t0 = now;
  }
  return std::chrono::duration<double>(now - f.t0).count();
}

void RcclComm::abort_comm(std::unique_lock<std::mutex>& held) {
  ncclComm_t c = static_cast<ncclComm_t>(comm_);
  comm_ = nullptr;
  if (!c) return;
  held.unlock();
  auto done = std::make_shared<std::atomic<bool>>(false);
  std::thread([c, done] {
    (void)ncclCommAbort(c);
    done->store(true);
  }).detach();
  for (int i = 0; i < 100 && !done->load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(20));
  held.lock();
}

int64_t RcclComm::inflight() const {
  std::lock_guard<std::mutex> lk(wmu_);
  return static_cast<int64_t>(inflight_.size());
}

void RcclComm::fail(const std::string& why) {
  std::lock_guard<std::mutex> lk(wmu_);
  if (!failed_) {
    fail_msg_ = why;
    failed_ = true;
  }
}

void RcclComm::check() {
  if (!failed_) return;
  std::lock_guard<std::mutex> lk(wmu_);
  throw CollectiveError(str_cat("RCCL communicator (rank ", rank_, " of ", size_, ") failed: ", fail_msg_));
}

void RcclComm::wait() {
  check();
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  for (int spins = 0;; ++spins) {
    Inflight front{};
    double tmo;
    {
      std::lock_guard<std::mutex> lk(wmu_);
      while (!inflight_.empty()) {
        const hipError_t q = hipEventQuery(inflight_.front().ev);
        if (q == hipErrorNotReady) break;
        free_events_.push_back(inflight_.front().ev);
        if (inflight_.front().start) free_events_.push_back(inflight_.front().start);
        inflight_.pop_front();
      }
      if (inflight_.empty()) {
        (void)hipGetLastError();
        return;
      }
      front = inflight_.front();
      tmo = timeout_s_;
    }
    double age;
    {
      std::lock_guard<std::mutex> lk(wmu_);
      age = front_age();
    }
    if (tmo > 0 && age > tmo) {
      const std::string why = str_cat("a collective did not complete within ", tmo,
                                      " s of starting (collective_timeout_s): a peer rank is missing, stuck, or "
                                      "issued a different collective sequence");
      {
        std::unique_lock<std::mutex> lk(wmu_);
        if (!failed_) {
          fail_msg_ = why;
          failed_ = true;
        }
        // release the stuck collective kernel: without the abort the next
        // synchronisation of this stream (a retry, the combine's sync) would
        // block forever
        abort_comm(lk);
      }
      throw CollectiveError(str_cat("RCCL collective timed out on rank ", rank_, " of ", size_, ": ", why));
    }
    if (spins < 64) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void RcclComm::watchdog() {
  (void)hipSetDevice(device_);
  std::unique_lock<std::mutex> lk(wmu_);
  while (!stop_) {
    wcv_.wait_for(lk, std::chrono::milliseconds(20));
    if (stop_) break;
    while (!inflight_.empty()) {
      const hipError_t q = hipEventQuery(inflight_.front().ev);
      if (q == hipErrorNotReady) break;
      free_events_.push_back(inflight_.front().ev);
      if (inflight_.front().start) free_events_.push_back(inflight_.front().start);
      inflight_.pop_front();
    }
    (void)hipGetLastError();
    if (failed_ || !comm_) continue;  // already reported to the main thread (and aborted)
    std::string why;
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &ae) == ncclSuccess && ae != ncclSuccess &&
        ae != ncclInProgress)
      why = str_cat("asynchronous RCCL error: ", ncclGetErrorString(ae));
    if (why.empty() && timeout_s_ > 0 && !inflight_.empty()) {
      // the main thread's own wait() raises at the timeout; past it plus a
      // grace period nobody is polling: the main thread is stuck elsewhere
      const double grace = std::min(60.0, std::max(1.0, 0.5 * timeout_s_));
      const double age = front_age();
      if (age > timeout_s_ + grace)
        why = str_cat("a collective has not completed after ", age, " s (collective_timeout_s = ", timeout_s_, ")");
    }
    if (why.empty()) continue;
    if (!exit_on_timeout_) {
      fail_msg_ = why;
      failed_ = true;
      abort_comm(lk);  // a thread blocked in a sync on this stream is released
      continue;
    }
    std::fprintf(stderr,
                 "tensorframes_amd: rank %d of %d: %s; aborting the RCCL communicator and exiting with status %d "
                 "so the launcher can tear the job down\n",
                 rank_, size_, why.c_str(), kExitCollectiveTimeout);
    std::fflush(stderr);
    // ncclCommAbort unblocks a collective kernel waiting for a peer; it is
    // given 2 s in a helper thread, then the process ends regardless (process
    // teardown drops the queued work)
    ncclComm_t c = static_cast<ncclComm_t>(comm_);
    std::thread([c] { (void)ncclCommAbort(c); }).detach();
    for (int i = 0; i < 100; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    std::_Exit(kExitCollectiveTimeout);
  }
}

void RcclComm::all_reduce(at::Tensor& t, k::RedOp op) {
  TFA_CHECK(t.is_cuda() && t.is_contiguous(), "RcclComm.all_reduce: contiguous device tensor expected");
  check();
  ++calls_;
  c10::hip::HIPGuard guard(t.device().index());
  hipEvent_t st = begin(cur_stream(t));
  if (test_stall_s_ > 0) k::device_stall(static_cast<uint64_t>(test_stall_s_ * 1e6), cur_stream(t));
  TFA_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), nccl_op(op),
                         static_cast<ncclComm_t>(comm_), cur_stream(t)));
  track(cur_stream(t), st);
}

at::Tensor RcclComm::all_gather(const at::Tensor& t0) {
  at::Tensor t = t0.contiguous();
  TFA_CHECK(t.is_cuda(), "RcclComm.all_gather: device tensor expected");
  check();
  ++calls_;
  c10::hip::HIPGuard guard(t.device().index());
  std::vector<int64_t> sz = t.sizes().vec();
  sz.insert(sz.begin(), size_);
  at::Tensor out = pool_empty(sz, t.options());
  hipEvent_t st = begin(cur_stream(t));
  TFA_NCCL(ncclAllGather(t.data_ptr(), out.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()),
                         static_cast<ncclComm_t>(comm_), cur_stream(t)));
  track(cur_stream(t), st);
  return out;
}

at::Tensor RcclComm::all_to_all_v(const at::Tensor& x0, const std::vector<int64_t>& send_rows,
                                  const std::vector<int64_t>& recv_rows) {
  at::Tensor x = x0.contiguous();
  TFA_CHECK(x.is_cuda(), "RcclComm.all_to_all_v: device tensor expected");
  check_rows(x, send_rows, size_);
  TFA_CHECK(static_cast<int>(recv_rows.size()) == size_, "all_to_all_v: bad receive counts");
  check();
  ++calls_;
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t row_bytes = x.dim() ? (x.numel() / std::max<int64_t>(x.size(0), 1)) * x.element_size() : 0;
  int64_t total = 0;
  for (int64_t r : recv_rows) total += r;
  std::vector<int64_t> sz = x.sizes().vec();
  sz[0] = total;
  at::Tensor out = pool_empty(sz, x.options());
  const hipStream_t s = cur_stream(x);
  // one grouped launch: every peer pair moves its rows over its own xGMI link
  // (the groupBy shuffle, reference DebugRowOps.scala:576)
  hipEvent_t st = begin(s);
  TFA_NCCL(ncclGroupStart());
  int64_t so = 0, ro = 0;
  for (int r = 0; r < size_; ++r) {
    if (send_rows[r])
      TFA_NCCL(ncclSend(static_cast<char*>(x.data_ptr()) + so * row_bytes, send_rows[r] * row_bytes, ncclUint8, r,
                        static_cast<ncclComm_t>(comm_), s));
    if (recv_rows[r])
      TFA_NCCL(ncclRecv(static_cast<char*>(out.data_ptr()) + ro * row_bytes, recv_rows[r] * row_bytes, ncclUint8, r,
                        static_cast<ncclComm_t>(comm_), s));
    so += send_rows[r];
    ro += recv_rows[r];
  }
  TFA_NCCL(ncclGroupEnd());
  track(s, st);
  return out;
}

void RcclComm::broadcast(at::Tensor& t, int root) {
  TFA_CHECK(t.is_cuda() && t.is_contiguous(), "RcclComm.broadcast: contiguous device tensor expected");
  check();
  ++calls_;
  c10::hip::HIPGuard guard(t.device().index());
  hipEvent_t st = begin(cur_stream(t));
  TFA_NCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), root,
                         static_cast<ncclComm_t>(comm_), cur_stream(t)));
  track(cur_stream(t), st);
}

void RcclComm::barrier() {
  // a one-element all-reduce on the current stream, then a bounded wait for it
  at::Tensor one = pool_empty({1}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, device_));
  TFA_CHECK(hipMemsetAsync(one.data_ptr(), 0, sizeof(int), cur_stream(one)) == hipSuccess,
            "RcclComm.barrier: memset failed");
  all_reduce(one, k::RedOp::SUM);
  wait();
}

void RcclComm::abort() {
  stop_ = true;
  wcv_.notify_all();
  if (wd_.joinable() && wd_.get_id() != std::this_thread::get_id()) wd_.join();
  if (comm_) {
    (void)ncclCommAbort(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
  }
  fail("aborted");
}

std::string RcclComm::async_error() {
  if (!comm_) return "aborted";
  ncclResult_t e = ncclSuccess;
  if (ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &e) != ncclSuccess) return "query failed";
  return e == ncclSuccess ? "" : ncclGetErrorString(e);
}

// ---------------------------------------------------------------- one-shot
OneShotComm::OneShotComm(int rank, int size, int device) : rank_(rank), size_(size), device_(device) {
  TFA_CHECK(size >= 1 && size <= k::kOneShotMaxRanks && rank >= 0 && rank < size, "OneShotComm: world ", size,
            " rank ", rank, " (at most ", k::kOneShotMaxRanks, " ranks)");
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  // uncached first: a peer GPU writes our flags and reads our slot over
  // xGMI, and neither side's L2 may keep a stale copy of those lines (the
  // kernel's system-scope accesses bypass L1 only); an allocation kind whose
  // memory cannot be exported over IPC is skipped
  auto try_alloc = [&](unsigned flags, const char* kind) {
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, k::kOneShotBufBytes, flags) != hipSuccess || !p) {
      (void)hipGetLastError();
      return false;
    }
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipFree(p);
      return false;
    }
    own_ = p;
    alloc_kind_ = kind;
    return true;
  };
  if (!try_alloc(hipDeviceMallocUncached, "uncached") && !try_alloc(hipDeviceMallocFinegrained, "fine-grained")) {
    TFA_CHECK(hipMalloc(&own_, k::kOneShotBufBytes) == hipSuccess, "OneShotComm: hipMalloc failed");
    alloc_kind_ = "coarse";
  }
  // flags and error word start at zero (epochs start at 1); done before the
  // handle is handed to any peer
  TFA_CHECK(hipMemset(own_, 0, k::kOneShotBufBytes) == hipSuccess, "OneShotComm: hipMemset failed");
  TFA_CHECK(hipDeviceSynchronize() == hipSuccess, "OneShotComm: sync failed");
  peers_.buf[rank] = own_;
}

OneShotComm::~OneShotComm() {
  for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
  if (own_) (void)hipFree(own_);
  (void)hipGetLastError();
}

std::string OneShotComm::ipc_handle() const {
  hipIpcMemHandle_t h;
  TFA_CHECK(hipIpcGetMemHandle(&h, own_) == hipSuccess, "OneShotComm: hipIpcGetMemHandle failed");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void OneShotComm::open(const std::vector<std::string>& handles) {
  TFA_CHECK(static_cast<int>(handles.size()) == size_, "OneShotComm.open: ", handles.size(), " handles for ", size_,
            " ranks");
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  for (int r = 0; r < size_; ++r) {
    if (r == rank_) continue;
    TFA_CHECK(handles[r].size() == sizeof(hipIpcMemHandle_t), "OneShotComm.open: bad handle from rank ", r);
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    TFA_CHECK(e == hipSuccess && p, "OneShotComm: hipIpcOpenMemHandle for rank ", r, " failed: ", hipGetErrorString(e));
    opened_.push_back(p);
    peers_.buf[r] = p;
  }
  ready_ = true;
}

void OneShotComm::all_reduce(at::Tensor& t, k::RedOp op) {
  TFA_CHECK(ready_, "OneShotComm: open() the peers first");
  TFA_CHECK(t.is_cuda() && t.is_contiguous() && t.device().index() == device_,
            "OneShotComm.all_reduce: contiguous tensor on device ", device_, " expected");
  TFA_CHECK(t.numel() * t.element_size() <= max_bytes(), "OneShotComm.all_reduce: payload over ", max_bytes(),
            " bytes");
  if (failed_)
    throw CollectiveError("one-shot all-reduce: the communicator failed earlier (a peer missed a collective)");
  ++calls_;
  ++epoch_;
  c10::hip::HIPGuard guard(t.device().index());
  k::oneshot_all_reduce(op, from_scalar_type(t.scalar_type()), t.data_ptr(), t.data_ptr(), t.numel(), rank_, size_,
                        peers_, epoch_, timeout_us_, cur_stream(t));
}

void OneShotComm::check() {
  int err = 0;
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  TFA_CHECK(hipMemcpy(&err, static_cast<char*>(own_) + k::kOneShotErrOffset, sizeof(err), hipMemcpyDeviceToHost) ==
                hipSuccess,
            "OneShotComm.check: hipMemcpy failed");
  if (err == 0) {
    if (failed_) throw CollectiveError("one-shot all-reduce: the communicator failed earlier");
    return;
  }
  // report once: clear the word (its timeout is not re-raised by later
  // checks); the comm stays failed, since the ranks' epochs no longer agree
  TFA_CHECK(hipMemset(static_cast<char*>(own_) + k::kOneShotErrOffset, 0, sizeof(int)) == hipSuccess,
            "OneShotComm.check: hipMemset failed");
  failed_ = true;
  throw CollectiveError(str_cat("one-shot all-reduce on rank ", rank_, " of ", size_, " timed out after ",
                                timeout_us_ / 1e6, " s waiting for a peer's flag (a rank did not join)"));
}

// ---------------------------------------------------------------- ShmComm
// Host tensors of the ranks of one node through a POSIX shared-memory
// segment: the reference's driver-side combine (RDD.reduce,
// DebugRowOps.scala:500, :524-525) and its shuffle (:576) for CPU ranks, and
// the host-side control collectives (row counts, has-data flags) of GPU
// ranks, at memcpy speed instead of through gloo's TCP loopback.
struct ShmComm::Ctrl {
  alignas(64) std::atomic<uint32_t> arrived;
  alignas(64) std::atomic<uint32_t> gen;
  alignas(64) std::atomic<uint32_t> attached;
  alignas(64) std::atomic<uint32_t> broken;  // a rank failed mid-collective: every later wait fails fast
};
static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics must be lock-free");

namespace {
constexpr size_t kShmMetaOffset = 256;  // after the barrier words: kMaxRanks x kMaxRanks int64
constexpr size_t kShmCtrlBytes = kShmMetaOffset + ShmComm::kMaxRanks * ShmComm::kMaxRanks * sizeof(int64_t);
static_assert(sizeof(ShmComm::kMaxRanks) && kShmCtrlBytes % 256 == 0, "control block alignment");
}  // namespace

int64_t* ShmComm::meta(int r) const {
  return reinterpret_cast<int64_t*>(base_ + kShmMetaOffset) + static_cast<int64_t>(r) * kMaxRanks;
}

char* ShmComm::result() const { return base_ + kShmCtrlBytes; }
char* ShmComm::slot(int r) const { return base_ + kShmCtrlBytes + slot_ * (1 + r); }

ShmComm::ShmComm(const std::string& name, int rank, int size, int64_t slot_bytes, bool create)
    : name_(name), rank_(rank), size_(size) {
  TFA_CHECK(size >= 1 && size <= kMaxRanks && rank >= 0 && rank < size, "ShmComm: world ", size, " rank ", rank,
            " (at most ", kMaxRanks, " ranks)");
  TFA_CHECK(!name.empty() && name[0] == '/', "ShmComm: segment name must start with '/'");
  slot_ = std::max<int64_t>(slot_bytes, 64 << 10) / 256 * 256;
  bytes_ = kShmCtrlBytes + static_cast<size_t>(slot_) * (size + 1);
  int fd = -1;
  if (create) {
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    TFA_CHECK(fd >= 0, "ShmComm: shm_open(", name, ") failed: ", std::strerror(errno));
    if (ftruncate(fd, static_cast<off_t>(bytes_)) != 0) {
      const int e = errno;
      close(fd);
      shm_unlink(name.c_str());
      TFA_CHECK(false, "ShmComm: ftruncate failed: ", std::strerror(e));
    }
    // reserve the tmpfs pages now: a /dev/shm too small for the segment then
    // fails here (the ranks agree and fall back to gloo) instead of raising
    // SIGBUS on the first touch of an unbacked page mid-collective
    if (const int e = posix_fallocate(fd, 0, static_cast<off_t>(bytes_)); e != 0) {
      close(fd);
      shm_unlink(name.c_str());
      TFA_CHECK(false, "ShmComm: cannot reserve ", bytes_, " bytes in /dev/shm: ", std::strerror(e));
    }
  } else {
    fd = shm_open(name.c_str(), O_RDWR, 0600);
    TFA_CHECK(fd >= 0, "ShmComm: shm_open(", name, ") failed: ", std::strerror(errno));
    struct stat st;
    const bool ok = fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) == bytes_;
    if (!ok) close(fd);
    TFA_CHECK(ok, "ShmComm: segment ", name, " has the wrong size (ranks disagree on world size or slot bytes)");
  }
  void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (create) shm_unlink(name.c_str());
    TFA_CHECK(false, "ShmComm: mmap failed: ", std::strerror(errno));
  }
  base_ = static_cast<char*>(p);
  linked_ = create;
  Ctrl* c = reinterpret_cast<Ctrl*>(base_);
  if (create) {
    // ftruncate zero-filled the segment: every counter starts at 0
    c->attached.store(1, std::memory_order_release);
  } else {
    c->attached.fetch_add(1, std::memory_order_acq_rel);
  }
}

ShmComm::~ShmComm() {
  if (base_) munmap(base_, bytes_);
  if (linked_) shm_unlink(name_.c_str());
}

void ShmComm::unlink() {
  if (linked_) shm_unlink(name_.c_str());
  linked_ = false;
}

int ShmComm::attached() const {
  return static_cast<int>(reinterpret_cast<Ctrl*>(base_)->attached.load(std::memory_order_acquire));
}

void ShmComm::fail_all(const std::string& why) {
  reinterpret_cast<Ctrl*>(base_)->broken.store(1, std::memory_order_release);
  throw CollectiveError(why);
}

void ShmComm::poison() { reinterpret_cast<Ctrl*>(base_)->broken.store(1, std::memory_order_release); }

bool ShmComm::poisoned() const { return reinterpret_cast<Ctrl*>(base_)->broken.load(std::memory_order_acquire) != 0; }

void ShmComm::reset_after_failure() {
  Ctrl* c = reinterpret_cast<Ctrl*>(base_);
  c->arrived.store(0, std::memory_order_relaxed);
  c->broken.store(0, std::memory_order_release);
}

void ShmComm::barrier() {
  Ctrl* c = reinterpret_cast<Ctrl*>(base_);
  if (c->broken.load(std::memory_order_acquire))
    throw CollectiveError("shm communicator: a rank failed in an earlier collective");
  const uint32_t g = c->gen.load(std::memory_order_acquire);
  if (c->arrived.fetch_add(1, std::memory_order_acq_rel) == static_cast<uint32_t>(size_ - 1)) {
    c->arrived.store(0, std::memory_order_relaxed);
    c->gen.store(g + 1, std::memory_order_release);
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t i = 0;; ++i) {
    if (c->gen.load(std::memory_order_acquire) != g) return;
    if (i < 4096) {
      __builtin_ia32_pause();
      continue;
    }
    if (c->broken.load(std::memory_order_acquire))
      throw CollectiveError("shm collective: another rank failed");
    if ((i & 63) == 0 && timeout_s_ > 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_)
      fail_all(str_cat("shm collective timed out on rank ", rank_, " of ", size_, " after ", timeout_s_,
                       " s (a rank did not join the collective)"));
    if (i < 16384) sched_yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

namespace {

// y = y op x over n elements of dtype st
void fold_into(char* y, const char* x, int64_t n, at::ScalarType st, k::RedOp op) {
  auto run = [&](auto tag) {
    using T = decltype(tag);
    T* a = reinterpret_cast<T*>(y);
    const T* b = reinterpret_cast<const T*>(x);
    switch (op) {
      case k::RedOp::SUM: for (int64_t i = 0; i < n; ++i) a[i] = static_cast<T>(a[i] + b[i]); break;
      case k::RedOp::PROD: for (int64_t i = 0; i < n; ++i) a[i] = static_cast<T>(a[i] * b[i]); break;
      case k::RedOp::MIN: for (int64_t i = 0; i < n; ++i) a[i] = b[i] < a[i] ? b[i] : a[i]; break;
      default: for (int64_t i = 0; i < n; ++i) a[i] = b[i] > a[i] ? b[i] : a[i]; break;
    }
  };
  switch (st) {
    case at::kFloat: run(float{}); break;
    case at::kDouble: run(double{}); break;
    case at::kInt: run(int32_t{}); break;
    case at::kLong: run(int64_t{}); break;
    case at::kShort: run(int16_t{}); break;
    case at::kByte: run(uint8_t{}); break;
    case at::kChar: run(int8_t{}); break;
    default: TFA_CHECK(false, "shm all_reduce: unsupported dtype ", c10::toString(st));
  }
}

}  // namespace

void ShmComm::all_reduce(at::Tensor& t, k::RedOp op) {
  TFA_CHECK(!t.is_cuda() && t.is_contiguous(), "ShmComm.all_reduce: contiguous host tensor expected");
  ++calls_;
  const int64_t es = t.element_size();
  const int64_t nbytes = t.numel() * es;
  char* data = static_cast<char*>(t.data_ptr());
  const int64_t chunk = slot_ / es * es;
  int64_t off = 0;
  do {
    const int64_t nb = std::min(chunk, nbytes - off);
    if (nb > 0) std::memcpy(slot(rank_), data + off, nb);
    barrier();
    if (nb > 0) {
      const int64_t n = nb / es;
      if (nb <= (64 << 10) || size_ == 1) {
        // small: every rank folds all ranks' values in rank order, so every
        // rank holds bitwise the same result
        std::memcpy(data + off, slot(0), nb);
        for (int r = 1; r < size_; ++r) fold_into(data + off, slot(r), n, t.scalar_type(), op);
      } else {
        // large: rank r folds its 1/W share of the chunk (still in rank
        // order) into the result slot, then every rank copies the result
        const int64_t per = (n + size_ - 1) / size_;
        const int64_t lo = std::min(n, per * rank_), hi = std::min(n, lo + per);
        if (hi > lo) {
          char* dst = result() + lo * es;
          std::memcpy(dst, slot(0) + lo * es, (hi - lo) * es);
          for (int r = 1; r < size_; ++r) fold_into(dst, slot(r) + lo * es, hi - lo, t.scalar_type(), op);
        }
        barrier();
        std::memcpy(data + off, result(), nb);
      }
    }
    barrier();
    off += chunk;
  } while (off < nbytes);
}

at::Tensor ShmComm::all_gather(const at::Tensor& t0) {
  at::Tensor t = t0.contiguous();
  TFA_CHECK(!t.is_cuda(), "ShmComm.all_gather: host tensor expected");
  ++calls_;
  std::vector<int64_t> sz = t.sizes().vec();
  sz.insert(sz.begin(), size_);
  at::Tensor out = at::empty(sz, t.options());
  const int64_t nbytes = t.numel() * t.element_size();
  const char* src = static_cast<const char*>(t.data_ptr());
  char* dst = static_cast<char*>(out.data_ptr());
  int64_t off = 0;
  do {
    const int64_t nb = std::min<int64_t>(slot_, nbytes - off);
    if (nb > 0) std::memcpy(slot(rank_), src + off, nb);
    barrier();
    if (nb > 0)
      for (int r = 0; r < size_; ++r) std::memcpy(dst + r * nbytes + off, slot(r), nb);
    barrier();
    off += slot_;
  } while (off < nbytes);
  return out;
}

void ShmComm::broadcast(at::Tensor& t, int root) {
  TFA_CHECK(!t.is_cuda() && t.is_contiguous(), "ShmComm.broadcast: contiguous host tensor expected");
  TFA_CHECK(root >= 0 && root < size_, "ShmComm.broadcast: bad root ", root);
  ++calls_;
  const int64_t nbytes = t.numel() * t.element_size();
  char* data = static_cast<char*>(t.data_ptr());
  int64_t off = 0;
  do {
    const int64_t nb = std::min<int64_t>(slot_, nbytes - off);
    if (rank_ == root && nb > 0) std::memcpy(slot(root), data + off, nb);
    barrier();
    if (rank_ != root && nb > 0) std::memcpy(data + off, slot(root), nb);
    barrier();
    off += slot_;
  } while (off < nbytes);
}

at::Tensor ShmComm::all_to_all_v(const at::Tensor& x0, const std::vector<int64_t>& send_rows,
                                 const std::vector<int64_t>& recv_rows) {
  at::Tensor x = x0.contiguous();
  TFA_CHECK(!x.is_cuda() && x.dim() >= 1, "ShmComm.all_to_all_v: host tensor of rank >= 1 expected");
  const int W = size_;
  check_rows(x, send_rows, W);
  ++calls_;
  int64_t row_elems = 1;
  for (int d = 1; d < x.dim(); ++d) row_elems *= x.size(d);
  const int64_t rb = row_elems * x.element_size();
  // 1. row counts: every rank publishes what it sends to each rank
  for (int d = 0; d < W; ++d) meta(rank_)[d] = send_rows[d];
  barrier();
  std::string err;
  if (static_cast<int>(recv_rows.size()) != W) err = "all_to_all_v: bad receive counts";
  std::vector<int64_t> send_b(W), send_off(W), recv_b(W), recv_off(W);
  int64_t so = 0, ro = 0, total = 0, rounds = 0;
  const int64_t sub = std::max<int64_t>(slot_ / W / 256 * 256, 256);  // per-destination piece per round
  for (int r = 0; r < W; ++r) {
    send_b[r] = send_rows[r] * rb;
    send_off[r] = so;
    so += send_b[r];
    const int64_t got = meta(r)[rank_];
    if (err.empty() && static_cast<int>(recv_rows.size()) == W && got != recv_rows[r])
      err = str_cat("all_to_all_v: rank ", r, " sends ", got, " rows, ", recv_rows[r], " expected");
    recv_b[r] = got * rb;
    recv_off[r] = ro;
    ro += recv_b[r];
    total += got;
    for (int d = 0; d < W; ++d) rounds = std::max(rounds, (meta(r)[d] * rb + sub - 1) / sub);
  }
  if (!err.empty()) fail_all(err);  // every rank then fails at its next barrier instead of waiting
  barrier();  // the counts are read everywhere: the metadata may be reused
  std::vector<int64_t> sz = x.sizes().vec();
  sz[0] = total;
  at::Tensor out = at::empty(sz, x.options());
  const char* src = static_cast<const char*>(x.data_ptr());
  char* dst = static_cast<char*>(out.data_ptr());
  // 2. rounds: each rank's slot holds up to `sub` bytes for every destination
  for (int64_t q = 0; q < rounds; ++q) {
    const int64_t lo = q * sub;
    for (int d = 0; d < W; ++d) {
      const int64_t len = std::min(sub, send_b[d] - lo);
      if (len > 0) std::memcpy(slot(rank_) + d * sub, src + send_off[d] + lo, len);
    }
    barrier();
    for (int s = 0; s < W; ++s) {
      const int64_t len = std::min(sub, recv_b[s] - lo);
      if (len > 0) std::memcpy(dst + recv_off[s] + lo, slot(s) + rank_ * sub, len);
    }
    barrier();
  }
  return out;
}

}  // namespace comm
}  // namespace tfa

// Engine-owned communicators: FakeComm (threads), RcclComm (RCCL), OneShotComm
// (IPC single-hop all-reduce). See comm.h.
#include "comm.h"

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <rccl/rccl.h>

#include <chrono>
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
}

RcclComm::~RcclComm() {
  if (comm_) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::all_reduce(at::Tensor& t, k::RedOp op) {
  TFA_CHECK(t.is_cuda() && t.is_contiguous(), "RcclComm.all_reduce: contiguous device tensor expected");
  ++calls_;
  c10::hip::HIPGuard guard(t.device().index());
  TFA_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), nccl_op(op),
                         static_cast<ncclComm_t>(comm_), cur_stream(t)));
}

at::Tensor RcclComm::all_gather(const at::Tensor& t0) {
  at::Tensor t = t0.contiguous();
  TFA_CHECK(t.is_cuda(), "RcclComm.all_gather: device tensor expected");
  ++calls_;
  c10::hip::HIPGuard guard(t.device().index());
  std::vector<int64_t> sz = t.sizes().vec();
  sz.insert(sz.begin(), size_);
  at::Tensor out = pool_empty(sz, t.options());
  TFA_NCCL(ncclAllGather(t.data_ptr(), out.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()),
                         static_cast<ncclComm_t>(comm_), cur_stream(t)));
  return out;
}

at::Tensor RcclComm::all_to_all_v(const at::Tensor& x0, const std::vector<int64_t>& send_rows,
                                  const std::vector<int64_t>& recv_rows) {
  at::Tensor x = x0.contiguous();
  TFA_CHECK(x.is_cuda(), "RcclComm.all_to_all_v: device tensor expected");
  check_rows(x, send_rows, size_);
  TFA_CHECK(static_cast<int>(recv_rows.size()) == size_, "all_to_all_v: bad receive counts");
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
  return out;
}

void RcclComm::broadcast(at::Tensor& t, int root) {
  TFA_CHECK(t.is_cuda() && t.is_contiguous(), "RcclComm.broadcast: contiguous device tensor expected");
  ++calls_;
  c10::hip::HIPGuard guard(t.device().index());
  TFA_NCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t.scalar_type()), root,
                         static_cast<ncclComm_t>(comm_), cur_stream(t)));
}

void RcclComm::barrier() {
  // a one-element all-reduce on the current stream, then wait for it
  at::Tensor one = at::ones({1}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, device_));
  all_reduce(one, k::RedOp::SUM);
  TFA_CHECK(hipStreamSynchronize(cur_stream(one)) == hipSuccess, "RcclComm.barrier: stream sync failed");
}

void RcclComm::abort() {
  if (comm_) {
    (void)ncclCommAbort(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
  }
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
  TFA_CHECK(hipMalloc(&own_, k::kOneShotBufBytes) == hipSuccess, "OneShotComm: hipMalloc failed");
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
  ++calls_;
  ++epoch_;
  c10::hip::HIPGuard guard(t.device().index());
  k::oneshot_all_reduce(op, from_scalar_type(t.scalar_type()), t.data_ptr(), t.data_ptr(), t.numel(), rank_, size_,
                        peers_, epoch_, cur_stream(t));
}

void OneShotComm::check() {
  int err = 0;
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
  TFA_CHECK(hipMemcpy(&err, static_cast<char*>(own_) + k::kOneShotErrOffset, sizeof(err), hipMemcpyDeviceToHost) ==
                hipSuccess,
            "OneShotComm.check: hipMemcpy failed");
  TFA_CHECK(err == 0, "one-shot all-reduce timed out waiting for a peer's flag (a rank did not join)");
}

}  // namespace comm
}  // namespace tfa

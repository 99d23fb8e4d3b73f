// Engine-owned communicators.
//
// The reference moves data between partitions only through Spark: RDD.reduce
// of per-partition partial rows to the driver (reference
// src/main/scala/org/tensorframes/impl/DebugRowOps.scala:500, :524-525,
// :732-750), the groupBy hash shuffle (:576) and collect. Here one process
// drives one GPU and the cross-rank traffic goes through these objects,
// issued on the engine's own (current HIP) stream:
//
//   * RcclComm   — an RCCL communicator of its own (ncclCommInitRank; the
//                  unique id is exchanged over the bootstrap store), used for
//                  payloads above the one-shot size and for all-gather /
//                  grouped send-recv all-to-all / broadcast;
//   * OneShotComm — the small-message path: a single-hop all-reduce through
//                  IPC-mapped peer buffers (kernels/oneshot.hip), exchanged
//                  once; works for ranks that share a GPU too;
//   * FakeComm   — N in-process ranks (threads) over host memory: the CPU
//                  test double that runs the same collective contract at
//                  N = 2/4/8 without a GPU.
//
// Collective contract (all kinds): every rank calls the same collectives in
// the same order with tensors of the same dtype / shape (all_to_all_v: row
// counts that agree pairwise). all_reduce folds the ranks' values in rank
// order, so every rank gets bitwise the same result.
#pragma once

#include <torch/extension.h>
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../kernels/kernels.h"

namespace tfa {
namespace comm {

k::RedOp parse_op(const std::string& op);

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual std::string kind() const = 0;
  // in place
  virtual void all_reduce(at::Tensor& t, k::RedOp op) = 0;
  // [size, *t.shape]
  virtual at::Tensor all_gather(const at::Tensor& t) = 0;
  // x: rows ordered by destination (send_rows[r] rows for rank r); returns
  // the received rows in source-rank order (recv_rows[s] from rank s)
  virtual at::Tensor all_to_all_v(const at::Tensor& x, const std::vector<int64_t>& send_rows,
                                  const std::vector<int64_t>& recv_rows) = 0;
  virtual void broadcast(at::Tensor& t, int root) = 0;
  virtual void barrier() = 0;
  int64_t calls() const { return calls_; }

 protected:
  int64_t calls_ = 0;
};

// ---------------------------------------------------------------- FakeComm
class FakeWorld {
 public:
  explicit FakeWorld(int n);
  int size() const { return n_; }
  void barrier();
  // publish this rank's tensor (and row counts), wait for everyone; the
  // returned views stay valid until the matching release()
  const std::vector<at::Tensor>& exchange(int rank, const at::Tensor& t, const std::vector<int64_t>& meta,
                                          std::vector<std::vector<int64_t>>* metas);
  void release() { barrier(); }

 private:
  int n_;
  std::mutex mu_;
  std::condition_variable cv_;
  int arrived_ = 0;
  uint64_t gen_ = 0;
  std::vector<at::Tensor> slots_;
  std::vector<std::vector<int64_t>> meta_;
};

class FakeComm : public Comm {
 public:
  FakeComm(std::shared_ptr<FakeWorld> w, int rank);
  int rank() const override { return rank_; }
  int size() const override { return w_->size(); }
  std::string kind() const override { return "fake"; }
  void all_reduce(at::Tensor& t, k::RedOp op) override;
  at::Tensor all_gather(const at::Tensor& t) override;
  at::Tensor all_to_all_v(const at::Tensor& x, const std::vector<int64_t>& send_rows,
                          const std::vector<int64_t>& recv_rows) override;
  void broadcast(at::Tensor& t, int root) override;
  void barrier() override { w_->barrier(); }

 private:
  std::shared_ptr<FakeWorld> w_;
  int rank_;
};

// ---------------------------------------------------------------- RCCL
std::string rccl_unique_id();  // 128 opaque bytes (rank 0 makes it, the store carries it)

class RcclComm : public Comm {
 public:
  RcclComm(const std::string& unique_id, int rank, int size, int device);
  ~RcclComm() override;
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string kind() const override { return "rccl"; }
  void all_reduce(at::Tensor& t, k::RedOp op) override;
  at::Tensor all_gather(const at::Tensor& t) override;
  at::Tensor all_to_all_v(const at::Tensor& x, const std::vector<int64_t>& send_rows,
                          const std::vector<int64_t>& recv_rows) override;
  void broadcast(at::Tensor& t, int root) override;
  void barrier() override;
  void abort();  // ncclCommAbort: unblocks a hung collective (timeout guard)
  std::string async_error();  // "" while healthy

 private:
  void* comm_ = nullptr;  // ncclComm_t
  int rank_, size_, device_;
};

// ---------------------------------------------------------------- one-shot
class OneShotComm {
 public:
  OneShotComm(int rank, int size, int device);
  ~OneShotComm();
  std::string ipc_handle() const;                        // this rank's buffer, for the peers
  void open(const std::vector<std::string>& handles);   // every rank's handle, in rank order
  bool ready() const { return ready_; }
  static int64_t max_bytes() { return static_cast<int64_t>(k::kOneShotSlotBytes); }
  // in place, on the device's current stream
  void all_reduce(at::Tensor& t, k::RedOp op);
  // throws if a flag wait timed out (reads the error word: synchronises)
  void check();
  int64_t calls() const { return calls_; }

 private:
  int rank_, size_, device_;
  void* own_ = nullptr;
  k::OneShotPeers peers_{};
  std::vector<void*> opened_;
  uint32_t epoch_ = 0;
  bool ready_ = false;
  int64_t calls_ = 0;
};

}  // namespace comm
}  // namespace tfa

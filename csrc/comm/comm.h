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
//   * ShmComm    — host tensors of the ranks of ONE node through a POSIX
//                  shared-memory segment (process-shared barrier + per-rank
//                  slots): the data path of CPU-only multi-process jobs and
//                  of the host-side control collectives of GPU jobs, in
//                  place of gloo's TCP loopback;
//   * FakeComm   — N in-process ranks (threads) over host memory: the CPU
//                  test double that runs the same collective contract at
//                  N = 2/4/8 without a GPU.
//
// Failure detection (the reference relied on Spark task failure
// around RDD.reduce and the shuffle, DebugRowOps.scala:500, :524-525, :576):
// every RcclComm collective records an event; wait() is a bounded wait on
// them that raises CollectiveError past the timeout, and a watchdog thread
// ends a process whose collective is still incomplete past the timeout plus a
// grace period (the main thread is stuck somewhere it cannot raise: it calls
// ncclCommAbort, prints the reason and exits with kExitCollectiveTimeout, so
// the launcher tears the job down). OneShotComm's flag waits and ShmComm's
// barriers are bounded by the same timeout.
//
// Collective contract (all kinds): every rank calls the same collectives in
// the same order with tensors of the same dtype / shape (all_to_all_v: row
// counts that agree pairwise). all_reduce folds the ranks' values in rank
// order, so every rank gets bitwise the same result.
#pragma once

#include <torch/extension.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../kernels/kernels.h"

namespace tfa {
namespace comm {

k::RedOp parse_op(const std::string& op);

// a collective that timed out, or a communicator that failed asynchronously
struct CollectiveError : std::runtime_error {
  explicit CollectiveError(const std::string& m) : std::runtime_error(m) {}
};

constexpr int kExitCollectiveTimeout = 76;  // exit status of a rank ended by the watchdog

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
  // seconds a collective may take (<= 0: unbounded) and whether the watchdog
  // ends the process when the main thread does not notice a stuck one
  void set_timeout(double seconds, bool exit_on_timeout);
  double timeout() const { return timeout_s_; }
  // bounded wait for every collective issued so far; raises CollectiveError
  // past the timeout (the comm is then failed: later calls raise too)
  void wait();
  // raises CollectiveError if the comm failed (timeout, async RCCL error)
  void check();
  bool failed() const { return failed_.load(); }
  int64_t inflight() const;
  // tests: all_reduce runs a spin kernel of this many seconds between its
  // start event and the RCCL call (a collective that started but does not
  // finish; RCCL refuses the two ranks on one device a real hang needs)
  void set_test_stall(double seconds) { test_stall_s_ = seconds; }

 private:
  // events around a collective, for wait() and the watchdog: a collective's
  // age counts from when its start event completed (the work queued ahead of
  // it on the stream has finished), not from when it was enqueued
  hipEvent_t begin(hipStream_t s);
  void track(hipStream_t s, hipEvent_t start);
  void fail(const std::string& why);
  // ncclCommAbort on a helper thread, given 2 s (releases a collective kernel
  // that waits for a peer); the communicator is unusable afterwards
  void abort_comm(std::unique_lock<std::mutex>& held);
  void watchdog();
  void* comm_ = nullptr;  // ncclComm_t
  int rank_, size_, device_;
  double timeout_s_ = 0;
  bool exit_on_timeout_ = true;
  double test_stall_s_ = 0;
  struct Inflight {
    hipEvent_t ev;     // after the collective
    hipEvent_t start;  // before it (null: counted from enqueue)
    std::chrono::steady_clock::time_point t0;  // enqueue, then the first time start was seen complete
    bool started;
  };
  hipEvent_t take_event();
  // the age of the oldest in-flight collective (0 while it has not started); wmu_ held
  double front_age();
  mutable std::mutex wmu_;
  std::condition_variable wcv_;
  std::deque<Inflight> inflight_;
  std::vector<hipEvent_t> free_events_;
  std::atomic<bool> failed_{false}, stop_{false};
  std::string fail_msg_;
  std::thread wd_;
};

// ---------------------------------------------------------------- one-shot
class OneShotComm {
 public:
  // the buffer is allocated uncached (hipDeviceMallocUncached) so no GPU's L2
  // holds lines a peer writes over xGMI; fine-grained, then plain hipMalloc
  // are the fallbacks (alloc_kind() says which; the self-test in
  // parallel/comm.py decides whether the path is used at all)
  OneShotComm(int rank, int size, int device);
  ~OneShotComm();
  std::string ipc_handle() const;                        // this rank's buffer, for the peers
  void open(const std::vector<std::string>& handles);   // every rank's handle, in rank order
  bool ready() const { return ready_; }
  static int64_t max_bytes() { return static_cast<int64_t>(k::kOneShotSlotBytes); }
  // in place, on the device's current stream
  void all_reduce(at::Tensor& t, k::RedOp op);
  // throws CollectiveError if a flag wait timed out (reads the error word:
  // synchronises; the word is cleared, the comm stays failed)
  void check();
  int64_t calls() const { return calls_; }
  void set_timeout(double seconds) { timeout_us_ = seconds > 0 ? static_cast<uint64_t>(seconds * 1e6) : 3600000000ull; }
  const std::string& alloc_kind() const { return alloc_kind_; }
  bool failed() const { return failed_; }

 private:
  int rank_, size_, device_;
  uint64_t timeout_us_ = 600000000ull;
  bool failed_ = false;
  std::string alloc_kind_;
  void* own_ = nullptr;
  k::OneShotPeers peers_{};
  std::vector<void*> opened_;
  uint32_t epoch_ = 0;
  bool ready_ = false;
  int64_t calls_ = 0;
};

// ---------------------------------------------------------------- ShmComm
// Layout of the segment: [control block][result slot][slot of rank 0]...[slot
// of rank W-1]; control = a process-shared sense-reversing barrier and, per
// rank, kMaxRanks int64 of metadata (all_to_all_v row counts). Every collective moves
// its payload through the slots in rounds of at most `slot_bytes`.
class ShmComm : public Comm {
 public:
  static constexpr int kMaxRanks = 64;
  // rank 0 creates the segment (create = true), the others attach after it;
  // unlink() once every rank is attached (the mapping stays valid)
  ShmComm(const std::string& name, int rank, int size, int64_t slot_bytes, bool create);
  ~ShmComm() override;
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string kind() const override { return "shm"; }
  void all_reduce(at::Tensor& t, k::RedOp op) override;
  at::Tensor all_gather(const at::Tensor& t) override;
  at::Tensor all_to_all_v(const at::Tensor& x, const std::vector<int64_t>& send_rows,
                          const std::vector<int64_t>& recv_rows) override;
  void broadcast(at::Tensor& t, int root) override;
  void barrier() override;
  void unlink();
  void set_timeout(double seconds) { timeout_s_ = seconds; }
  // failure agreement (parallel/dist.agreed): a rank whose local phase
  // failed poisons the segment, so every rank waiting in (or entering) a
  // collective raises at once; once every rank has left the communicator
  // (synchronised on another channel) rank 0 clears the barrier state
  void poison();
  void reset_after_failure();
  bool poisoned() const;
  int64_t slot_bytes() const { return slot_; }
  int attached() const;  // ranks that have mapped the segment so far

 private:
  struct Ctrl;
  char* slot(int r) const;
  char* result() const;
  int64_t* meta(int r) const;
  [[noreturn]] void fail_all(const std::string& why);
  std::string name_;
  int rank_, size_;
  int64_t slot_;
  size_t bytes_ = 0;
  char* base_ = nullptr;
  double timeout_s_ = 600;
  bool linked_ = false;
};

}  // namespace comm
}  // namespace tfa

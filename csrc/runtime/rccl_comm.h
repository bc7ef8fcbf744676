// RCCL communicator: the framework's GPU collective backend (RCCL over xGMI on MI355X).
//
// One communicator per (process group, device).  The unique id is created by the group's rank 0
// and distributed through the TCP store by the Python layer; every call enqueues on the HIP stream
// the caller passes (the framework's dedicated communication stream), so collectives overlap with
// compute on other streams and can be captured into hipGraphs.  Buffers are raw device pointers.
#pragma once
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

namespace pde {

class RcclComm {
 public:
  RcclComm(const std::string& unique_id, int rank, int world, int device);
  ~RcclComm();
  static std::string make_unique_id();
  static int version();

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }

  void all_reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream);
  void broadcast(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int root, uintptr_t stream);
  void reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, int root, uintptr_t stream);
  void all_gather(uintptr_t send, uintptr_t recv, int64_t count_per_rank, int dtype, uintptr_t stream);
  void reduce_scatter(uintptr_t send, uintptr_t recv, int64_t count_per_rank, int dtype, int op, uintptr_t stream);
  void all_to_all(uintptr_t send, uintptr_t recv, int64_t count_per_rank, int dtype, uintptr_t stream);
  void send(uintptr_t buf, int64_t count, int dtype, int peer, uintptr_t stream);
  void recv(uintptr_t buf, int64_t count, int dtype, int peer, uintptr_t stream);
  void group_start();
  void group_end();
  std::shared_ptr<RcclComm> split(int color, int key);
  void abort();
  void destroy();
  std::string async_error();
  int comm_count() const;   // ncclCommCount: ranks RCCL itself sees in this communicator
  int cu_device() const;    // ncclCommCuDevice: the HIP device RCCL bound this rank to

 private:
  explicit RcclComm(ncclComm_t c, int device);
  ncclComm_t get() const;
  std::atomic<ncclComm_t> comm_{nullptr};   // nulled by abort() (possibly from the watchdog thread)
  int rank_ = 0, world_ = 1, device_ = 0;
};

// Failure detection for GPU collectives ("failure detection"): every collective the
// Python layer enqueues is followed by `watch(stream)`, which records a private HIP event behind
// it.  A background thread polls the events; one that is still pending after `timeout_ms` (a peer
// died or hangs, so the RCCL kernel can never finish) -- or an asynchronous RCCL error -- aborts
// the communicator (ncclCommAbort unblocks the hung kernels) and latches an error message that the
// next wait / collective on the group raises.  No-op while the stream is being graph-captured.
class CommWatchdog {
 public:
  CommWatchdog(std::shared_ptr<RcclComm> comm, int64_t timeout_ms, int poll_ms);
  ~CommWatchdog();
  void watch(uintptr_t stream, const std::string& what);
  std::string error();
  int64_t pending();
  void stop();

 private:
  struct Item {
    hipEvent_t ev;
    std::chrono::steady_clock::time_point t0;
    std::string what;
  };
  void loop();
  std::shared_ptr<RcclComm> comm_;
  int64_t timeout_ms_;
  int poll_ms_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> items_;
  std::string error_;
  bool stop_ = false;
  std::thread th_;
};

}  // namespace pde

// RCCL communicator: the framework's GPU collective backend (RCCL over xGMI on MI355X).
//
// One communicator per (process group, device).  The unique id is created by the group's rank 0
// and distributed through the TCP store by the Python layer; every call enqueues on the HIP stream
// the caller passes (the framework's dedicated communication stream), so collectives overlap with
// compute on other streams and can be captured into hipGraphs.  Buffers are raw device pointers.
#pragma once
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <memory>
#include <string>

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

 private:
  explicit RcclComm(ncclComm_t c, int device);
  void check_open() const;
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, world_ = 1, device_ = 0;
};

}  // namespace pde

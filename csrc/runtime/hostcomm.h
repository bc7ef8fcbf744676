// Host-memory collectives over TCP (the framework's CPU backend; the role ProcessGroupGloo plays in
// the reference's `--backend gloo` runs, /root/reference/toy/main.py:41).
//
// Full mesh of TCP connections bootstrapped through the rendezvous store.  Large all-reduces use a
// ring reduce-scatter + all-gather (bandwidth optimal, 2(W-1)/W bytes per rank), small ones a direct
// exchange reduced in rank order; both give bitwise-identical results on every rank.  All socket
// I/O is poll()-driven full duplex, so simultaneous send/recv on a pair never deadlocks.  Every op
// runs on one worker thread in submission order: synchronous calls are submit+wait, asynchronous
// ones return a Work handle (used by DDP to overlap gradient reduction with backward).
#pragma once
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "store.h"

namespace pde {

enum class DType : int { F32 = 0, F64 = 1, I32 = 2, I64 = 3, U8 = 4, I8 = 5, BF16 = 6, F16 = 7, BOOL = 8 };
enum class ROp : int { SUM = 0, PRODUCT = 1, MIN = 2, MAX = 3, AVG = 4, BAND = 5, BOR = 6, BXOR = 7 };

size_t dtype_size(DType d);
void reduce_into(void* dst, const void* src, int64_t count, DType d, ROp op);
void finalize_avg(void* buf, int64_t count, DType d, int world);

class Work {
 public:
  explicit Work(std::shared_future<void> f) : f_(std::move(f)) {}
  void wait() { f_.get(); }
  bool is_completed() const { return f_.wait_for(std::chrono::seconds(0)) == std::future_status::ready; }

 private:
  std::shared_future<void> f_;
};

class HostComm {
 public:
  HostComm(std::shared_ptr<StoreClient> store, const std::string& prefix, int rank, int world, int64_t timeout_ms);
  ~HostComm();
  int rank() const { return rank_; }
  int world() const { return world_; }

  std::shared_ptr<Work> submit(std::function<void()> fn);

  // blocking primitives (run on the worker thread via submit)
  void allreduce(void* buf, int64_t count, DType d, ROp op);
  void broadcast(void* buf, int64_t bytes, int root);
  void allgather(const void* in, void* out, int64_t bytes);
  void reduce_scatter(const void* in, void* out, int64_t count_per_rank, DType d, ROp op);
  void reduce(void* buf, int64_t count, DType d, ROp op, int root);
  void gather(const void* in, void* out, int64_t bytes, int root);
  void scatter(const void* in, void* out, int64_t bytes, int root);
  void alltoall(const void* in, void* out, int64_t bytes_per_rank);
  void p2p(const std::vector<std::tuple<int, uintptr_t, int64_t>>& sends,
           const std::vector<std::tuple<int, uintptr_t, int64_t>>& recvs);
  void send(const void* buf, int64_t bytes, int dst);
  void recv(void* buf, int64_t bytes, int src);
  void barrier();
  void shutdown();

 private:
  struct Xfer {
    int peer;
    const char* sbuf;
    size_t sn;
    char* rbuf;
    size_t rn;
  };
  void exchange(std::vector<Xfer>& ops);
  void ring_allreduce(char* buf, int64_t count, DType d, ROp op);
  void direct_allreduce(char* buf, int64_t count, DType d, ROp op);
  Clock::time_point deadline() const { return Clock::now() + std::chrono::milliseconds(timeout_ms_); }
  void worker();

  std::shared_ptr<StoreClient> store_;
  int rank_, world_;
  int64_t timeout_ms_;
  std::vector<int> fds_;
  int listen_fd_ = -1;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<std::function<void()>, std::shared_ptr<std::promise<void>>>> q_;
  bool stop_ = false;
};

}  // namespace pde

// RCCL communicator: see rccl_comm.h.
#include "rccl_comm.h"

#include <chrono>
#include <cstring>
#include <stdexcept>

namespace pde {

namespace {

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(r));
}

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP ") + what + " failed: " + hipGetErrorString(e));
}

// framework dtype codes (same numbering as hostcomm.h DType)
ncclDataType_t to_nccl_dtype(int d) {
  switch (d) {
    case 0: return ncclFloat32;
    case 1: return ncclFloat64;
    case 2: return ncclInt32;
    case 3: return ncclInt64;
    case 4: return ncclUint8;
    case 5: return ncclInt8;
    case 6: return ncclBfloat16;
    case 7: return ncclFloat16;
    case 8: return ncclUint8;
  }
  throw std::invalid_argument("dtype not supported by RCCL");
}

size_t nccl_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;
  }
}

ncclRedOp_t to_nccl_op(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMin;
    case 3: return ncclMax;
    case 4: return ncclAvg;
  }
  throw std::invalid_argument("reduce op not supported by RCCL (bitwise ops are host-only)");
}

hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
void* P(uintptr_t p) { return reinterpret_cast<void*>(p); }

}  // namespace

std::string RcclComm::make_unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

int RcclComm::version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

RcclComm::RcclComm(const std::string& unique_id, int rank, int world, int device)
    : rank_(rank), world_(world), device_(device) {
  if (unique_id.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("bad RCCL unique id");
  ncclUniqueId id;
  std::memcpy(&id, unique_id.data(), sizeof(id));
  hip_check(hipSetDevice(device), "hipSetDevice");
  ncclComm_t c = nullptr;
  nccl_check(ncclCommInitRank(&c, world, id, rank), "ncclCommInitRank");
  comm_.store(c);
}

RcclComm::RcclComm(ncclComm_t c, int device) : comm_(c), device_(device) {
  nccl_check(ncclCommUserRank(c, &rank_), "ncclCommUserRank");
  nccl_check(ncclCommCount(c, &world_), "ncclCommCount");
}

RcclComm::~RcclComm() {
  try {
    destroy();
  } catch (...) {
  }
}

ncclComm_t RcclComm::get() const {
  ncclComm_t c = comm_.load();
  if (!c) throw std::runtime_error("RCCL communicator is destroyed or aborted");
  return c;
}

void RcclComm::all_reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream) {
  ncclComm_t comm = get();
  nccl_check(ncclAllReduce(P(send), P(recv), (size_t)count, to_nccl_dtype(dtype), to_nccl_op(op), comm, S(stream)),
             "ncclAllReduce");
}

void RcclComm::broadcast(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int root, uintptr_t stream) {
  ncclComm_t comm = get();
  nccl_check(ncclBroadcast(P(send), P(recv), (size_t)count, to_nccl_dtype(dtype), root, comm, S(stream)),
             "ncclBroadcast");
}

void RcclComm::reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, int root, uintptr_t stream) {
  ncclComm_t comm = get();
  nccl_check(ncclReduce(P(send), P(recv), (size_t)count, to_nccl_dtype(dtype), to_nccl_op(op), root, comm, S(stream)),
             "ncclReduce");
}

void RcclComm::all_gather(uintptr_t send, uintptr_t recv, int64_t count, int dtype, uintptr_t stream) {
  ncclComm_t comm = get();
  nccl_check(ncclAllGather(P(send), P(recv), (size_t)count, to_nccl_dtype(dtype), comm, S(stream)), "ncclAllGather");
}

void RcclComm::reduce_scatter(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream) {
  ncclComm_t comm = get();
  nccl_check(ncclReduceScatter(P(send), P(recv), (size_t)count, to_nccl_dtype(dtype), to_nccl_op(op), comm,
                               S(stream)),
             "ncclReduceScatter");
}

void RcclComm::all_to_all(uintptr_t send, uintptr_t recv, int64_t count, int dtype, uintptr_t stream) {
  ncclComm_t comm = get();
  const ncclDataType_t t = to_nccl_dtype(dtype);
  const size_t bytes = (size_t)count * nccl_size(t);
  nccl_check(ncclGroupStart(), "ncclGroupStart");
  for (int p = 0; p < world_; ++p) {
    nccl_check(ncclSend((const char*)P(send) + p * bytes, (size_t)count, t, p, comm, S(stream)), "ncclSend");
    nccl_check(ncclRecv((char*)P(recv) + p * bytes, (size_t)count, t, p, comm, S(stream)), "ncclRecv");
  }
  nccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

void RcclComm::send(uintptr_t buf, int64_t count, int dtype, int peer, uintptr_t stream) {
  ncclComm_t comm = get();
  nccl_check(ncclSend(P(buf), (size_t)count, to_nccl_dtype(dtype), peer, comm, S(stream)), "ncclSend");
}

void RcclComm::recv(uintptr_t buf, int64_t count, int dtype, int peer, uintptr_t stream) {
  ncclComm_t comm = get();
  nccl_check(ncclRecv(P(buf), (size_t)count, to_nccl_dtype(dtype), peer, comm, S(stream)), "ncclRecv");
}

void RcclComm::group_start() { nccl_check(ncclGroupStart(), "ncclGroupStart"); }
void RcclComm::group_end() { nccl_check(ncclGroupEnd(), "ncclGroupEnd"); }

std::shared_ptr<RcclComm> RcclComm::split(int color, int key) {
  ncclComm_t comm = get();
  ncclComm_t out = nullptr;
  nccl_check(ncclCommSplit(comm, color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &out, nullptr), "ncclCommSplit");
  if (!out) return nullptr;
  return std::shared_ptr<RcclComm>(new RcclComm(out, device_));
}

void RcclComm::abort() {
  ncclComm_t c = comm_.exchange(nullptr);
  if (c) ncclCommAbort(c);
}

void RcclComm::destroy() {
  ncclComm_t c = comm_.exchange(nullptr);
  if (c) ncclCommDestroy(c);
}

int RcclComm::comm_count() const {
  int n = 0;
  nccl_check(ncclCommCount(get(), &n), "ncclCommCount");
  return n;
}

int RcclComm::cu_device() const {
  int d = -1;
  nccl_check(ncclCommCuDevice(get(), &d), "ncclCommCuDevice");
  return d;
}

std::string RcclComm::async_error() {
  ncclComm_t c = comm_.load();
  if (!c) return "destroyed";
  ncclResult_t r = ncclSuccess;
  ncclCommGetAsyncError(c, &r);
  return r == ncclSuccess ? "" : ncclGetErrorString(r);
}

// ------------------------------------------------------------------------------------ watchdog
CommWatchdog::CommWatchdog(std::shared_ptr<RcclComm> comm, int64_t timeout_ms, int poll_ms)
    : comm_(std::move(comm)), timeout_ms_(timeout_ms), poll_ms_(poll_ms < 1 ? 1 : poll_ms) {
  th_ = std::thread([this] { loop(); });
}

CommWatchdog::~CommWatchdog() { stop(); }

void CommWatchdog::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  for (auto& it : items_) hipEventDestroy(it.ev);
  items_.clear();
}

void CommWatchdog::watch(uintptr_t stream, const std::string& what) {
  hipStream_t s = S(stream);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return;
  hipEvent_t ev = nullptr;
  hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreateWithFlags");
  hip_check(hipEventRecord(ev, s), "hipEventRecord");
  {
    std::lock_guard<std::mutex> g(mu_);
    items_.push_back(Item{ev, std::chrono::steady_clock::now(), what});
  }
  cv_.notify_all();
}

std::string CommWatchdog::error() {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

int64_t CommWatchdog::pending() {
  std::lock_guard<std::mutex> g(mu_);
  return (int64_t)items_.size();
}

void CommWatchdog::loop() {
  hipSetDevice(comm_->device());
  // The polls below must not count as unsafe calls against a capture another thread runs in the
  // default (global) mode -- a hipEventQuery there invalidates that capture. Relaxed mode exempts
  // this thread; the events it queries are never part of a capture (watch() skips capturing streams).
  hipStreamCaptureMode relaxed = hipStreamCaptureModeRelaxed;
  hipThreadExchangeStreamCaptureMode(&relaxed);
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    if (items_.empty()) {
      cv_.wait(lk, [this] { return stop_ || !items_.empty(); });
      continue;
    }
    // completed events retire in order; the oldest pending one decides the timeout
    while (!items_.empty()) {
      const hipError_t q = hipEventQuery(items_.front().ev);
      if (q == hipErrorNotReady) break;
      hipEventDestroy(items_.front().ev);
      items_.pop_front();
    }
    std::string fail;
    if (!items_.empty() && error_.empty()) {
      const auto age = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() -
                                                                             items_.front().t0).count();
      if (age > timeout_ms_)
        fail = "RCCL watchdog: collective '" + items_.front().what + "' did not complete within " +
               std::to_string(timeout_ms_) + " ms (peer failure or hang); communicator aborted";
    }
    if (fail.empty() && error_.empty()) {
      const std::string ae = comm_->async_error();
      if (!ae.empty() && ae != "destroyed") fail = "RCCL asynchronous error: " + ae + "; communicator aborted";
    }
    if (!fail.empty()) {
      error_ = fail;
      lk.unlock();
      comm_->abort();                       // unblocks the hung RCCL kernels
      lk.lock();
      for (auto& it : items_) hipEventDestroy(it.ev);
      items_.clear();
      continue;
    }
    cv_.wait_for(lk, std::chrono::milliseconds(poll_ms_), [this] { return stop_; });
  }
}

}  // namespace pde

// Host TCP collectives: see hostcomm.h.
#include "hostcomm.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace pde {

size_t dtype_size(DType d) {
  switch (d) {
    case DType::F32: case DType::I32: return 4;
    case DType::F64: case DType::I64: return 8;
    case DType::U8: case DType::I8: case DType::BOOL: return 1;
    case DType::BF16: case DType::F16: return 2;
  }
  throw std::invalid_argument("bad dtype");
}

namespace {

inline float bf16_to_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);   // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float f16_to_f(uint16_t h) {
  const uint32_t s = (h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ffu;
  uint32_t u;
  if (e == 0) {
    if (m == 0) u = s;
    else {  // subnormal
      float f = std::ldexp((float)m, -24);
      std::memcpy(&u, &f, 4);
      u |= s;
    }
  } else if (e == 31) {
    u = s | 0x7f800000u | (m << 13);
  } else {
    u = s | ((e + 112) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f_to_f16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t s = (u >> 16) & 0x8000u;
  const int e = (int)((u >> 23) & 0xff) - 127 + 15;
  uint32_t m = u & 0x7fffffu;
  if (((u >> 23) & 0xff) == 0xff) return (uint16_t)(s | 0x7c00u | (m ? 0x200u : 0));
  if (e >= 31) return (uint16_t)(s | 0x7c00u);
  if (e <= 0) {
    if (e < -10) return (uint16_t)s;
    m |= 0x800000u;
    const int shift = 14 - e;
    uint32_t r = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (r & 1))) ++r;
    return (uint16_t)(s | r);
  }
  uint32_t r = ((uint32_t)e << 10) | (m >> 13);
  const uint32_t rem = m & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (r & 1))) ++r;
  return (uint16_t)(s | r);
}

template <typename T>
void red(T* d, const T* s, int64_t n, ROp op) {
  switch (op) {
    case ROp::SUM: case ROp::AVG: for (int64_t i = 0; i < n; ++i) d[i] = d[i] + s[i]; break;
    case ROp::PRODUCT: for (int64_t i = 0; i < n; ++i) d[i] = d[i] * s[i]; break;
    case ROp::MIN: for (int64_t i = 0; i < n; ++i) d[i] = std::min(d[i], s[i]); break;
    case ROp::MAX: for (int64_t i = 0; i < n; ++i) d[i] = std::max(d[i], s[i]); break;
    default: throw std::invalid_argument("bitwise reduction needs an integer dtype");
  }
}

template <typename T>
void red_int(T* d, const T* s, int64_t n, ROp op) {
  switch (op) {
    case ROp::BAND: for (int64_t i = 0; i < n; ++i) d[i] &= s[i]; break;
    case ROp::BOR: for (int64_t i = 0; i < n; ++i) d[i] |= s[i]; break;
    case ROp::BXOR: for (int64_t i = 0; i < n; ++i) d[i] ^= s[i]; break;
    default: red(d, s, n, op);
  }
}

template <float (*L)(uint16_t), uint16_t (*S)(float)>
void red_half(uint16_t* d, const uint16_t* s, int64_t n, ROp op) {
  for (int64_t i = 0; i < n; ++i) {
    float a = L(d[i]), b = L(s[i]), r;
    switch (op) {
      case ROp::SUM: case ROp::AVG: r = a + b; break;
      case ROp::PRODUCT: r = a * b; break;
      case ROp::MIN: r = std::min(a, b); break;
      case ROp::MAX: r = std::max(a, b); break;
      default: throw std::invalid_argument("bitwise reduction needs an integer dtype");
    }
    d[i] = S(r);
  }
}

}  // namespace

void reduce_into(void* dst, const void* src, int64_t n, DType d, ROp op) {
  switch (d) {
    case DType::F32: red((float*)dst, (const float*)src, n, op); break;
    case DType::F64: red((double*)dst, (const double*)src, n, op); break;
    case DType::I32: red_int((int32_t*)dst, (const int32_t*)src, n, op); break;
    case DType::I64: red_int((int64_t*)dst, (const int64_t*)src, n, op); break;
    case DType::U8: red_int((uint8_t*)dst, (const uint8_t*)src, n, op); break;
    case DType::I8: red_int((int8_t*)dst, (const int8_t*)src, n, op); break;
    case DType::BOOL: {
      auto* a = (uint8_t*)dst;
      auto* b = (const uint8_t*)src;
      for (int64_t i = 0; i < n; ++i) {
        switch (op) {
          case ROp::SUM: case ROp::MAX: case ROp::BOR: a[i] = (a[i] | b[i]) ? 1 : 0; break;
          case ROp::PRODUCT: case ROp::MIN: case ROp::BAND: a[i] = (a[i] & b[i]) ? 1 : 0; break;
          case ROp::BXOR: a[i] = (a[i] ^ b[i]) ? 1 : 0; break;
          default: throw std::invalid_argument("AVG on bool");
        }
      }
      break;
    }
    case DType::BF16: red_half<bf16_to_f, f_to_bf16>((uint16_t*)dst, (const uint16_t*)src, n, op); break;
    case DType::F16: red_half<f16_to_f, f_to_f16>((uint16_t*)dst, (const uint16_t*)src, n, op); break;
  }
}

void finalize_avg(void* buf, int64_t n, DType d, int world) {
  switch (d) {
    case DType::F32: { auto* p = (float*)buf; for (int64_t i = 0; i < n; ++i) p[i] /= (float)world; break; }
    case DType::F64: { auto* p = (double*)buf; for (int64_t i = 0; i < n; ++i) p[i] /= (double)world; break; }
    case DType::I32: { auto* p = (int32_t*)buf; for (int64_t i = 0; i < n; ++i) p[i] /= world; break; }
    case DType::I64: { auto* p = (int64_t*)buf; for (int64_t i = 0; i < n; ++i) p[i] /= world; break; }
    case DType::U8: { auto* p = (uint8_t*)buf; for (int64_t i = 0; i < n; ++i) p[i] /= world; break; }
    case DType::I8: { auto* p = (int8_t*)buf; for (int64_t i = 0; i < n; ++i) p[i] /= world; break; }
    case DType::BF16: {
      auto* p = (uint16_t*)buf;
      for (int64_t i = 0; i < n; ++i) p[i] = f_to_bf16(bf16_to_f(p[i]) / (float)world);
      break;
    }
    case DType::F16: {
      auto* p = (uint16_t*)buf;
      for (int64_t i = 0; i < n; ++i) p[i] = f_to_f16(f16_to_f(p[i]) / (float)world);
      break;
    }
    case DType::BOOL: throw std::invalid_argument("AVG on bool");
  }
}

// ------------------------------------------------------------------------------------------------
HostComm::HostComm(std::shared_ptr<StoreClient> store, const std::string& prefix, int rank, int world,
                   int64_t timeout_ms)
    : store_(std::move(store)), rank_(rank), world_(world), timeout_ms_(timeout_ms), fds_(world, -1) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("bad rank/world");
  if (world > 1) {
    int port = 0;
    listen_fd_ = tcp_listen("0.0.0.0", 0, &port, world);
    store_->set(prefix + "/addr/" + std::to_string(rank), store_->local_address() + ":" + std::to_string(port));
    const auto dl = deadline();
    // connect to lower ranks, accept from higher ranks
    for (int j = 0; j < rank; ++j) {
      const std::string a = store_->get(prefix + "/addr/" + std::to_string(j));
      const auto c = a.rfind(':');
      const int fd = tcp_connect(a.substr(0, c), std::stoi(a.substr(c + 1)), dl);
      set_bufsizes(fd, 4 << 20);
      const int32_t me = rank;
      send_all(fd, &me, 4, dl);
      fds_[j] = fd;
    }
    for (int k = rank + 1; k < world; ++k) {
      pollfd pf{listen_fd_, POLLIN, 0};
      while (true) {
        const int r = ::poll(&pf, 1, (int)std::min<int64_t>(ms_left(dl), 1000));
        if (r > 0) break;
        if (Clock::now() >= dl) throw TimeoutError("host comm: timed out waiting for peers to connect");
      }
      const int fd = ::accept(listen_fd_, nullptr, nullptr);
      if (fd < 0) throw NetError(errno_str("accept"));
      set_nodelay(fd);
      set_bufsizes(fd, 4 << 20);
      int32_t peer = -1;
      recv_all(fd, &peer, 4, dl);
      if (peer <= rank || peer >= world || fds_[peer] != -1) throw NetError("host comm: bad handshake");
      fds_[peer] = fd;
    }
    ::close(listen_fd_);
    listen_fd_ = -1;
  }
  th_ = std::thread([this] { worker(); });
}

HostComm::~HostComm() { shutdown(); }

void HostComm::shutdown() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  for (int& fd : fds_) {
    if (fd >= 0) ::close(fd);
    fd = -1;
  }
}

std::shared_ptr<Work> HostComm::submit(std::function<void()> fn) {
  auto pr = std::make_shared<std::promise<void>>();
  auto w = std::make_shared<Work>(pr->get_future().share());
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) throw std::runtime_error("host comm is shut down");
    q_.emplace_back(std::move(fn), pr);
  }
  cv_.notify_one();
  return w;
}

void HostComm::worker() {
  while (true) {
    std::pair<std::function<void()>, std::shared_ptr<std::promise<void>>> item;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      item = std::move(q_.front());
      q_.pop_front();
    }
    try {
      item.first();
      item.second->set_value();
    } catch (...) {
      item.second->set_exception(std::current_exception());
    }
  }
}

// Full-duplex progress over several peers at once.
void HostComm::exchange(std::vector<Xfer>& ops) {
  const auto dl = deadline();
  std::vector<size_t> sent(ops.size(), 0), got(ops.size(), 0);
  std::vector<pollfd> pf;
  std::vector<int> idx;
  while (true) {
    pf.clear();
    idx.clear();
    for (size_t i = 0; i < ops.size(); ++i) {
      // several transfers to one peer (point-to-point batches) progress strictly in list order per
      // direction: the byte streams of two sends to one socket must not interleave
      bool send_turn = true, recv_turn = true;
      for (size_t j = 0; j < i; ++j) {
        if (ops[j].peer != ops[i].peer) continue;
        if (sent[j] < ops[j].sn) send_turn = false;
        if (got[j] < ops[j].rn) recv_turn = false;
      }
      short ev = 0;
      if (send_turn && sent[i] < ops[i].sn) ev |= POLLOUT;
      if (recv_turn && got[i] < ops[i].rn) ev |= POLLIN;
      if (ev) {
        pf.push_back({fds_[ops[i].peer], ev, 0});
        idx.push_back((int)i);
      }
    }
    if (pf.empty()) return;
    const int r = ::poll(pf.data(), pf.size(), (int)std::min<int64_t>(ms_left(dl), 1000));
    if (r < 0) {
      if (errno == EINTR) continue;
      throw NetError(errno_str("poll"));
    }
    if (r == 0) {
      if (Clock::now() >= dl) throw TimeoutError("host comm: collective timed out (a peer may have died)");
      continue;
    }
    for (size_t k = 0; k < pf.size(); ++k) {
      const int i = idx[k];
      Xfer& x = ops[i];
      if (pf[k].revents & (POLLERR | POLLNVAL)) throw NetError("host comm: socket error with a peer");
      if ((pf[k].revents & POLLOUT) && sent[i] < x.sn) {
        const ssize_t n = ::send(pf[k].fd, x.sbuf + sent[i], std::min<size_t>(x.sn - sent[i], 1 << 20),
                                 MSG_DONTWAIT | MSG_NOSIGNAL);
        if (n > 0) sent[i] += (size_t)n;
        else if (n < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) throw NetError(errno_str("send"));
      }
      if ((pf[k].revents & (POLLIN | POLLHUP)) && got[i] < x.rn) {
        const ssize_t n = ::recv(pf[k].fd, x.rbuf + got[i], x.rn - got[i], MSG_DONTWAIT);
        if (n > 0) got[i] += (size_t)n;
        else if (n == 0) throw NetError("host comm: peer closed the connection");
        else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) throw NetError(errno_str("recv"));
      }
    }
  }
}

void HostComm::direct_allreduce(char* buf, int64_t count, DType d, ROp op) {
  const size_t bytes = (size_t)count * dtype_size(d);
  std::vector<char> all((size_t)world_ * bytes);
  std::memcpy(all.data() + (size_t)rank_ * bytes, buf, bytes);
  std::vector<Xfer> ops;
  for (int j = 0; j < world_; ++j)
    if (j != rank_) ops.push_back({j, buf, bytes, all.data() + (size_t)j * bytes, bytes});
  exchange(ops);
  // reduce in rank order: identical on every rank
  std::memcpy(buf, all.data(), bytes);
  for (int j = 1; j < world_; ++j) reduce_into(buf, all.data() + (size_t)j * bytes, count, d, op);
}

void HostComm::ring_allreduce(char* buf, int64_t count, DType d, ROp op) {
  const size_t es = dtype_size(d);
  const int W = world_, next = (rank_ + 1) % W, prev = (rank_ - 1 + W) % W;
  auto lo = [&](int c) { return (int64_t)c * count / W; };
  auto hi = [&](int c) { return (int64_t)(c + 1) * count / W; };
  int64_t maxc = 0;
  for (int c = 0; c < W; ++c) maxc = std::max(maxc, hi(c) - lo(c));
  std::vector<char> tmp((size_t)maxc * es);
  for (int s = 0; s < W - 1; ++s) {           // reduce-scatter: rank r ends owning chunk r+1
    const int sc = ((rank_ - s) % W + W) % W, rc = ((rank_ - s - 1) % W + W) % W;
    std::vector<Xfer> ops{{next, buf + lo(sc) * es, (size_t)(hi(sc) - lo(sc)) * es, nullptr, 0},
                          {prev, nullptr, 0, tmp.data(), (size_t)(hi(rc) - lo(rc)) * es}};
    if (next == prev) {
      ops = {{next, buf + lo(sc) * es, (size_t)(hi(sc) - lo(sc)) * es, tmp.data(), (size_t)(hi(rc) - lo(rc)) * es}};
    }
    exchange(ops);
    reduce_into(buf + lo(rc) * es, tmp.data(), hi(rc) - lo(rc), d, op);
  }
  for (int s = 0; s < W - 1; ++s) {           // all-gather of the reduced chunks
    const int sc = ((rank_ + 1 - s) % W + W) % W, rc = ((rank_ - s) % W + W) % W;
    std::vector<Xfer> ops{{next, buf + lo(sc) * es, (size_t)(hi(sc) - lo(sc)) * es, nullptr, 0},
                          {prev, nullptr, 0, buf + lo(rc) * es, (size_t)(hi(rc) - lo(rc)) * es}};
    if (next == prev) {
      ops = {{next, buf + lo(sc) * es, (size_t)(hi(sc) - lo(sc)) * es, buf + lo(rc) * es,
              (size_t)(hi(rc) - lo(rc)) * es}};
    }
    exchange(ops);
  }
}

void HostComm::allreduce(void* buf, int64_t count, DType d, ROp op) {
  if (world_ > 1 && count > 0) {
    const size_t bytes = (size_t)count * dtype_size(d);
    if (bytes <= (64u << 10) || count < world_) direct_allreduce((char*)buf, count, d, op);
    else ring_allreduce((char*)buf, count, d, op);
  }
  if (op == ROp::AVG) finalize_avg(buf, count, d, world_);
}

void HostComm::broadcast(void* buf, int64_t bytes, int root) {
  if (world_ == 1 || bytes == 0) return;
  std::vector<Xfer> ops;
  if (rank_ == root) {
    for (int j = 0; j < world_; ++j)
      if (j != root) ops.push_back({j, (const char*)buf, (size_t)bytes, nullptr, 0});
  } else {
    ops.push_back({root, nullptr, 0, (char*)buf, (size_t)bytes});
  }
  exchange(ops);
}

void HostComm::allgather(const void* in, void* out, int64_t bytes) {
  char* o = (char*)out;
  if ((const char*)in != o + (size_t)rank_ * bytes) std::memmove(o + (size_t)rank_ * bytes, in, (size_t)bytes);
  if (world_ == 1 || bytes == 0) return;
  const int W = world_, next = (rank_ + 1) % W, prev = (rank_ - 1 + W) % W;
  for (int s = 0; s < W - 1; ++s) {
    const int sc = ((rank_ - s) % W + W) % W, rc = ((rank_ - s - 1) % W + W) % W;
    std::vector<Xfer> ops{{next, o + (size_t)sc * bytes, (size_t)bytes, nullptr, 0},
                          {prev, nullptr, 0, o + (size_t)rc * bytes, (size_t)bytes}};
    if (next == prev) ops = {{next, o + (size_t)sc * bytes, (size_t)bytes, o + (size_t)rc * bytes, (size_t)bytes}};
    exchange(ops);
  }
}

void HostComm::reduce_scatter(const void* in, void* out, int64_t cnt, DType d, ROp op) {
  const size_t es = dtype_size(d), cb = (size_t)cnt * es;
  std::vector<char> work((size_t)world_ * cb);
  std::memcpy(work.data(), in, work.size());
  if (world_ > 1 && cnt > 0) {
    const int W = world_, next = (rank_ + 1) % W, prev = (rank_ - 1 + W) % W;
    std::vector<char> tmp(cb);
    for (int s = 0; s < W - 1; ++s) {         // rank r ends owning chunk r
      const int sc = ((rank_ - s - 1) % W + W) % W, rc = ((rank_ - s - 2) % W + W) % W;
      std::vector<Xfer> ops{{next, work.data() + sc * cb, cb, nullptr, 0}, {prev, nullptr, 0, tmp.data(), cb}};
      if (next == prev) ops = {{next, work.data() + sc * cb, cb, tmp.data(), cb}};
      exchange(ops);
      reduce_into(work.data() + rc * cb, tmp.data(), cnt, d, op);
    }
  }
  std::memcpy(out, work.data() + (size_t)rank_ * cb, cb);
  if (op == ROp::AVG) finalize_avg(out, cnt, d, world_);
}

void HostComm::reduce(void* buf, int64_t count, DType d, ROp op, int root) {
  if (rank_ == root) {
    allreduce(buf, count, d, op);
  } else {
    std::vector<char> tmp((size_t)count * dtype_size(d));
    std::memcpy(tmp.data(), buf, tmp.size());
    allreduce(tmp.data(), count, d, op);
  }
}

void HostComm::gather(const void* in, void* out, int64_t bytes, int root) {
  if (rank_ == root) {
    char* o = (char*)out;
    std::memmove(o + (size_t)root * bytes, in, (size_t)bytes);
    std::vector<Xfer> ops;
    for (int j = 0; j < world_; ++j)
      if (j != root) ops.push_back({j, nullptr, 0, o + (size_t)j * bytes, (size_t)bytes});
    exchange(ops);
  } else {
    std::vector<Xfer> ops{{root, (const char*)in, (size_t)bytes, nullptr, 0}};
    exchange(ops);
  }
}

void HostComm::scatter(const void* in, void* out, int64_t bytes, int root) {
  if (rank_ == root) {
    const char* i = (const char*)in;
    std::vector<Xfer> ops;
    for (int j = 0; j < world_; ++j)
      if (j != root) ops.push_back({j, i + (size_t)j * bytes, (size_t)bytes, nullptr, 0});
    exchange(ops);
    std::memmove(out, i + (size_t)root * bytes, (size_t)bytes);
  } else {
    std::vector<Xfer> ops{{root, nullptr, 0, (char*)out, (size_t)bytes}};
    exchange(ops);
  }
}

void HostComm::alltoall(const void* in, void* out, int64_t b) {
  const char* i = (const char*)in;
  char* o = (char*)out;
  std::memmove(o + (size_t)rank_ * b, i + (size_t)rank_ * b, (size_t)b);
  std::vector<Xfer> ops;
  for (int j = 0; j < world_; ++j)
    if (j != rank_) ops.push_back({j, i + (size_t)j * b, (size_t)b, o + (size_t)j * b, (size_t)b});
  exchange(ops);
}

void HostComm::p2p(const std::vector<std::tuple<int, uintptr_t, int64_t>>& sends,
                   const std::vector<std::tuple<int, uintptr_t, int64_t>>& recvs) {
  // one full-duplex exchange for a whole batch of sends and receives: a pairwise exchange whose
  // payload exceeds the socket buffers cannot deadlock (both sides read while they write)
  std::vector<Xfer> ops;
  for (const auto& s : sends) {
    const int p = std::get<0>(s);
    if (p < 0 || p >= world_ || p == rank_) throw std::invalid_argument("p2p: bad destination rank");
    ops.push_back({p, reinterpret_cast<const char*>(std::get<1>(s)), (size_t)std::get<2>(s), nullptr, 0});
  }
  for (const auto& r : recvs) {
    const int p = std::get<0>(r);
    if (p < 0 || p >= world_ || p == rank_) throw std::invalid_argument("p2p: bad source rank");
    ops.push_back({p, nullptr, 0, reinterpret_cast<char*>(std::get<1>(r)), (size_t)std::get<2>(r)});
  }
  exchange(ops);
}

void HostComm::send(const void* buf, int64_t bytes, int dst) {
  if (dst == rank_ || dst < 0 || dst >= world_) throw std::invalid_argument("bad send peer");
  std::vector<Xfer> ops{{dst, (const char*)buf, (size_t)bytes, nullptr, 0}};
  exchange(ops);
}

void HostComm::recv(void* buf, int64_t bytes, int src) {
  if (src == rank_ || src < 0 || src >= world_) throw std::invalid_argument("bad recv peer");
  std::vector<Xfer> ops{{src, nullptr, 0, (char*)buf, (size_t)bytes}};
  exchange(ops);
}

void HostComm::barrier() {
  int32_t one = 1;
  allreduce(&one, 1, DType::I32, ROp::SUM);
}

}  // namespace pde

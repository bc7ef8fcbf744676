// TCP rendezvous store: see store.h.  Wire format (little endian):
//   request  = u32 len | u8 cmd | payload        reply = u32 len | payload
//   str      = u32 len | bytes
#include "store.h"

#include <algorithm>

namespace pde {

void put_u32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
void put_i64(std::string& s, int64_t v) { s.append(reinterpret_cast<const char*>(&v), 8); }
void put_str(std::string& s, const std::string& v) {
  put_u32(s, (uint32_t)v.size());
  s.append(v);
}

namespace {

struct Reader {
  const std::string& s;
  size_t p;
  bool ok = true;
  uint32_t u32() {
    if (p + 4 > s.size()) { ok = false; return 0; }
    uint32_t v;
    std::memcpy(&v, s.data() + p, 4);
    p += 4;
    return v;
  }
  int64_t i64() {
    if (p + 8 > s.size()) { ok = false; return 0; }
    int64_t v;
    std::memcpy(&v, s.data() + p, 8);
    p += 8;
    return v;
  }
  std::string str() {
    const uint32_t n = u32();
    if (!ok || p + n > s.size()) { ok = false; return {}; }
    std::string v = s.substr(p, n);
    p += n;
    return v;
  }
};

}  // namespace

// ------------------------------------------------------------------------------------------------
StoreServer::StoreServer(const std::string& host, int port) {
  listen_fd_ = tcp_listen(host, port, &port_);
  if (::pipe(wake_pipe_) != 0) throw NetError(errno_str("pipe"));
  th_ = std::thread([this] { loop(); });
}

StoreServer::~StoreServer() { stop(); }

void StoreServer::stop() {
  if (stop_.exchange(true)) return;
  char c = 1;
  ssize_t r = ::write(wake_pipe_[1], &c, 1);
  (void)r;
  if (th_.joinable()) th_.join();
  for (auto& c2 : conns_) ::close(c2.fd);
  conns_.clear();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  ::close(wake_pipe_[0]);
  ::close(wake_pipe_[1]);
  listen_fd_ = -1;
}

void StoreServer::reply(int fd, const std::string& payload) {
  std::string m;
  put_u32(m, (uint32_t)payload.size());
  m += payload;
  try {
    send_all(fd, m.data(), m.size(), Clock::now() + std::chrono::seconds(30));
  } catch (...) {
    // the client went away; its connection is reaped by the poll loop
  }
}

bool StoreServer::ready(const Waiter& w) const {
  for (auto& k : w.keys)
    if (!kv_.count(k)) return false;
  return true;
}

void StoreServer::wake_waiters() {
  std::vector<Waiter> keep;
  for (auto& w : waiters_) {
    if (ready(w)) {
      reply(w.fd, w.reply_value ? kv_[w.keys[0]] : std::string(1, '\1'));
    } else {
      keep.push_back(w);
    }
  }
  waiters_.swap(keep);
}

bool StoreServer::handle(Conn& c) {
  while (c.in.size() >= 4) {
    uint32_t len;
    std::memcpy(&len, c.in.data(), 4);
    if (c.in.size() < 4 + (size_t)len) break;
    std::string msg = c.in.substr(4, len);
    c.in.erase(0, 4 + (size_t)len);
    if (msg.empty()) return false;
    const auto cmd = (StoreCmd)(uint8_t)msg[0];
    Reader r{msg, 1};
    switch (cmd) {
      case StoreCmd::SET: {
        std::string k = r.str(), v = r.str();
        if (!r.ok) return false;
        kv_[k] = v;
        reply(c.fd, "");
        wake_waiters();
        break;
      }
      case StoreCmd::GET: {
        std::string k = r.str();
        if (!r.ok) return false;
        auto it = kv_.find(k);
        if (it != kv_.end()) reply(c.fd, it->second);
        else waiters_.push_back(Waiter{c.fd, {k}, true});
        break;
      }
      case StoreCmd::ADD: {
        std::string k = r.str();
        int64_t d = r.i64();
        if (!r.ok) return false;
        int64_t cur = 0;
        auto it = kv_.find(k);
        if (it != kv_.end()) cur = std::stoll(it->second);
        cur += d;
        kv_[k] = std::to_string(cur);
        std::string out;
        put_i64(out, cur);
        reply(c.fd, out);
        wake_waiters();
        break;
      }
      case StoreCmd::CHECK:
      case StoreCmd::WAIT: {
        const uint32_t n = r.u32();
        Waiter w{c.fd, {}, false};
        for (uint32_t i = 0; i < n && r.ok; ++i) w.keys.push_back(r.str());
        if (!r.ok) return false;
        if (cmd == StoreCmd::CHECK) reply(c.fd, std::string(1, ready(w) ? '\1' : '\0'));
        else if (ready(w)) reply(c.fd, std::string(1, '\1'));
        else waiters_.push_back(w);
        break;
      }
      case StoreCmd::DEL: {
        std::string k = r.str();
        if (!r.ok) return false;
        const bool had = kv_.erase(k) > 0;
        reply(c.fd, std::string(1, had ? '\1' : '\0'));
        break;
      }
      case StoreCmd::CAS: {
        std::string k = r.str(), expected = r.str(), desired = r.str();
        if (!r.ok) return false;
        auto it = kv_.find(k);
        if ((it == kv_.end() && expected.empty()) || (it != kv_.end() && it->second == expected)) {
          kv_[k] = desired;
          reply(c.fd, desired);
          wake_waiters();
        } else {
          reply(c.fd, it == kv_.end() ? expected : it->second);
        }
        break;
      }
      case StoreCmd::NUMKEYS: {
        std::string out;
        put_i64(out, (int64_t)kv_.size());
        reply(c.fd, out);
        break;
      }
      case StoreCmd::PING:
        reply(c.fd, "");
        break;
      default:
        return false;
    }
  }
  return true;
}

void StoreServer::loop() {
  std::vector<pollfd> pfds;
  char buf[65536];
  while (!stop_.load()) {
    pfds.clear();
    pfds.push_back({listen_fd_, POLLIN, 0});
    pfds.push_back({wake_pipe_[0], POLLIN, 0});
    for (auto& c : conns_) pfds.push_back({c.fd, POLLIN, 0});
    int r = ::poll(pfds.data(), pfds.size(), 1000);
    if (r < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (stop_.load()) break;
    if (pfds[0].revents & POLLIN) {
      int fd = ::accept(listen_fd_, nullptr, nullptr);
      if (fd >= 0) {
        set_nodelay(fd);
        conns_.push_back(Conn{fd, {}});
      }
    }
    std::vector<int> dead;
    for (size_t i = 2; i < pfds.size(); ++i) {
      if (!(pfds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      auto it = std::find_if(conns_.begin(), conns_.end(), [&](const Conn& c) { return c.fd == pfds[i].fd; });
      if (it == conns_.end()) continue;
      ssize_t k = ::recv(it->fd, buf, sizeof(buf), 0);
      if (k <= 0) {
        dead.push_back(it->fd);
        continue;
      }
      it->in.append(buf, (size_t)k);
      if (!handle(*it)) dead.push_back(it->fd);
    }
    for (int fd : dead) {
      ::close(fd);
      conns_.erase(std::remove_if(conns_.begin(), conns_.end(), [&](const Conn& c) { return c.fd == fd; }),
                   conns_.end());
      waiters_.erase(std::remove_if(waiters_.begin(), waiters_.end(), [&](const Waiter& w) { return w.fd == fd; }),
                     waiters_.end());
    }
  }
}

// ------------------------------------------------------------------------------------------------
StoreClient::StoreClient(const std::string& host, int port, int64_t timeout_ms)
    : host_(host), port_(port), timeout_ms_(timeout_ms) {
  fd_ = tcp_connect(host, port, Clock::now() + std::chrono::milliseconds(timeout_ms));
}

StoreClient::~StoreClient() {
  if (fd_ >= 0) ::close(fd_);
}

std::string StoreClient::local_address() const {
  sockaddr_in a{};
  socklen_t len = sizeof(a);
  if (getsockname(fd_, (sockaddr*)&a, &len) != 0) return "127.0.0.1";
  char s[INET_ADDRSTRLEN];
  inet_ntop(AF_INET, &a.sin_addr, s, sizeof(s));
  return s;
}

std::string StoreClient::roundtrip(const std::string& req, int64_t timeout_ms) {
  std::lock_guard<std::mutex> g(mu_);
  const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? timeout_ms_ : timeout_ms);
  std::string m;
  put_u32(m, (uint32_t)req.size());
  m += req;
  try {
    send_all(fd_, m.data(), m.size(), deadline);
    uint32_t len = 0;
    recv_all(fd_, &len, 4, deadline);
    std::string out(len, '\0');
    if (len) recv_all(fd_, &out[0], len, deadline);
    return out;
  } catch (const TimeoutError&) {
    // a late reply to this request would desynchronise the stream: start a fresh connection
    // (the server drops the parked request together with the old connection)
    ::close(fd_);
    fd_ = tcp_connect(host_, port_, Clock::now() + std::chrono::milliseconds(timeout_ms_));
    throw;
  }
}

void StoreClient::set(const std::string& key, const std::string& value) {
  std::string r(1, (char)StoreCmd::SET);
  put_str(r, key);
  put_str(r, value);
  roundtrip(r, -1);
}

std::string StoreClient::get(const std::string& key) {
  std::string r(1, (char)StoreCmd::GET);
  put_str(r, key);
  try {
    return roundtrip(r, -1);
  } catch (const TimeoutError&) {
    throw TimeoutError("store get('" + key + "') timed out");
  }
}

int64_t StoreClient::add(const std::string& key, int64_t delta) {
  std::string r(1, (char)StoreCmd::ADD);
  put_str(r, key);
  put_i64(r, delta);
  std::string out = roundtrip(r, -1);
  int64_t v = 0;
  std::memcpy(&v, out.data(), std::min<size_t>(8, out.size()));
  return v;
}

bool StoreClient::check(const std::vector<std::string>& keys) {
  std::string r(1, (char)StoreCmd::CHECK);
  put_u32(r, (uint32_t)keys.size());
  for (auto& k : keys) put_str(r, k);
  return roundtrip(r, -1) == std::string(1, '\1');
}

void StoreClient::wait(const std::vector<std::string>& keys, int64_t timeout_ms) {
  std::string r(1, (char)StoreCmd::WAIT);
  put_u32(r, (uint32_t)keys.size());
  for (auto& k : keys) put_str(r, k);
  try {
    roundtrip(r, timeout_ms);
  } catch (const TimeoutError&) {
    throw TimeoutError("store wait timed out");
  }
}

bool StoreClient::del(const std::string& key) {
  std::string r(1, (char)StoreCmd::DEL);
  put_str(r, key);
  return roundtrip(r, -1) == std::string(1, '\1');
}

std::string StoreClient::compare_set(const std::string& key, const std::string& expected, const std::string& desired) {
  std::string r(1, (char)StoreCmd::CAS);
  put_str(r, key);
  put_str(r, expected);
  put_str(r, desired);
  return roundtrip(r, -1);
}

int64_t StoreClient::num_keys() {
  std::string r(1, (char)StoreCmd::NUMKEYS);
  std::string out = roundtrip(r, -1);
  int64_t v = 0;
  std::memcpy(&v, out.data(), std::min<size_t>(8, out.size()));
  return v;
}

}  // namespace pde

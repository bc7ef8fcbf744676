// Small socket utilities shared by the TCP store and the host collectives.
#pragma once
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace pde {

struct NetError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct TimeoutError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

using Clock = std::chrono::steady_clock;

inline int64_t ms_left(Clock::time_point deadline) {
  auto d = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
  return d < 0 ? 0 : d;
}

inline std::string errno_str(const char* what) { return std::string(what) + ": " + std::strerror(errno); }

inline void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

inline void set_bufsizes(int fd, int bytes) {
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &bytes, sizeof(bytes));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &bytes, sizeof(bytes));
}

// Listen on host:port (port 0 = ephemeral). Returns fd; *bound_port receives the real port.
inline int tcp_listen(const std::string& host, int port, int* bound_port, int backlog = 256) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) throw NetError(errno_str("socket"));
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (host.empty() || host == "0.0.0.0") {
    a.sin_addr.s_addr = htonl(INADDR_ANY);
  } else if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    ::close(fd);
    throw NetError("bad listen address " + host);
  }
  if (::bind(fd, (sockaddr*)&a, sizeof(a)) < 0) {
    std::string e = errno_str(("bind " + host + ":" + std::to_string(port)).c_str());
    ::close(fd);
    throw NetError(e);
  }
  if (::listen(fd, backlog) < 0) {
    ::close(fd);
    throw NetError(errno_str("listen"));
  }
  socklen_t len = sizeof(a);
  getsockname(fd, (sockaddr*)&a, &len);
  if (bound_port) *bound_port = ntohs(a.sin_port);
  return fd;
}

inline bool resolve_ipv4(const std::string& host, sockaddr_in* out) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return false;
  *out = *(sockaddr_in*)res->ai_addr;
  freeaddrinfo(res);
  return true;
}

// Connect with retries until the deadline (the peer may not be listening yet).
inline int tcp_connect(const std::string& host, int port, Clock::time_point deadline) {
  sockaddr_in a{};
  if (!resolve_ipv4(host, &a)) throw NetError("cannot resolve " + host);
  a.sin_port = htons((uint16_t)port);
  int delay_ms = 5;
  while (true) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) throw NetError(errno_str("socket"));
    if (::connect(fd, (sockaddr*)&a, sizeof(a)) == 0) {
      set_nodelay(fd);
      return fd;
    }
    ::close(fd);
    if (Clock::now() >= deadline)
      throw TimeoutError("timed out connecting to " + host + ":" + std::to_string(port));
    std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms));
    delay_ms = std::min(delay_ms * 2, 200);
  }
}

// Blocking full send / recv with a deadline (poll-based so a dead peer cannot hang us forever).
inline void send_all(int fd, const void* buf, size_t n, Clock::time_point deadline) {
  const char* p = (const char*)buf;
  while (n) {
    pollfd pf{fd, POLLOUT, 0};
    int r = ::poll(&pf, 1, (int)std::min<int64_t>(ms_left(deadline), 1000));
    if (r < 0 && errno != EINTR) throw NetError(errno_str("poll"));
    if (r <= 0) {
      if (Clock::now() >= deadline) throw TimeoutError("send timed out");
      continue;
    }
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      throw NetError(errno_str("send"));
    }
    p += k;
    n -= (size_t)k;
  }
}

inline void recv_all(int fd, void* buf, size_t n, Clock::time_point deadline) {
  char* p = (char*)buf;
  while (n) {
    pollfd pf{fd, POLLIN, 0};
    int r = ::poll(&pf, 1, (int)std::min<int64_t>(ms_left(deadline), 1000));
    if (r < 0 && errno != EINTR) throw NetError(errno_str("poll"));
    if (r <= 0) {
      if (Clock::now() >= deadline) throw TimeoutError("recv timed out");
      continue;
    }
    ssize_t k = ::recv(fd, p, n, 0);
    if (k == 0) throw NetError("peer closed the connection");
    if (k < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      throw NetError(errno_str("recv"));
    }
    p += k;
    n -= (size_t)k;
  }
}

}  // namespace pde

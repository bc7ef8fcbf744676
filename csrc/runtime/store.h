// TCP key-value rendezvous store (the role c10d's TCPStore plays for init_process_group).
//
// Rank 0 hosts a StoreServer (one poll() thread, all state in memory); every rank talks to it
// through a StoreClient.  Operations: set / get (blocks until the key exists) / add (atomic int64
// counter) / check / wait / delete / compare_set / num_keys.  Every client call has a deadline, so
// a dead peer surfaces as a TimeoutError instead of a hang.
#pragma once
#include <atomic>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "net.h"

namespace pde {

enum class StoreCmd : uint8_t { SET = 1, GET, ADD, CHECK, WAIT, DEL, CAS, NUMKEYS, PING };

class StoreServer {
 public:
  StoreServer(const std::string& host, int port);
  ~StoreServer();
  int port() const { return port_; }
  void stop();

 private:
  struct Conn {
    int fd;
    std::string in;
  };
  struct Waiter {
    int fd;
    std::vector<std::string> keys;
    bool reply_value;  // GET replies the value; WAIT replies a status byte
  };
  void loop();
  bool handle(Conn& c);                   // false: close connection
  void reply(int fd, const std::string& payload);
  void wake_waiters();
  bool ready(const Waiter& w) const;

  int listen_fd_ = -1, port_ = 0;
  int wake_pipe_[2] = {-1, -1};
  std::atomic<bool> stop_{false};
  std::thread th_;
  std::map<std::string, std::string> kv_;
  std::vector<Conn> conns_;
  std::vector<Waiter> waiters_;
};

class StoreClient {
 public:
  StoreClient(const std::string& host, int port, int64_t timeout_ms);
  ~StoreClient();
  void set(const std::string& key, const std::string& value);
  std::string get(const std::string& key);
  int64_t add(const std::string& key, int64_t delta);
  bool check(const std::vector<std::string>& keys);
  void wait(const std::vector<std::string>& keys, int64_t timeout_ms = -1);
  bool del(const std::string& key);
  std::string compare_set(const std::string& key, const std::string& expected, const std::string& desired);
  int64_t num_keys();
  int64_t timeout_ms() const { return timeout_ms_; }
  void set_timeout_ms(int64_t t) { timeout_ms_ = t; }
  // Local IPv4 address of the connection to the store (the interface that reaches rank 0).
  std::string local_address() const;

 private:
  std::string roundtrip(const std::string& req, int64_t timeout_ms);
  std::string host_;
  int port_ = 0;
  int fd_ = -1;
  int64_t timeout_ms_;
  std::mutex mu_;
};

// message helpers
void put_u32(std::string& s, uint32_t v);
void put_i64(std::string& s, int64_t v);
void put_str(std::string& s, const std::string& v);

}  // namespace pde

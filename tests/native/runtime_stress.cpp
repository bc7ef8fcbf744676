// Native stress test of the host-side distributed runtime (csrc/runtime/store.cpp, hostcomm.cpp),
// built WITHOUT Python and WITH sanitizers by tests/test_sanitizers_cpu.py:
//   -fsanitize=address,undefined  (heap / stack misuse, UB in the reduction kernels and framing)
//   -fsanitize=thread             (data races between the store's event loop, the HostComm worker
//                                  threads and the submitting threads)
// W ranks run as threads of one process, each with its own StoreClient and HostComm, exactly as
// W processes would (every byte still goes through TCP sockets).  Exits non-zero on any wrong result.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "hostcomm.h"
#include "store.h"

using namespace pde;

namespace {

std::atomic<int> failures{0};

void check(bool ok, const char* what, int rank) {
  if (!ok) {
    std::fprintf(stderr, "rank %d: FAILED %s\n", rank, what);
    failures.fetch_add(1);
  }
}

void rank_main(int port, int rank, int world, int iters) {
  auto store = std::make_shared<StoreClient>("127.0.0.1", port, 60000);
  // store primitives
  store->set("k/" + std::to_string(rank), std::string(100 + rank, char('a' + rank)));
  int64_t v = store->add("counter", 1);
  check(v >= 1 && v <= world, "store add", rank);
  store->wait({"k/0"}, 30000);
  check(store->get("k/0") == std::string(100, 'a'), "store get", rank);
  HostComm comm(store, "stress", rank, world, 60000);
  for (int it = 0; it < iters; ++it) {
    // all-reduce: small (direct) and large (ring), f32 / i64 / bf16 payloads
    for (int64_t n : {int64_t(7), int64_t(4097), int64_t(300001)}) {
      std::vector<float> f(n);
      for (int64_t i = 0; i < n; ++i) f[i] = float((i % 13) * (rank + 1));
      comm.allreduce(f.data(), n, DType::F32, ROp::SUM);
      bool ok = true;
      const float tri = float(world * (world + 1) / 2);
      for (int64_t i = 0; i < n; ++i) ok &= f[i] == float(i % 13) * tri;
      check(ok, "allreduce f32", rank);
      std::vector<int64_t> q(n, rank);
      comm.allreduce(q.data(), n, DType::I64, ROp::MAX);
      ok = true;
      for (int64_t i = 0; i < n; ++i) ok &= q[i] == world - 1;
      check(ok, "allreduce i64 max", rank);
      std::vector<uint16_t> h(n, 0x3f80);   // bf16 1.0
      comm.allreduce(h.data(), n, DType::BF16, ROp::AVG);
      ok = true;
      for (int64_t i = 0; i < n; ++i) ok &= h[i] == 0x3f80;
      check(ok, "allreduce bf16 avg", rank);
    }
    // broadcast / allgather / reduce_scatter / alltoall
    std::vector<int32_t> b(1000, rank == 1 % world ? 42 : -1);
    comm.broadcast(b.data(), b.size() * 4, 1 % world);
    check(b[0] == 42 && b[999] == 42, "broadcast", rank);
    std::vector<int32_t> mine(64, rank), all(64 * world);
    comm.allgather(mine.data(), all.data(), 64 * 4);
    bool ok = true;
    for (int r = 0; r < world; ++r) ok &= all[r * 64] == r && all[r * 64 + 63] == r;
    check(ok, "allgather", rank);
    std::vector<float> rs_in(16 * world), rs_out(16);
    for (int c = 0; c < world; ++c)
      for (int i = 0; i < 16; ++i) rs_in[c * 16 + i] = float(c);
    comm.reduce_scatter(rs_in.data(), rs_out.data(), 16, DType::F32, ROp::SUM);
    check(rs_out[0] == float(rank * world) && rs_out[15] == float(rank * world), "reduce_scatter", rank);
    std::vector<int32_t> a2a_in(world * 8), a2a_out(world * 8);
    for (int d = 0; d < world; ++d)
      for (int i = 0; i < 8; ++i) a2a_in[d * 8 + i] = 100 * rank + d;
    comm.alltoall(a2a_in.data(), a2a_out.data(), 8 * 4);
    ok = true;
    for (int s = 0; s < world; ++s) ok &= a2a_out[s * 8] == 100 * s + rank;
    check(ok, "alltoall", rank);
    // async submissions racing with a synchronous barrier from this thread
    std::vector<double> d(5000, 1.0);
    auto w = comm.submit([&] { comm.allreduce(d.data(), d.size(), DType::F64, ROp::SUM); });
    w->wait();
    check(d[0] == double(world) && d[4999] == double(world), "async allreduce", rank);
    comm.barrier();
  }
  comm.shutdown();
}

}  // namespace

int main(int argc, char** argv) {
  const int world = argc > 1 ? std::atoi(argv[1]) : 4;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 3;
  StoreServer server("127.0.0.1", 0);
  std::vector<std::thread> ths;
  for (int r = 0; r < world; ++r) ths.emplace_back(rank_main, server.port(), r, world, iters);
  for (auto& t : ths) t.join();
  server.stop();
  if (failures.load()) {
    std::fprintf(stderr, "%d failures\n", failures.load());
    return 1;
  }
  std::printf("runtime stress ok: world=%d iters=%d\n", world, iters);
  return 0;
}

// pybind11 module `_runtime`: the framework's native distributed runtime.
// Buffers cross the boundary as integer addresses (tensor.data_ptr()); the Python layer keeps the
// tensors alive until the returned Work completes.  Blocking calls release the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "hostcomm.h"
#include "peer_allreduce.h"
#include "rccl_comm.h"
#include "store.h"

namespace py = pybind11;
using namespace pde;

namespace {

template <typename F>
std::shared_ptr<Work> run(HostComm& c, bool async, F&& fn) {
  auto w = c.submit(std::forward<F>(fn));
  if (!async) {
    py::gil_scoped_release nogil;
    w->wait();
  }
  return w;
}

void* ptr(uintptr_t p) { return reinterpret_cast<void*>(p); }

}  // namespace

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "Native distributed runtime of pytorch_distributed_example_amd (TCP store, host TCP collectives, RCCL)";

  py::register_exception<TimeoutError>(m, "TimeoutError", PyExc_TimeoutError);
  py::register_exception<NetError>(m, "NetError", PyExc_ConnectionError);

  py::class_<StoreServer, std::shared_ptr<StoreServer>>(m, "StoreServer")
      .def(py::init<const std::string&, int>(), py::arg("host") = "0.0.0.0", py::arg("port") = 0)
      .def_property_readonly("port", &StoreServer::port)
      .def("stop", &StoreServer::stop, py::call_guard<py::gil_scoped_release>());

  py::class_<StoreClient, std::shared_ptr<StoreClient>>(m, "StoreClient")
      .def(py::init<const std::string&, int, int64_t>(), py::arg("host"), py::arg("port"),
           py::arg("timeout_ms") = 300000, py::call_guard<py::gil_scoped_release>())
      .def("set",
           [](StoreClient& s, const std::string& k, py::bytes v) {
             std::string val = v;
             py::gil_scoped_release nogil;
             s.set(k, val);
           })
      .def("get",
           [](StoreClient& s, const std::string& k) {
             std::string v;
             {
               py::gil_scoped_release nogil;
               v = s.get(k);
             }
             return py::bytes(v);
           })
      .def("add", &StoreClient::add, py::call_guard<py::gil_scoped_release>())
      .def("check", &StoreClient::check, py::call_guard<py::gil_scoped_release>())
      .def("wait", &StoreClient::wait, py::arg("keys"), py::arg("timeout_ms") = -1,
           py::call_guard<py::gil_scoped_release>())
      .def("delete_key", &StoreClient::del, py::call_guard<py::gil_scoped_release>())
      .def("compare_set",
           [](StoreClient& s, const std::string& k, py::bytes e, py::bytes d) {
             std::string ee = e, dd = d, out;
             {
               py::gil_scoped_release nogil;
               out = s.compare_set(k, ee, dd);
             }
             return py::bytes(out);
           })
      .def("num_keys", &StoreClient::num_keys, py::call_guard<py::gil_scoped_release>())
      .def_property("timeout_ms", &StoreClient::timeout_ms, &StoreClient::set_timeout_ms)
      .def("local_address", &StoreClient::local_address);

  py::class_<Work, std::shared_ptr<Work>>(m, "Work")
      .def("wait", &Work::wait, py::call_guard<py::gil_scoped_release>())
      .def("is_completed", &Work::is_completed);

  py::class_<HostComm, std::shared_ptr<HostComm>>(m, "HostComm")
      .def(py::init<std::shared_ptr<StoreClient>, const std::string&, int, int, int64_t>(), py::arg("store"),
           py::arg("prefix"), py::arg("rank"), py::arg("world"), py::arg("timeout_ms") = 300000,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &HostComm::rank)
      .def_property_readonly("world", &HostComm::world)
      .def("allreduce",
           [](HostComm& c, uintptr_t buf, int64_t n, int dt, int op, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->allreduce(ptr(buf), n, (DType)dt, (ROp)op); });
           },
           py::arg("buf"), py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("async_op") = false)
      .def("broadcast",
           [](HostComm& c, uintptr_t buf, int64_t bytes, int root, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->broadcast(ptr(buf), bytes, root); });
           },
           py::arg("buf"), py::arg("bytes"), py::arg("root"), py::arg("async_op") = false)
      .def("allgather",
           [](HostComm& c, uintptr_t in, uintptr_t out, int64_t bytes, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->allgather(ptr(in), ptr(out), bytes); });
           },
           py::arg("inp"), py::arg("out"), py::arg("bytes"), py::arg("async_op") = false)
      .def("reduce_scatter",
           [](HostComm& c, uintptr_t in, uintptr_t out, int64_t n, int dt, int op, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->reduce_scatter(ptr(in), ptr(out), n, (DType)dt, (ROp)op); });
           },
           py::arg("inp"), py::arg("out"), py::arg("count_per_rank"), py::arg("dtype"), py::arg("op"),
           py::arg("async_op") = false)
      .def("reduce",
           [](HostComm& c, uintptr_t buf, int64_t n, int dt, int op, int root, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->reduce(ptr(buf), n, (DType)dt, (ROp)op, root); });
           },
           py::arg("buf"), py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("root"),
           py::arg("async_op") = false)
      .def("gather",
           [](HostComm& c, uintptr_t in, uintptr_t out, int64_t bytes, int root, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->gather(ptr(in), ptr(out), bytes, root); });
           },
           py::arg("inp"), py::arg("out"), py::arg("bytes"), py::arg("root"), py::arg("async_op") = false)
      .def("scatter",
           [](HostComm& c, uintptr_t in, uintptr_t out, int64_t bytes, int root, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->scatter(ptr(in), ptr(out), bytes, root); });
           },
           py::arg("inp"), py::arg("out"), py::arg("bytes"), py::arg("root"), py::arg("async_op") = false)
      .def("alltoall",
           [](HostComm& c, uintptr_t in, uintptr_t out, int64_t bytes, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->alltoall(ptr(in), ptr(out), bytes); });
           },
           py::arg("inp"), py::arg("out"), py::arg("bytes_per_rank"), py::arg("async_op") = false)
      .def("p2p",
           [](HostComm& c, std::vector<std::tuple<int, uintptr_t, int64_t>> sends,
              std::vector<std::tuple<int, uintptr_t, int64_t>> recvs, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->p2p(sends, recvs); });
           },
           py::arg("sends"), py::arg("recvs"), py::arg("async_op") = false)
      .def("send",
           [](HostComm& c, uintptr_t buf, int64_t bytes, int dst, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->send(ptr(buf), bytes, dst); });
           },
           py::arg("buf"), py::arg("bytes"), py::arg("dst"), py::arg("async_op") = false)
      .def("recv",
           [](HostComm& c, uintptr_t buf, int64_t bytes, int src, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->recv(ptr(buf), bytes, src); });
           },
           py::arg("buf"), py::arg("bytes"), py::arg("src"), py::arg("async_op") = false)
      .def("barrier",
           [](HostComm& c, bool async) {
             HostComm* cp = &c;
             return run(c, async, [=] { cp->barrier(); });
           },
           py::arg("async_op") = false)
      .def("shutdown", &HostComm::shutdown, py::call_guard<py::gil_scoped_release>());

  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int rank, int world, int device) {
             std::string u = uid;
             py::gil_scoped_release nogil;
             return std::make_shared<RcclComm>(u, rank, world, device);
           }),
           py::arg("unique_id"), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def_static("make_unique_id", [] { return py::bytes(RcclComm::make_unique_id()); })
      .def_static("version", &RcclComm::version)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("device", &RcclComm::device)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
           py::arg("op"), py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
           py::arg("root"), py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def("reduce", &RcclComm::reduce, py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &RcclComm::all_gather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("all_to_all", &RcclComm::all_to_all, py::call_guard<py::gil_scoped_release>())
      .def("send", &RcclComm::send, py::call_guard<py::gil_scoped_release>())
      .def("recv", &RcclComm::recv, py::call_guard<py::gil_scoped_release>())
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end, py::call_guard<py::gil_scoped_release>())
      .def("split", &RcclComm::split, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &RcclComm::destroy, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &RcclComm::async_error)
      .def("comm_count", &RcclComm::comm_count)
      .def("cu_device", &RcclComm::cu_device);
  py::class_<CommWatchdog, std::shared_ptr<CommWatchdog>>(m, "CommWatchdog")
      .def(py::init<std::shared_ptr<RcclComm>, int64_t, int>(), py::arg("comm"), py::arg("timeout_ms"),
           py::arg("poll_ms") = 20)
      .def("watch", &CommWatchdog::watch, py::arg("stream"), py::arg("what") = "collective")
      .def("error", &CommWatchdog::error)
      .def("pending", &CommWatchdog::pending)
      .def("stop", &CommWatchdog::stop, py::call_guard<py::gil_scoped_release>());
  py::class_<PeerAllReduce, std::shared_ptr<PeerAllReduce>>(m, "PeerAllReduce")
      .def(py::init<int, int, int, int64_t, bool>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("capacity_bytes"), py::arg("uncached_data") = false, py::call_guard<py::gil_scoped_release>())
      .def("handle", [](PeerAllReduce& p) { return py::bytes(p.handle()); })
      .def("open",
           [](PeerAllReduce& p, const std::vector<py::bytes>& hs) {
             std::vector<std::string> v;
             for (auto& h : hs) v.emplace_back(std::string(h));
             py::gil_scoped_release nogil;
             p.open(v);
           })
      .def("all_reduce_f32", &PeerAllReduce::all_reduce_f32, py::arg("inp"), py::arg("out"), py::arg("count"),
           py::arg("scale"), py::arg("algo"), py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def("all_reduce_bf16", &PeerAllReduce::all_reduce_bf16, py::arg("inp"), py::arg("out"), py::arg("count"),
           py::arg("scale"), py::arg("algo"), py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("capacity_bytes", &PeerAllReduce::capacity_bytes)
      .def_property_readonly("rank", &PeerAllReduce::rank)
      .def_property_readonly("world", &PeerAllReduce::world)
      .def_property_readonly("device", &PeerAllReduce::device)
      .def_property_readonly("is_open", &PeerAllReduce::is_open)
      .def("device_args", [](PeerAllReduce& p) { return py::bytes(p.device_args()); })
      .def("device_probe_f32", &PeerAllReduce::device_probe_f32, py::arg("inp"), py::arg("out"), py::arg("count"),
           py::arg("scale"), py::arg("two"), py::arg("stream"))
      .def("register_buffer",
           [](PeerAllReduce& p, uintptr_t ptr, int64_t bytes) {
             int id = -1;
             std::string h = p.register_buffer(ptr, bytes, &id);
             return py::make_tuple(id, py::bytes(h));
           })
      .def("open_registered",
           [](PeerAllReduce& p, int id, const std::vector<py::bytes>& hs) {
             std::vector<std::string> v;
             for (auto& h : hs) v.emplace_back(std::string(h));
             py::gil_scoped_release nogil;
             p.open_registered(id, v);
           })
      .def("all_reduce_registered_f32", &PeerAllReduce::all_reduce_registered_f32, py::arg("id"), py::arg("off"),
           py::arg("count"), py::arg("scale"), py::arg("algo"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("all_reduce_registered", &PeerAllReduce::all_reduce_registered, py::arg("id"), py::arg("off"),
           py::arg("count"), py::arg("esz"), py::arg("scale"), py::arg("algo"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("registered_bytes", &PeerAllReduce::registered_bytes)
      .def("registered_device_args",
           [](PeerAllReduce& p, int id) { return py::bytes(p.registered_device_args(id)); })
      .def("debug_skip_stage", &PeerAllReduce::debug_skip_stage)
      .def("error", &PeerAllReduce::error, py::call_guard<py::gil_scoped_release>())
      .def("error_async", &PeerAllReduce::error_async)
      .def("reset_error", &PeerAllReduce::reset_error)
      .def("set_timeout_ms", &PeerAllReduce::set_timeout_ms)
      .def("set_one_shot_max_bytes", &PeerAllReduce::set_one_shot_max_bytes)
      .def("set_max_blocks", &PeerAllReduce::set_max_blocks)
      .def("set_ip_block_cap", &PeerAllReduce::set_ip_block_cap)
      .def("close", &PeerAllReduce::close, py::call_guard<py::gil_scoped_release>());
}

// pybind11 module ``paddle2_amd._runtime``: host-only native runtime (no HIP dependency, so it
// loads on CPU-only machines and inside data-loader workers).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <condition_variable>
#include <deque>

#include "runtime.h"

namespace py = pybind11;

namespace pdrt {

// Bounded blocking queue of Python objects (reference: LoDTensorBlockingQueue,
// paddle/fluid/operators/reader/lod_tensor_blocking_queue.h): the producer thread of the data
// loader pushes ready batches, the training loop pops; both wait with the GIL released.
class BlockingQueue {
 public:
  explicit BlockingQueue(size_t cap) : cap_(cap ? cap : 1) {}

  bool push(py::object obj, double timeout_s) {
    {
      py::gil_scoped_release rel;
      std::unique_lock<std::mutex> lk(mu_);
      auto pred = [&] { return closed_ || q_.size() < cap_; };
      if (timeout_s < 0) not_full_.wait(lk, pred);
      else if (!not_full_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred)) return false;
      if (closed_) return false;
      q_.push_back(std::move(obj));
    }
    not_empty_.notify_one();
    return true;
  }

  py::object pop(double timeout_s) {
    py::object out;
    bool got = false;
    {
      py::gil_scoped_release rel;
      std::unique_lock<std::mutex> lk(mu_);
      auto pred = [&] { return closed_ || !q_.empty(); };
      bool ok = true;
      if (timeout_s < 0) not_empty_.wait(lk, pred);
      else ok = not_empty_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred);
      if (ok && !q_.empty()) {
        out = std::move(q_.front());
        q_.pop_front();
        got = true;
      }
    }
    if (!got) return py::none();
    not_full_.notify_one();
    return out;
  }

  void close() {
    {
      std::lock_guard<std::mutex> g(mu_);
      closed_ = true;
    }
    not_full_.notify_all();
    not_empty_.notify_all();
  }

  void reopen() {
    std::lock_guard<std::mutex> g(mu_);
    closed_ = false;
  }

  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return q_.size();
  }

  bool closed() {
    std::lock_guard<std::mutex> g(mu_);
    return closed_;
  }

  size_t capacity() const { return cap_; }

 private:
  size_t cap_;
  std::deque<py::object> q_;
  bool closed_ = false;
  std::mutex mu_;
  std::condition_variable not_full_, not_empty_;
};

}  // namespace pdrt

PYBIND11_MODULE(_runtime, m) {
  using namespace pdrt;
  m.doc() = "paddle2_amd host runtime: TCPStore, comm watchdog, host tracer, blocking queue";

  py::class_<TCPStoreServer>(m, "TCPStoreServer")
      .def(py::init<const std::string&, int>(), py::arg("host"), py::arg("port"))
      .def_property_readonly("port", &TCPStoreServer::port)
      .def("shutdown", &TCPStoreServer::shutdown, py::call_guard<py::gil_scoped_release>());

  py::class_<TCPStoreClient>(m, "TCPStoreClient")
      .def(py::init<const std::string&, int, double>(), py::arg("host"), py::arg("port"), py::arg("timeout"),
           py::call_guard<py::gil_scoped_release>())
      .def("set", [](TCPStoreClient& c, const std::string& k, py::bytes v) {
             std::string s = v;
             py::gil_scoped_release rel;
             c.set(k, s);
           })
      .def("get", [](TCPStoreClient& c, const std::string& k) {
             std::string s;
             {
               py::gil_scoped_release rel;
               s = c.get(k);
             }
             return py::bytes(s);
           })
      .def("add", &TCPStoreClient::add, py::call_guard<py::gil_scoped_release>())
      .def("check", &TCPStoreClient::check, py::call_guard<py::gil_scoped_release>())
      .def("wait", &TCPStoreClient::wait, py::call_guard<py::gil_scoped_release>())
      .def("delete_key", &TCPStoreClient::remove, py::call_guard<py::gil_scoped_release>())
      .def("num_keys", &TCPStoreClient::num_keys, py::call_guard<py::gil_scoped_release>())
      .def("compare_set", [](TCPStoreClient& c, const std::string& k, py::bytes e, py::bytes d) {
             std::string es = e, ds = d, out;
             {
               py::gil_scoped_release rel;
               out = c.compare_set(k, es, ds);
             }
             return py::bytes(out);
           })
      .def("append", [](TCPStoreClient& c, const std::string& k, py::bytes v) {
             std::string s = v;
             py::gil_scoped_release rel;
             return c.append(k, s);
           })
      .def("set_timeout", &TCPStoreClient::set_timeout)
      .def_property_readonly("timeout", &TCPStoreClient::timeout);

  m.def("tracer_enable", &tracer_enable);
  m.def("tracer_enabled", &tracer_enabled);
  m.def("tracer_push", &tracer_push, py::arg("name"), py::arg("type") = 0);
  m.def("tracer_pop", &tracer_pop);
  m.def("tracer_instant", &tracer_instant);
  m.def("tracer_now_ns", &tracer_now_ns);
  m.def("tracer_clear", &tracer_clear);
  m.def("tracer_chrome_json", &tracer_chrome_json, py::arg("pid") = 0);
  m.def("tracer_events", [] {
    py::list out;
    for (auto& e : tracer_events())
      out.append(py::make_tuple(tracer_name(e.name_id), e.type, e.tid, e.start_ns, e.end_ns));
    return out;
  });

  m.def("watchdog_start", &watchdog_start, py::arg("poll_s") = 1.0, py::arg("abort_on_timeout") = false);
  m.def("watchdog_stop", &watchdog_stop, py::call_guard<py::gil_scoped_release>());
  m.def("watchdog_begin", &watchdog_begin, py::arg("desc"), py::arg("timeout_s"), py::arg("hip_event") = 0);
  m.def("watchdog_take_finished", &watchdog_take_finished);
  m.def("watchdog_end", &watchdog_end);
  m.def("watchdog_timed_out", &watchdog_timed_out);
  m.def("watchdog_inflight", &watchdog_inflight);

  py::class_<FleetTask>(m, "FleetTask")
      .def(py::init<>())
      .def_readwrite("id", &FleetTask::id)
      .def_readwrite("rank", &FleetTask::rank)
      .def_readwrite("role", &FleetTask::role)
      .def_readwrite("max_run_times", &FleetTask::max_run_times)
      .def_readwrite("run_per_steps", &FleetTask::run_per_steps)
      .def_readwrite("run_at_offset", &FleetTask::run_at_offset)
      .def_readwrite("upstream", &FleetTask::upstream)
      .def_readwrite("downstream", &FleetTask::downstream);

  py::class_<FleetCarrier>(m, "FleetCarrier")
      .def(py::init<int, int>(), py::arg("rank"), py::arg("num_threads") = 2)
      .def("add_task", &FleetCarrier::add_task)
      .def("add_remote_task", &FleetCarrier::add_remote_task)
      .def("set_compute",
           [](FleetCarrier& c, py::function fn) {
             // the callback runs on a loop thread: take the GIL, surface Python errors as C++ exceptions
             auto holder = std::make_shared<py::function>(std::move(fn));
             c.set_compute([holder](int64_t task, int64_t step) {
               py::gil_scoped_acquire g;
               try {
                 (*holder)(task, step);
               } catch (py::error_already_set& e) {
                 throw std::runtime_error(e.what());
               }
             });
           })
      .def("listen", &FleetCarrier::listen, py::arg("host") = "127.0.0.1")
      .def("set_peer", &FleetCarrier::set_peer)
      .def("start", &FleetCarrier::start)
      .def("wait", &FleetCarrier::wait, py::arg("timeout_s") = -1.0, py::call_guard<py::gil_scoped_release>())
      .def("trace", &FleetCarrier::trace)
      .def("clear_trace", &FleetCarrier::clear_trace)
      .def("shutdown", &FleetCarrier::shutdown, py::call_guard<py::gil_scoped_release>());

  py::class_<InterpPlan>(m, "InterpPlan")
      .def_readonly("n", &InterpPlan::n)
      .def_readonly("num_edges_raw", &InterpPlan::num_edges_raw)
      .def_readonly("downstream", &InterpPlan::downstream)
      .def_readonly("dep_count", &InterpPlan::dep_count)
      .def_readonly("order", &InterpPlan::order)
      .def_readonly("waits", &InterpPlan::waits)
      .def_property_readonly("record", [](const InterpPlan& p) { return std::vector<int>(p.record.begin(), p.record.end()); })
      .def_readonly("free_after", &InterpPlan::free_after)
      .def_readonly("reader_count", &InterpPlan::reader_count);
  m.def("build_interp_plan", &build_interp_plan, py::arg("reads"), py::arg("writes"), py::arg("stream"),
        py::arg("barrier"), py::arg("keep"));
  py::class_<ReadyQueue>(m, "ReadyQueue")
      .def(py::init<const InterpPlan&>())
      .def("start", &ReadyQueue::start)
      .def("pop", &ReadyQueue::pop, py::arg("timeout_s") = -1.0, py::call_guard<py::gil_scoped_release>())
      .def("done", &ReadyQueue::done)
      .def("fail", &ReadyQueue::fail)
      .def("finished", &ReadyQueue::finished);
  py::class_<BlockingQueue>(m, "BlockingQueue")
      .def(py::init<size_t>(), py::arg("capacity"))
      .def("push", &BlockingQueue::push, py::arg("obj"), py::arg("timeout") = -1.0)
      .def("pop", &BlockingQueue::pop, py::arg("timeout") = -1.0)
      .def("close", &BlockingQueue::close)
      .def("reopen", &BlockingQueue::reopen)
      .def("size", &BlockingQueue::size)
      .def("closed", &BlockingQueue::closed)
      .def_property_readonly("capacity", &BlockingQueue::capacity);
}

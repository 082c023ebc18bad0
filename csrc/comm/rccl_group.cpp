// ProcessGroupRCCL core: RCCL communicators, comm streams, event fences and tasks (pybind module
// paddle2_amd._rccl; the torch-facing process group is paddle2_amd/distributed/rccl_pg.py).
//
// Reference roles: paddle/fluid/distributed/collective/process_group_nccl.cc — per-device comm stream with
// calc->comm / comm->calc event sync (:840-847), the generic Collective path (:902), dedicated lo->hi p2p
// communicators (:1023-1028), group start/end coalescing (:999-1037); paddle/phi/core/distributed/
// nccl_comm_context.cc:79-248 (native ncclAvg / PreMulSum); comm_context_manager.cc:61-122 (rank 0 creates the
// unique id, publishes it through the TCPStore, every rank ncclCommInitRank's).
//
// MI355X design:
//  * one high-priority HIP stream per communicator: collectives overlap the compute stream, and p2p on its
//    own lo->hi communicator + stream never queues behind a large reduce-scatter of the data-parallel group
//    (xGMI links are point-to-point; independent streams keep several links busy at once);
//  * every operation: record an event on the caller's (calc) stream, make the comm stream wait on it, enqueue
//    the RCCL call, record the end event on the comm stream -> Task.  Task.wait(stream) makes the caller's
//    stream wait on the end event (no host block); Task.synchronize() blocks the host with async-error polling
//    and a timeout that aborts the communicator instead of hanging; use_calc_stream enqueues straight on the
//    caller's stream (no events);
//  * coalescing: group_start() opens ncclGroupStart; operations inside fence each communicator they touch once
//    and return no task; group_end() closes the group and returns ONE task over every touched communicator;
//  * AVG is ncclAvg and PreMulSum a ncclRedOpCreatePreMulSum op (host scalar), destroyed right after enqueue;
//  * events come from a per-group pool; communicators are created lazily through the caller's store object
//    (anything with set(key, bytes) / get(key) -> bytes: the native TCPStore or a c10d store).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "rccl_core.h"

namespace py = pybind11;
using pdrccl::RcclGroup;
using pdrccl::Task;

namespace {
// A Python store (the native TCPStore or a c10d store: set(key, bytes) / get(key) -> bytes) behind the core's Store
// interface.  Every RcclGroup method runs with the GIL released (a communicator's creation blocks in the store and
// in ncclCommInitRank, which may need this process's store server thread); the store calls take it back.
class PyStore : public pdrccl::Store {
 public:
  explicit PyStore(py::object s) : s_(std::move(s)) {}
  ~PyStore() override {
    py::gil_scoped_acquire g;
    s_ = py::object();
  }
  void set(const std::string& key, const std::string& value) override {
    py::gil_scoped_acquire g;
    s_.attr("set")(key, py::bytes(value));
  }
  std::string get(const std::string& key) override {
    py::gil_scoped_acquire g;
    py::bytes b = s_.attr("get")(key);
    return std::string(b);
  }

 private:
  py::object s_;
};
}  // namespace

PYBIND11_MODULE(_rccl, m) {
  m.doc() = "RCCL process-group core (communicators, comm streams, event fences, tasks)";
  m.def("version", [] {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<Task, std::shared_ptr<Task>>(m, "Task")
      .def("wait", &Task::wait, py::arg("stream"))
      .def("is_completed", &Task::is_completed)
      .def("synchronize", &Task::synchronize, py::call_guard<py::gil_scoped_release>());
  py::class_<RcclGroup>(m, "RcclGroup")
      .def(py::init([](py::object store, std::string prefix, int rank, int nranks, int device, int timeout_ms) {
             return std::make_unique<RcclGroup>(std::make_shared<PyStore>(std::move(store)), std::move(prefix), rank,
                                                nranks, device, timeout_ms);
           }),
           py::arg("store"), py::arg("prefix"), py::arg("rank"), py::arg("nranks"), py::arg("device"),
           py::arg("timeout_ms"))
      .def_property_readonly("rank", &RcclGroup::rank)
      .def_property_readonly("size", &RcclGroup::size)
      .def_property("timeout_ms", &RcclGroup::timeout_ms, &RcclGroup::set_timeout_ms)
      .def("comm_stream", &RcclGroup::comm_stream, py::call_guard<py::gil_scoped_release>())
      .def("p2p_stream", &RcclGroup::p2p_stream, py::call_guard<py::gil_scoped_release>())
      .def("num_comms", &RcclGroup::num_comms)
      .def("all_reduce", &RcclGroup::all_reduce, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclGroup::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("reduce", &RcclGroup::reduce, py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &RcclGroup::all_gather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclGroup::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("all_to_all", &RcclGroup::all_to_all, py::call_guard<py::gil_scoped_release>())
      .def("all_to_all_v", &RcclGroup::all_to_all_v, py::call_guard<py::gil_scoped_release>())
      .def("send", &RcclGroup::send, py::call_guard<py::gil_scoped_release>())
      .def("recv", &RcclGroup::recv, py::call_guard<py::gil_scoped_release>())
      .def("group_start", &RcclGroup::group_start, py::call_guard<py::gil_scoped_release>())
      .def("group_end", &RcclGroup::group_end, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &RcclGroup::barrier, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclGroup::abort, py::call_guard<py::gil_scoped_release>())
      .def("shutdown", &RcclGroup::shutdown, py::call_guard<py::gil_scoped_release>());
}

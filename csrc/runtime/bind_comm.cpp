// Python bindings of the membership-fence communicators (see bind_comm.hpp).
// Every call that can block (library init, connect, collectives, shrink,
// finalize) releases the GIL: the first RCCL call initialises the library
// (seconds) and must not stall the worker's serving thread.
#include "bind_comm.hpp"

#include <pybind11/stl.h>

#include <chrono>

#include "fence.hpp"
#include "shmcomm.hpp"

namespace py = pybind11;

namespace kiosk {

void bind_comm(py::module_& m) {
  py::register_exception<FenceInterrupted>(m, "FenceInterrupted",
                                           PyExc_RuntimeError);
  m.def("rccl_library", &rccl_library, py::call_guard<py::gil_scoped_release>());
  m.def("rccl_version", &rccl_version, py::call_guard<py::gil_scoped_release>());
  m.def("fence_use_library", &rccl_use_library, py::arg("path"),
        py::call_guard<py::gil_scoped_release>());
  m.def("rccl_loaded_libraries", &rccl_loaded_libraries,
        py::call_guard<py::gil_scoped_release>());
  m.def("fence_can_shrink", &rccl_can_shrink,
        py::call_guard<py::gil_scoped_release>());
  m.def("fence_warmup", &rccl_warmup, py::arg("timeout") = 60.0,
        py::call_guard<py::gil_scoped_release>());
  m.def("fence_preload", &rccl_preload,
        py::call_guard<py::gil_scoped_release>());
  m.def("fence_dlopen", &rccl_dlopen,
        py::call_guard<py::gil_scoped_release>());
  m.def("fence_unique_id", [] {
    std::string id;
    {
      py::gil_scoped_release release;
      id = rccl_unique_id();
    }
    return py::bytes(id);
  });

  py::class_<Fence>(m, "Fence")
      .def(py::init([](py::bytes uid, int nranks, int rank, double timeout) {
             std::string id = uid;
             py::gil_scoped_release release;
             return new Fence(id, nranks, rank, timeout);
           }),
           py::arg("unique_id"), py::arg("nranks"), py::arg("rank"),
           py::arg("timeout") = 60.0)
      .def(py::init<int, int, double>(), py::arg("nranks"), py::arg("rank"),
           py::arg("timeout") = 60.0)
      .def(
          "connect",
          [](Fence& f, py::bytes uid) {
            std::string id = uid;
            py::gil_scoped_release release;
            f.connect(id);
          },
          py::arg("unique_id"))
      .def("allreduce", &Fence::allreduce,
           py::call_guard<py::gil_scoped_release>())
      .def(
          "shrink",
          [](Fence& f, const std::vector<int>& excluded, double timeout,
             bool abort_parent) -> Fence& {
            py::gil_scoped_release release;
            f.shrink(excluded, timeout, abort_parent);
            return f;
          },
          py::arg("excluded"), py::arg("timeout") = 60.0,
          py::arg("abort_parent") = true, py::return_value_policy::reference)
      .def("destroy", &Fence::destroy, py::call_guard<py::gil_scoped_release>())
      .def("abort", &Fence::abort, py::call_guard<py::gil_scoped_release>())
      .def("request_abort", &Fence::request_abort)
      .def("request_interrupt", &Fence::request_interrupt)
      .def_property_readonly("abort_requested", &Fence::abort_requested)
      .def_property_readonly("nranks", &Fence::nranks)
      .def_property_readonly("rank", &Fence::rank)
      .def("set_timeout", &Fence::set_timeout, py::arg("timeout"))
      .def_property_readonly("timeout", &Fence::timeout);

  m.def("shm_unique_id", &shm_unique_id, py::arg("dir") = "");
  py::class_<ShmComm>(m, "ShmComm")
      .def(py::init<const std::string&, int, int, double, bool>(),
           py::arg("unique_id"), py::arg("nranks"), py::arg("rank"),
           py::arg("timeout") = 30.0, py::arg("detect_dead_peers") = true)
      .def("poll_ready", &ShmComm::poll_ready)
      .def("wait_ready", &ShmComm::wait_ready,
           py::call_guard<py::gil_scoped_release>())
      .def(
          "allreduce",
          [](ShmComm& c, const std::vector<long long>& values) {
            std::vector<long long> out;
            double us = 0.0;
            {
              py::gil_scoped_release release;
              const auto t0 = std::chrono::steady_clock::now();
              out = c.allreduce(values);
              us = std::chrono::duration<double, std::micro>(
                       std::chrono::steady_clock::now() - t0)
                       .count();
            }
            return py::make_tuple(out, us);
          },
          py::arg("values"))
      .def(
          "shrink",
          [](ShmComm& c, const std::vector<int>& excluded) {
            return c.shrink(excluded);
          },
          py::arg("excluded"))
      .def("request_abort", &ShmComm::request_abort)
      .def_property_readonly("abort_requested", &ShmComm::abort_requested)
      .def("close", &ShmComm::close)
      .def_property_readonly("nranks", &ShmComm::nranks)
      .def_property_readonly("rank", &ShmComm::rank)
      .def_property_readonly("unique_id", &ShmComm::id);
}

}  // namespace kiosk

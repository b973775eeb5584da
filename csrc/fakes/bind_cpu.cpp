// `_kiosk_fence_cpu`: the node-communicator bindings of `_kiosk_hip`
// (bind_comm.cpp) built for a CPU host against the shared-memory fake HIP +
// RCCL (fake_hip_rccl.cpp), so the production Fence / RcclNodeTransport /
// node agent run unchanged in N CPU processes (tests/test_node_fence.py,
// FENCE=rccl with KIOSK_NATIVE=fake).  Never loaded on a GPU box.
#include <pybind11/pybind11.h>

namespace py = pybind11;

#include <stdexcept>

#include "runtime/bind_comm.hpp"
#include "runtime/fence.hpp"

extern "C" void fake_hip_launch_kernel();
extern "C" void fake_hip_graph_launch();

namespace kiosk {
// engine.cpp's helper (the fence needs it for its HIP calls)
void check_hip(hipError_t err, const char* what) {
  if (err != hipSuccess) throw std::runtime_error(what);
}
}  // namespace kiosk

PYBIND11_MODULE(_kiosk_fence_cpu, m) {
  m.doc() = "kiosk node-communicator bindings over the CPU fake HIP + RCCL";
  m.attr("arch") = "cpu-fake";
  kiosk::bind_comm(m);
  // the modelled HIP launch paths (fake_hip_rccl.cpp): the CPU mock engine
  // launches through them, so RCCL's runtime-lock holds reach it
  m.def("fake_launch_kernel", &fake_hip_launch_kernel,
        py::call_guard<py::gil_scoped_release>());
  m.def("fake_graph_launch", &fake_hip_graph_launch,
        py::call_guard<py::gil_scoped_release>());
}

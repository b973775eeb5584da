// Bindings of the node-communicator objects (RCCL Fence, ShmComm), shared by
// the gfx950 module `_kiosk_hip` and the CPU test module `_kiosk_fence_cpu`
// (csrc/fakes/bind_cpu.cpp, linked against the fake HIP + RCCL).
#pragma once

#include <pybind11/pybind11.h>

namespace kiosk {
void bind_comm(pybind11::module_& m);
}  // namespace kiosk

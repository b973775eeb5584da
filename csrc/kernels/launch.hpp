// Kernel launches that never wait on the HIP runtime's fat-binary registry.
//
// hipLaunchKernel(GGL) and hipFuncSetAttribute look a kernel's host stub up
// in the runtime's fat-binary registry under one process-wide lock.  RCCL
// holds that lock for ~1.1 s while its 573 MB fat binary registers (the
// dlopen of librccl) and ~0.55 s while its code object loads onto the device
// (the "kernels" phase of the first ncclCommInitRank).  Measured on MI355X
// with the node communicator's first generation running on another thread
// of a worker: a warm-start launch waited 1127 ms and an init-kernel launch
// 546 ms, while hipGraphLaunch, hipMalloc and stream calls did not wait at
// all (profiles/r4_collision).  So every kernel here is launched through a
// hipFunction_t resolved once, at *_prepare time (hipGetFuncBySymbol), with
// hipModuleLaunchKernel, which does not consult the registry.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <tuple>
#include <type_traits>
#include <utility>

namespace kiosk {

// hipFunction_t of a __global__ host stub; the first call per kernel asks
// the runtime (under the registry lock), later ones hit a local cache.
// nullptr if the kernel is unknown to the runtime.
hipFunction_t resolve_kernel(const void* stub);

namespace detail {

template <typename Tuple, std::size_t... I>
void fill_args(void** argv, Tuple& values, std::index_sequence<I...>) {
  ((argv[I] = static_cast<void*>(&std::get<I>(values))), ...);
}

}  // namespace detail

// Launches `kernel` like hipLaunchKernelGGL(kernel, grid, block, lds,
// stream, args...).  Arguments are converted to the kernel's exact
// parameter types first (the runtime copies each one with the size the
// kernel's metadata gives it).
template <typename... Params, typename... Args>
hipError_t launch_kernel(void (*kernel)(Params...), dim3 grid, dim3 block,
                         unsigned lds, hipStream_t stream, Args&&... args) {
  static_assert(sizeof...(Params) == sizeof...(Args),
                "launch_kernel: argument count does not match the kernel");
  hipFunction_t f = resolve_kernel(reinterpret_cast<const void*>(kernel));
  if (f == nullptr) return hipErrorInvalidDeviceFunction;
  std::tuple<std::decay_t<Params>...> values(
      static_cast<std::decay_t<Params>>(std::forward<Args>(args))...);
  void* argv[sizeof...(Params) + 1] = {nullptr};
  detail::fill_args(argv, values, std::index_sequence_for<Params...>{});
  return hipModuleLaunchKernel(f, grid.x, grid.y, grid.z, block.x, block.y,
                               block.z, lds, stream, argv, nullptr);
}

// Resolves (and caches) `kernel`'s handle: call from *_prepare so that no
// launch ever pays the registry lookup.
template <typename... Params>
hipError_t prepare_kernel(void (*kernel)(Params...)) {
  return resolve_kernel(reinterpret_cast<const void*>(kernel))
             ? hipSuccess
             : hipErrorInvalidDeviceFunction;
}

}  // namespace kiosk

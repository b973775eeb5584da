// Kernel launches through handles resolved once.
//
// Every kernel here is launched with hipModuleLaunchKernel on a
// hipFunction_t looked up once, at *_prepare time (hipGetFuncBySymbol),
// instead of hipLaunchKernel, which looks the host stub up in the runtime's
// fat-binary registry on every launch.
//
// What this does NOT buy, measured on MI355X (profiles/r4_collision): while
// RCCL registers its 573 MB fat binary (~1.1 s) or loads its code object
// onto the device (~0.55 s, first communicator) on another thread of the
// process, a kernel launch waits either way -- hipLaunchKernel 1127 / 546 ms,
// hipModuleLaunchKernel 1045 / 539 ms.  Only hipGraphLaunch (and memory /
// stream calls) did not wait.  So the worker's READY path is graph launches
// only (the engine's warm-start graph, engine.cpp), and its engine is built
// before the node agent first touches RCCL (worker/main.py).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <tuple>
#include <type_traits>
#include <utility>

namespace kiosk {

// hipFunction_t of a __global__ host stub on the current device; the first
// call per (kernel, device) asks the runtime (under the registry lock),
// later ones hit a local cache.  nullptr if the kernel is unknown to the
// runtime.  (The handle is per device: a process that drives a second
// device gets that device's)
hipFunction_t resolve_kernel(const void* stub);

// Runs `prepare` for the current device unless it already succeeded there:
// a failure is not cached (the next call retries), and each device of the
// process is prepared on its own.
template <typename F>
hipError_t prepare_per_device(std::atomic<unsigned long long>& done,
                              F&& prepare) {
  int device = 0;
  hipError_t err = hipGetDevice(&device);
  if (err != hipSuccess) return err;
  const unsigned long long bit = 1ull << (device & 63);
  if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
  err = prepare();
  if (err == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
  return err;
}

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

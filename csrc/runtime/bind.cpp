// Python bindings for the native module `_kiosk_hip`.
//
// Raw-pointer entry points (gemm, init, sums) let tests drive the kernels
// on torch-allocated tensors (tensor.data_ptr(), the current stream);
// Engine / Fence are the runtime objects the worker uses.  Every
// long-running call releases the GIL.
#include <chrono>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../kernels/kernels.hpp"
#include "engine.hpp"
#include "bind_comm.hpp"
#include "trace.hpp"

namespace py = pybind11;
using kiosk::check_hip;

namespace {

template <typename T>
T* ptr(unsigned long long p) {
  return reinterpret_cast<T*>(static_cast<uintptr_t>(p));
}

hipStream_t stream_of(unsigned long long s) {
  return reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(s));
}

// DLPack (the legacy, unversioned ABI every torch build reads): a device
// buffer of ours handed to torch without a copy.  Only the structs the
// exchange needs; the layout is DLPack's.
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;
constexpr uint8_t kDLUInt = 1;

struct DeviceBuffer {
  DLManagedTensor managed{};
  int64_t shape[1] = {0};
  int64_t strides[1] = {1};
};

void free_device_buffer(DLManagedTensor* t) {
  auto* buf = static_cast<DeviceBuffer*>(t->manager_ctx);
  if (buf->managed.dl_tensor.data) hipFree(buf->managed.dl_tensor.data);
  delete buf;
}

// `nbytes` of device memory from hipMalloc as a uint8 DLPack capsule:
// torch.utils.dlpack.from_dlpack() makes it a tensor that frees it when
// the last view dies.  The PyTorch engine's arena comes from here: one
// allocation outside torch's caching allocator, so closing the engine
// returns the HBM to the device instead of to a cached segment.
py::capsule device_buffer(size_t nbytes, int device) {
  auto* buf = new DeviceBuffer();
  void* data = nullptr;
  hipError_t err;
  {
    py::gil_scoped_release release;
    err = hipSetDevice(device);
    if (err == hipSuccess) err = hipMalloc(&data, nbytes);
  }
  if (err != hipSuccess) {
    delete buf;
    check_hip(err, "hipMalloc(device_buffer)");
  }
  buf->shape[0] = static_cast<int64_t>(nbytes);
  DLTensor& t = buf->managed.dl_tensor;
  t.data = data;
  t.device = {kDLROCM, device};
  t.ndim = 1;
  t.dtype = {kDLUInt, 8, 1};
  t.shape = buf->shape;
  t.strides = buf->strides;
  t.byte_offset = 0;
  buf->managed.manager_ctx = buf;
  buf->managed.deleter = free_device_buffer;
  // a capsule nobody consumed (renamed "used_dltensor" once torch took
  // ownership) frees the buffer itself
  return py::capsule(&buf->managed, "dltensor", [](PyObject* cap) {
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* m = static_cast<DLManagedTensor*>(
          PyCapsule_GetPointer(cap, "dltensor"));
      if (m && m->deleter) m->deleter(m);
    }
  });
}

py::dict warm_to_dict(const kiosk::WarmStartResult& r) {
  py::dict d;
  d["blocks"] = r.blocks;
  d["cus_touched"] = r.distinct_cus;
  d["xccs_touched"] = r.distinct_xccs;
  d["iters"] = r.iters;
  d["lds_bytes"] = r.lds_bytes;
  d["kernel_us"] = r.kernel_us;
  d["span_us"] = r.span_us;
  d["wall_us"] = r.wall_us;
  d["checksum"] = r.checksum;
  d["cu_mask"] = r.cu_keys;
  return d;
}

py::dict fwd_to_dict(const kiosk::ForwardResult& r) {
  py::dict d;
  d["ms"] = r.ms;
  d["gpu_ms"] = r.gpu_ms;
  d["checksum"] = r.checksum;
  d["rows"] = r.rows;
  d["passes"] = r.passes;
  d["graph"] = r.graph;
  return d;
}

// A hipGraph recorded from the caller's own launches on one stream (the
// PyTorch engine's forward and warm start).  torch.cuda.CUDAGraph would also
// capture torch's RNG state and open a private memory pool: 10-27 ms on a
// woken standby's first capture, on its critical path (profiles/r5_boot);
// this engine uses neither.  Capture is thread-local, as the built-in
// engine's, so the node agent's thread may call HIP meanwhile.
class StreamGraph {
 public:
  explicit StreamGraph(unsigned long long stream)
      : stream_(stream_of(stream)) {}
  ~StreamGraph() { reset(); }
  StreamGraph(const StreamGraph&) = delete;
  StreamGraph& operator=(const StreamGraph&) = delete;

  void begin() {
    reset();
    check_hip(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal),
              "hipStreamBeginCapture");
    capturing_ = true;
  }
  // ends the capture and instantiates; after a failed enqueue the caller
  // calls abort() instead
  void end() {
    if (!capturing_) {
      throw std::runtime_error("StreamGraph.end: not capturing");
    }
    capturing_ = false;
    hipGraph_t graph = nullptr;
    hipError_t err = hipStreamEndCapture(stream_, &graph);
    if (err != hipSuccess) {
      if (graph) hipGraphDestroy(graph);
      check_hip(err, "hipStreamEndCapture");
    }
    const auto t0 = std::chrono::steady_clock::now();
    err = hipGraphInstantiate(&exec_, graph, nullptr, nullptr, 0);
    instantiate_us_ = std::chrono::duration<double, std::micro>(
                          std::chrono::steady_clock::now() - t0).count();
    hipGraphDestroy(graph);
    if (err != hipSuccess) exec_ = nullptr;
    check_hip(err, "hipGraphInstantiate");
  }
  void abort() {
    if (!capturing_) return;
    capturing_ = false;
    hipGraph_t graph = nullptr;
    (void)hipStreamEndCapture(stream_, &graph);
    if (graph) hipGraphDestroy(graph);
  }
  void launch() {
    if (!exec_) throw std::runtime_error("StreamGraph.launch: no graph");
    check_hip(hipGraphLaunch(exec_, stream_), "hipGraphLaunch");
  }
  void reset() {
    abort();
    if (exec_) hipGraphExecDestroy(exec_);
    exec_ = nullptr;
  }
  bool ready() const { return exec_ != nullptr; }
  double instantiate_us() const { return instantiate_us_; }

 private:
  hipStream_t stream_;
  hipGraphExec_t exec_ = nullptr;
  bool capturing_ = false;
  double instantiate_us_ = 0.0;
};

}  // namespace

PYBIND11_MODULE(_kiosk_hip, m) {
  m.doc() = "MI355X (gfx950) kernels + runtime for kiosk_autoscaler_amd";
  m.attr("arch") = "gfx950";
  m.attr("gemm_tile") = py::make_tuple(kiosk::kGemmBM, kiosk::kGemmBN,
                                       kiosk::kGemmBK);
  m.attr("gemm_lds_bytes") = kiosk::kGemmLdsBytes;
  m.attr("gemm_ring_lds_bytes") = kiosk::kGemmRingLdsBytes;
  m.def("gemm_set_splitk_fused", &kiosk::gemm_set_splitk_fused,
        py::arg("mode"),
        "4-wave split-K combine: 0 = partial planes + reduce kernel, "
        "1 = in-launch by the last slice (both planes)");
  m.def("gemm_set_group_m", &kiosk::gemm_set_group_m,
        "tile rows per group of the 256-row GEMM tile order (A/B knob)");
  m.def("gemm_group_m", &kiosk::gemm_group_m);
  m.def("gemm_splitk_fused", &kiosk::gemm_splitk_fused);
  m.def("gemm_set_mfma32", &kiosk::gemm_set_mfma32, py::arg("on"));
  m.def("gemm_mfma32", &kiosk::gemm_mfma32);
  m.def("gemm_set_pair", &kiosk::gemm_set_pair, py::arg("on"));
  m.def("gemm_pair", &kiosk::gemm_pair);
  m.attr("sum_blocks") = kiosk::kSumBlocks;

  m.def("gemm_shape_ok", &kiosk::gemm_shape_ok);
  m.def("gemm_pick_variant", &kiosk::gemm_pick_variant, py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("have_workspace") = false);
  m.def("gemm_workspace_bytes", &kiosk::gemm_workspace_bytes);
  m.def(
      "gemm",
      [](unsigned long long a, unsigned long long b, unsigned long long c,
         unsigned long long bias, unsigned long long res, int M, int N, int K,
         int epilogue, unsigned long long stream, int variant,
         unsigned long long workspace, unsigned long long workspace_bytes) {
        // per device, once (an atomic test after the first success)
        check_hip(kiosk::gemm_prepare(), "gemm_prepare");
        check_hip(kiosk::launch_gemm_variant(
                      ptr<const uint16_t>(a), ptr<const uint16_t>(b),
                      ptr<uint16_t>(c), ptr<const float>(bias),
                      ptr<const uint16_t>(res), M, N, K, epilogue, variant,
                      stream_of(stream), ptr<float>(workspace),
                      static_cast<size_t>(workspace_bytes)),
                  "launch_gemm");
      },
      py::arg("a"), py::arg("b"), py::arg("c"), py::arg("bias") = 0,
      py::arg("res") = 0, py::arg("M"), py::arg("N"), py::arg("K"),
      py::arg("epilogue") = 0, py::arg("stream") = 0, py::arg("variant") = 0,
      py::arg("workspace") = 0, py::arg("workspace_bytes") = 0,
      py::call_guard<py::gil_scoped_release>());
  m.def(
      "init_uniform_bf16",
      [](unsigned long long p, size_t n, unsigned long long seed, float lo,
         float hi, unsigned long long stream) {
        check_hip(kiosk::launch_init_uniform_bf16(ptr<uint16_t>(p), n, seed,
                                                  lo, hi, stream_of(stream)),
                  "init_uniform_bf16");
      },
      py::arg("ptr"), py::arg("n"), py::arg("seed"), py::arg("lo") = -1.0f,
      py::arg("hi") = 1.0f, py::arg("stream") = 0,
      py::call_guard<py::gil_scoped_release>());
  // the input of a captured forward: the seed is read on the device at
  // replay time, so one graph serves every job (models/torch_kiosk.py)
  m.def(
      "init_uniform_bf16_devseed",
      [](unsigned long long p, size_t n, unsigned long long seed_ptr,
         float lo, float hi, unsigned long long stream) {
        check_hip(kiosk::launch_init_uniform_bf16_devseed(
                      ptr<uint16_t>(p), n, ptr<const uint64_t>(seed_ptr), lo,
                      hi, stream_of(stream)),
                  "init_uniform_bf16_devseed");
      },
      py::arg("ptr"), py::arg("n"), py::arg("seed_ptr"), py::arg("lo") = -1.0f,
      py::arg("hi") = 1.0f, py::arg("stream") = 0,
      py::call_guard<py::gil_scoped_release>());
  // hipMemsetAsync (a runtime blit kernel, already loaded with the first
  // stream): the PyTorch engine clears its buffers with it, so its boot
  // loads no torch fill kernel from libtorch_hip's code objects
  m.def(
      "memset_async",
      [](unsigned long long p, int value, size_t nbytes,
         unsigned long long stream) {
        check_hip(hipMemsetAsync(ptr<void>(p), value, nbytes,
                                 stream_of(stream)),
                  "hipMemsetAsync");
      },
      py::arg("ptr"), py::arg("value"), py::arg("nbytes"),
      py::arg("stream") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("prepare_kernels",
        [] {
          check_hip(kiosk::gemm_prepare(), "gemm_prepare");
          check_hip(kiosk::misc_prepare(), "misc_prepare");
          check_hip(kiosk::warmstart_prepare(), "warmstart_prepare");
        },
        "raise LDS limits / load code objects once, outside any capture",
        py::call_guard<py::gil_scoped_release>());
  m.def(
      "init_uniform_f32",
      [](unsigned long long p, size_t n, unsigned long long seed, float lo,
         float hi, unsigned long long stream) {
        check_hip(kiosk::launch_init_uniform_f32(ptr<float>(p), n, seed, lo,
                                                 hi, stream_of(stream)),
                  "init_uniform_f32");
      },
      py::arg("ptr"), py::arg("n"), py::arg("seed"), py::arg("lo") = -1.0f,
      py::arg("hi") = 1.0f, py::arg("stream") = 0,
      py::call_guard<py::gil_scoped_release>());
  m.def(
      "partial_sums",
      [](unsigned long long p, size_t n, unsigned long long out,
         unsigned long long stream) {
        check_hip(kiosk::launch_partial_sums(ptr<const uint16_t>(p), n,
                                             ptr<float>(out),
                                             stream_of(stream)),
                  "partial_sums");
      },
      py::arg("ptr"), py::arg("n"), py::arg("out"), py::arg("stream") = 0,
      py::call_guard<py::gil_scoped_release>());
  m.def(
      "warmstart_raw",
      [](unsigned long long w, size_t n, unsigned long long record,
         int nblocks, int iters, int lds_bytes, unsigned long long stream) {
        check_hip(kiosk::launch_warmstart(ptr<const uint16_t>(w), n,
                                          ptr<uint32_t>(record), nblocks,
                                          iters, lds_bytes, stream_of(stream)),
                  "launch_warmstart");
      },
      py::arg("w"), py::arg("n"), py::arg("record"), py::arg("nblocks"),
      py::arg("iters"), py::arg("lds_bytes"), py::arg("stream") = 0,
      py::call_guard<py::gil_scoped_release>());
  // WORKER_PIN=visible: the worker's GPU on the calling thread (the HIP
  // current device is per thread)
  m.def(
      "set_device",
      [](int device) { check_hip(hipSetDevice(device), "hipSetDevice"); },
      py::arg("device"), py::call_guard<py::gil_scoped_release>());
  m.def(
      "preinit_device",
      [](int device) {
        std::vector<std::pair<std::string, long long>> stages;
        {
          py::gil_scoped_release release;
          stages = kiosk::preinit_device(device);
        }
        py::dict d;
        for (const auto& kv : stages) d[py::str(kv.first)] = kv.second;
        return d;
      },
      py::arg("device") = 0);
  m.def(
      "graph_prewarm",
      [](int device) {
        const auto t0 = std::chrono::steady_clock::now();
        check_hip(kiosk::graph_prewarm(device), "graph_prewarm");
        return std::chrono::duration<double, std::milli>(
                   std::chrono::steady_clock::now() - t0).count();
      },
      py::arg("device") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("release_kept_stream", &kiosk::release_kept_stream,
        py::call_guard<py::gil_scoped_release>());
  // the stream preinit_device warmed (its hardware queue already set up)
  m.def("take_stream", &kiosk::take_stream, py::arg("device") = 0);
  m.def("return_stream", &kiosk::return_stream, py::arg("handle"),
        py::arg("device") = 0, py::call_guard<py::gil_scoped_release>());
  m.def(
      "preload_modules",
      [](int device) {
        std::vector<std::pair<std::string, long long>> stages;
        {
          py::gil_scoped_release release;
          stages = kiosk::preload_modules(device);
        }
        py::dict d;
        for (const auto& kv : stages) d[py::str(kv.first)] = kv.second;
        return d;
      },
      py::arg("device") = 0);
  // (free, total) HBM bytes of the current device: a device-mode standby
  // reports it so KEYS_PER_POD is sized against what is actually free
  m.def("mem_info", [] {
    size_t free_b = 0, total_b = 0;
    {
      py::gil_scoped_release release;
      check_hip(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    }
    return py::make_tuple(free_b, total_b);
  });
  // PCI address of a HIP ordinal ("dddd:bb:dd.f"): the manager checks it
  // against the KFD-topology slot it pinned the process to (the
  // ordinal <-> PCI mapping was assumed, never verified)
  m.def(
      "device_pci_bus_id",
      [](int device) {
        char buf[64] = {0};
        {
          py::gil_scoped_release release;
          check_hip(hipDeviceGetPCIBusId(buf, sizeof(buf) - 1, device),
                    "hipDeviceGetPCIBusId");
        }
        return std::string(buf);
      },
      py::arg("device") = 0);
  m.def("device_buffer", &device_buffer, py::arg("nbytes"),
        py::arg("device") = 0);
  // compute units of a device: one attribute query (torch's
  // get_device_properties fills every property first, ~0.1 s on MI355X)
  m.def(
      "device_cus",
      [](int device) {
        int cus = 0;
        check_hip(hipDeviceGetAttribute(
                      &cus, hipDeviceAttributeMultiprocessorCount, device),
                  "hipDeviceGetAttribute");
        return cus;
      },
      py::arg("device") = 0);
  m.def("synchronize", [] { check_hip(hipDeviceSynchronize(), "sync"); },
        py::call_guard<py::gil_scoped_release>());
  m.def("roctx_available", &kiosk::roctx_available);
  m.def("roctx_push", [](const std::string& name) {
    kiosk::roctx_push(name.c_str());
  });
  m.def("roctx_pop", &kiosk::roctx_pop);
  m.def("roctx_mark", [](const std::string& name) {
    kiosk::roctx_mark(name.c_str());
  });

  py::class_<kiosk::Engine>(m, "Engine")
      .def(py::init<int, int, int, int, int, unsigned long long>(),
           py::arg("device"), py::arg("dim"), py::arg("hidden"),
           py::arg("layers"), py::arg("max_rows"), py::arg("seed"),
           py::call_guard<py::gil_scoped_release>())
      .def(
          "warmstart",
          [](kiosk::Engine& e, int iters, int lds_bytes) {
            kiosk::WarmStartResult r;
            {
              py::gil_scoped_release release;
              r = e.warmstart(iters, lds_bytes);
            }
            return warm_to_dict(r);
          },
          py::arg("iters") = 4096,
          py::arg("lds_bytes") = kiosk::kGemmRingLdsBytes)
      .def("prepare", &kiosk::Engine::prepare, py::arg("rows"),
           py::call_guard<py::gil_scoped_release>())
      .def(
          "forward",
          [](kiosk::Engine& e, int rows, int passes,
             unsigned long long seed) {
            kiosk::ForwardResult r;
            {
              py::gil_scoped_release release;
              r = e.forward(rows, passes, seed);
            }
            return fwd_to_dict(r);
          },
          py::arg("rows"), py::arg("passes") = 1, py::arg("seed") = 0)
      .def("spin", &kiosk::Engine::spin, py::arg("ms"),
           py::call_guard<py::gil_scoped_release>())
      .def("close", &kiosk::Engine::close,
           py::call_guard<py::gil_scoped_release>())
      .def("stage_times",
           [](const kiosk::Engine& e) {
             py::dict d;
             for (const auto& kv : e.stages()) d[py::str(kv.first)] = kv.second;
             return d;
           })
      .def("info", &kiosk::Engine::info)
      .def("copy_output", &kiosk::Engine::copy_output, py::arg("dst"),
           py::arg("rows"), py::call_guard<py::gil_scoped_release>())
      .def("weight_ptr", &kiosk::Engine::weight_ptr)
      .def("act_ptr", &kiosk::Engine::act_ptr)
      .def_property_readonly("stream", &kiosk::Engine::stream_handle)
      .def_property_readonly("dim", &kiosk::Engine::dim)
      .def_property_readonly("hidden", &kiosk::Engine::hidden)
      .def_property_readonly("layers", &kiosk::Engine::layers)
      .def_property_readonly("max_rows", &kiosk::Engine::max_rows);

  py::class_<StreamGraph>(m, "StreamGraph")
      .def(py::init<unsigned long long>(), py::arg("stream"))
      .def("begin", &StreamGraph::begin,
           py::call_guard<py::gil_scoped_release>())
      .def("end", &StreamGraph::end, py::call_guard<py::gil_scoped_release>())
      .def("abort", &StreamGraph::abort,
           py::call_guard<py::gil_scoped_release>())
      .def("launch", &StreamGraph::launch,
           py::call_guard<py::gil_scoped_release>())
      .def("reset", &StreamGraph::reset,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("ready", &StreamGraph::ready)
      .def_property_readonly("instantiate_us", &StreamGraph::instantiate_us);
  // hipMemcpyAsync (either direction, pinned host memory): inside a
  // StreamGraph capture it becomes a copy node
  m.def(
      "memcpy_async",
      [](unsigned long long dst, unsigned long long src, size_t nbytes,
         unsigned long long stream) {
        check_hip(hipMemcpyAsync(ptr<void>(dst), ptr<const void>(src), nbytes,
                                 hipMemcpyDefault, stream_of(stream)),
                  "hipMemcpyAsync");
      },
      py::arg("dst"), py::arg("src"), py::arg("nbytes"), py::arg("stream") = 0,
      py::call_guard<py::gil_scoped_release>());

  kiosk::bind_comm(m);
}

// Worker inference engine (see engine.hpp).
#include "engine.hpp"

#include <time.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <set>

#include "../kernels/kernels.hpp"
#include "trace.hpp"

namespace kiosk {

void check_hip(hipError_t err, const char* what) {
  if (err != hipSuccess) {
    throw std::runtime_error(std::string(what) + ": " +
                             hipGetErrorString(err));
  }
}

long long monotonic_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<long long>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

namespace {
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// The stream preinit_device warmed up (its first launches paid the queue
// setup): kept for the next Engine instead of being destroyed, so a fresh
// standby's first assignment does not pay hipStreamCreate again (~14 ms on
// MI355X, profiles/r2_worker_final/).  The engine takes ownership.
std::mutex g_kept_mu;
hipStream_t g_kept_stream = nullptr;
int g_kept_device = -1;

hipStream_t take_kept_stream(int device) {
  std::lock_guard<std::mutex> lock(g_kept_mu);
  if (g_kept_device != device) return nullptr;
  hipStream_t s = g_kept_stream;
  g_kept_stream = nullptr;
  g_kept_device = -1;
  return s;
}

// Destroys a kept stream on the device it was created on (a process may
// preinit more than one device; the current device is restored).
void destroy_on_device(hipStream_t s, int device) {
  if (!s) return;
  int current = -1;
  (void)hipGetDevice(&current);
  if (device >= 0 && device != current) (void)hipSetDevice(device);
  (void)hipStreamDestroy(s);
  if (device >= 0 && device != current && current >= 0) {
    (void)hipSetDevice(current);
  }
}

void keep_stream(hipStream_t s, int device) {
  hipStream_t old = nullptr;
  int old_device = -1;
  {
    std::lock_guard<std::mutex> lock(g_kept_mu);
    old = g_kept_stream;
    old_device = g_kept_device;
    g_kept_stream = s;
    g_kept_device = device;
  }
  destroy_on_device(old, old_device);
}
}  // namespace

unsigned long long take_stream(int device) {
  return static_cast<unsigned long long>(
      reinterpret_cast<uintptr_t>(take_kept_stream(device)));
}

void return_stream(unsigned long long handle, int device) {
  keep_stream(reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(handle)),
              device);
}

void release_kept_stream() {
  hipStream_t s = nullptr;
  int device = -1;
  {
    std::lock_guard<std::mutex> lock(g_kept_mu);
    s = g_kept_stream;
    device = g_kept_device;
    g_kept_stream = nullptr;
    g_kept_device = -1;
  }
  destroy_on_device(s, device);
}

hipError_t graph_prewarm(int device) {
  // The HIP runtime's first hipGraphInstantiate of a graph with a node pays
  // a one-time set-up (5-16 ms on MI355X, whatever the graph holds; the
  // next instantiations take 0.02-0.06 ms, profiles/r5_boot): paid here,
  // by the standby's boot, on a graph of one 4-byte memset built without a
  // stream (no capture, no queue).
  hipError_t err = hipSetDevice(device);
  if (err != hipSuccess) return err;
  void* buf = nullptr;
  err = hipMalloc(&buf, 256);
  if (err != hipSuccess) return err;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  err = hipGraphCreate(&graph, 0);
  if (err == hipSuccess) {
    hipMemsetParams params{};
    params.dst = buf;
    params.value = 0;
    params.elementSize = 4;
    params.width = 1;
    params.height = 1;
    params.pitch = 4;
    hipGraphNode_t node = nullptr;
    err = hipGraphAddMemsetNode(&node, graph, nullptr, 0, &params);
  }
  if (err == hipSuccess) err = hipGraphInstantiate(&exec, graph, nullptr,
                                                   nullptr, 0);
  if (exec) hipGraphExecDestroy(exec);
  if (graph) hipGraphDestroy(graph);
  hipError_t free_err = hipFree(buf);
  return err != hipSuccess ? err : free_err;
}

std::vector<std::pair<std::string, long long>> preinit_device(int device) {
  TraceRange range("kiosk.preinit");
  std::vector<std::pair<std::string, long long>> stages;
  stages.emplace_back("preinit_enter", monotonic_ns());
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_hip(hipFree(nullptr), "hip context init");
  stages.emplace_back("preinit_context", monotonic_ns());
  // every launch handle resolved now: no later launch consults the
  // runtime's fat-binary registry (kernels/launch.hpp).  (Run beside the
  // stream's creation on a helper thread, the two only slowed each other:
  // 19 + 17 ms against 7 + 12 ms, profiles/r5_boot.)
  check_hip(gemm_prepare(), "gemm_prepare");
  check_hip(misc_prepare(), "misc_prepare");
  check_hip(warmstart_prepare(), "warmstart_prepare");
  stages.emplace_back("preinit_prepared", monotonic_ns());
  hipStream_t stream = take_kept_stream(device);
  if (!stream) {
    check_hip(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking),
              "hipStreamCreate");
  }
  stages.emplace_back("preinit_stream", monotonic_ns());
  // the engine's first graph then instantiates in 0.05 ms instead of 6-16
  try {
    check_hip(graph_prewarm(device), "graph_prewarm");
  } catch (...) {
    (void)hipStreamDestroy(stream);
    throw;
  }
  stages.emplace_back("preinit_graph_prewarm", monotonic_ns());
  // 128x128 operands + bias + output + sums + warm-start record
  const size_t elems = 128 * 128;
  char* scratch = nullptr;
  // split-K probe: 2 partial planes + the 4-wave path's ticket counter
  const size_t ws_bytes = 2 * 64 * 256 * sizeof(float) + 256;
  const size_t bytes =
      4 * elems * 2 + 128 * 4 + kSumBlocks * 4 + 4096 + ws_bytes;
  check_hip(hipMalloc(reinterpret_cast<void**>(&scratch), bytes),
            "hipMalloc(preinit)");
  uint16_t* a = reinterpret_cast<uint16_t*>(scratch);
  uint16_t* b = a + elems;
  uint16_t* c = b + elems;
  uint16_t* r = c + elems;
  float* bias = reinterpret_cast<float*>(r + elems);
  float* sums = bias + 128;
  uint32_t* rec = reinterpret_cast<uint32_t*>(sums + kSumBlocks);
  float* ws = reinterpret_cast<float*>(scratch + bytes - ws_bytes);
  check_hip(launch_init_uniform_bf16(a, 4 * elems, 1, -1.f, 1.f, stream),
            "preinit init");
  check_hip(launch_init_uniform_f32(bias, 128, 2, -1.f, 1.f, stream),
            "preinit init f32");
  check_hip(hipStreamSynchronize(stream), "preinit first sync");
  stages.emplace_back("preinit_first_launch", monotonic_ns());
  for (int epi = 0; epi < 3; ++epi) {
    check_hip(launch_gemm(a, b, c, bias, r, 128, 128, 128, epi, stream),
              "preinit gemm");
  }
  // the 256x256 ring kernel needs a 256-wide operand: reuse the buffers
  // as [128 x 256] / [256 x 64] views (N = 256, K = 64)
  for (int epi = 0; epi < 3; ++epi) {
    for (int bn : {256, 128}) {
      check_hip(launch_gemm256(a, b, c, bias, r, 64, 256, 64, epi, stream,
                               bn),
                "preinit gemm256");
    }
    check_hip(launch_gemm256(a, b, c, bias, r, 64, 256, 64, epi, stream, 256,
                             4),
              "preinit gemm256 4-wave");
    // split-K partial kernel + this epilogue's reduce kernel
    check_hip(launch_gemm256_splitk(a, b, c, bias, r, 64, 256, 64, epi, 2, ws,
                                    ws_bytes, stream),
              "preinit gemm256 split-K");
    // K = 128 in two 64-deep slices: the 4-wave fused split-K kernel (B
    // spans the b, c views; the output tile c is written only by the last
    // slice, after both slices have read their operands)
    check_hip(launch_gemm256_splitk(a, b, c, bias, r, 64, 256, 128, epi, 2,
                                    ws, ws_bytes, stream),
              "preinit gemm256 4-wave split-K");
  }
  check_hip(launch_partial_sums(c, elems, sums, stream), "preinit sums");
  check_hip(launch_warmstart(a, elems, rec, 1, 1, kGemmRingLdsBytes, stream),
            "preinit warmstart");
  check_hip(hipStreamSynchronize(stream), "preinit sync");
  check_hip(hipFree(scratch), "hipFree(preinit)");
  keep_stream(stream, device);
  stages.emplace_back("preinit_done", monotonic_ns());
  return stages;
}

std::vector<std::pair<std::string, long long>> preload_modules(int device) {
  TraceRange range("kiosk.preload");
  std::vector<std::pair<std::string, long long>> stages;
  stages.emplace_back("preload_enter", monotonic_ns());
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_hip(hipFree(nullptr), "hip context init");
  stages.emplace_back("preload_context", monotonic_ns());
  check_hip(gemm_prepare(), "gemm_prepare");
  check_hip(misc_prepare(), "misc_prepare");
  check_hip(warmstart_prepare(), "warmstart_prepare");
  stages.emplace_back("preload_done", monotonic_ns());
  return stages;
}

void Engine::stage(const char* name) {
  stages_.emplace_back(name, monotonic_ns());
}

void Engine::launch_or_throw(hipError_t err, const char* what) {
  check_hip(err, what);
}

Engine::Engine(int device, int dim, int hidden, int layers, int max_rows,
               unsigned long long seed)
    : device_(device), dim_(dim), hidden_(hidden), layers_(layers),
      max_rows_(max_rows) {
  if (!gemm_shape_ok(1, hidden, dim) || !gemm_shape_ok(1, dim, hidden)) {
    throw std::invalid_argument(
        "model dims must be multiples of 128 (dim and hidden)");
  }
  if (layers < 1 || max_rows < 1) {
    throw std::invalid_argument("layers and max_rows must be >= 1");
  }
  // a constructor that throws never runs the destructor: release whatever
  // was created before the failure, then rethrow
  try {
    init(device, seed);
  } catch (...) {
    close();
    throw;
  }
}

void Engine::init(int device, unsigned long long seed) {
  const int dim = dim_, hidden = hidden_, layers = layers_;
  const int max_rows = max_rows_;
  stage("engine_enter");
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_hip(hipFree(nullptr), "hip context init");
  stage("hip_context");
  check_hip(hipDeviceGetAttribute(&cu_count_, hipDeviceAttributeMultiprocessorCount,
                                  device),
            "hipDeviceGetAttribute");
  stream_ = take_kept_stream(device);
  if (!stream_) {
    check_hip(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking),
              "hipStreamCreate");
  }
  check_hip(hipEventCreate(&ev0_), "hipEventCreate");
  check_hip(hipEventCreate(&ev1_), "hipEventCreate");
  check_hip(gemm_prepare(), "gemm_prepare");   // (no-ops after preinit)
  check_hip(misc_prepare(), "misc_prepare");
  check_hip(warmstart_prepare(), "warmstart_prepare");
  stage("stream_ready");

  // One arena: per-layer W1 [H,D], b1 [H], W2 [D,H], b2 [D]; then x, y, h,
  // partial sums and the device-side seed.
  const size_t A = 256;
  std::vector<size_t> offsets;
  size_t off = 0;
  for (int l = 0; l < layers; ++l) {
    offsets.push_back(off); off = align_up(off + size_t(hidden) * dim * 2, A);
    offsets.push_back(off); off = align_up(off + size_t(hidden) * 4, A);
    offsets.push_back(off); off = align_up(off + size_t(dim) * hidden * 2, A);
    offsets.push_back(off); off = align_up(off + size_t(dim) * 4, A);
  }
  const size_t x_off = off; off = align_up(off + size_t(max_rows) * dim * 2, A);
  const size_t y_off = off; off = align_up(off + size_t(max_rows) * dim * 2, A);
  const size_t h_off = off; off = align_up(off + size_t(max_rows) * hidden * 2, A);
  const size_t p_off = off; off = align_up(off + kSumBlocks * 4, A);
  const size_t s_off = off; off = align_up(off + 8, A);
  // split-K workspace: the largest fp32 partial set either GEMM can want
  // for any row count up to max_rows (the split count changes only at
  // 256-row boundaries, so probing those and max_rows covers every M)
  size_t ws = 0;
  for (int m = 256; m < max_rows + 256; m += 256) {
    const int rows = std::min(m, max_rows);
    ws = std::max(ws, gemm_workspace_bytes(rows, hidden, dim));
    ws = std::max(ws, gemm_workspace_bytes(rows, dim, hidden));
  }
  const size_t w_off = off; off = align_up(off + ws, A);
  workspace_bytes_ = ws;
  arena_bytes_ = off;
  check_hip(hipMalloc(reinterpret_cast<void**>(&arena_), arena_bytes_),
            "hipMalloc(arena)");
  for (int l = 0; l < layers; ++l) {
    w1_.push_back(reinterpret_cast<uint16_t*>(arena_ + offsets[4 * l + 0]));
    b1_.push_back(reinterpret_cast<float*>(arena_ + offsets[4 * l + 1]));
    w2_.push_back(reinterpret_cast<uint16_t*>(arena_ + offsets[4 * l + 2]));
    b2_.push_back(reinterpret_cast<float*>(arena_ + offsets[4 * l + 3]));
  }
  x_ = reinterpret_cast<uint16_t*>(arena_ + x_off);
  y_ = reinterpret_cast<uint16_t*>(arena_ + y_off);
  h_ = reinterpret_cast<uint16_t*>(arena_ + h_off);
  partials_ = reinterpret_cast<float*>(arena_ + p_off);
  seed_dev_ = reinterpret_cast<unsigned long long*>(arena_ + s_off);
  workspace_ = ws ? reinterpret_cast<float*>(arena_ + w_off) : nullptr;
  check_hip(hipHostMalloc(reinterpret_cast<void**>(&seed_host_), 8),
            "hipHostMalloc(seed)");
  check_hip(hipHostMalloc(reinterpret_cast<void**>(&partials_host_),
                          kSumBlocks * 4),
            "hipHostMalloc(partials)");
  stage("hbm_alloc");

  // Random-init weights on the device (PyTorch nn.Linear-style bounds).
  const float bd = 1.0f / std::sqrt(static_cast<float>(dim));
  const float bh = 1.0f / std::sqrt(static_cast<float>(hidden));
  for (int l = 0; l < layers; ++l) {
    const unsigned long long s = seed * 1000003ull + 16ull * l;
    launch_or_throw(launch_init_uniform_bf16(w1_[l], size_t(hidden) * dim,
                                             s + 1, -bd, bd, stream_),
                    "init W1");
    launch_or_throw(launch_init_uniform_f32(b1_[l], hidden, s + 2, -bd, bd,
                                            stream_),
                    "init b1");
    launch_or_throw(launch_init_uniform_bf16(w2_[l], size_t(dim) * hidden,
                                             s + 3, -bh, bh, stream_),
                    "init W2");
    launch_or_throw(launch_init_uniform_f32(b2_[l], dim, s + 4, -bh, bh,
                                            stream_),
                    "init b2");
  }
  check_hip(hipStreamSynchronize(stream_), "weights init sync");
  stage("weights_init");
}

Engine::~Engine() {
  try {
    close();
  } catch (...) {
  }
}

void Engine::close() {
  if (closed_) return;
  closed_ = true;
  for (auto& kv : graphs_) {
    hipGraphExecDestroy(kv.second.second);
    hipGraphDestroy(kv.second.first);
  }
  graphs_.clear();
  if (warm_exec_) hipGraphExecDestroy(warm_exec_);
  if (warm_graph_) hipGraphDestroy(warm_graph_);
  warm_exec_ = nullptr;
  warm_graph_ = nullptr;
  if (stream_) hipStreamSynchronize(stream_);
  if (warm_rec_) hipFree(warm_rec_);
  if (warm_host_) hipHostFree(warm_host_);
  warm_rec_ = nullptr;
  warm_host_ = nullptr;
  if (arena_) hipFree(arena_);
  if (seed_host_) hipHostFree(seed_host_);
  if (partials_host_) hipHostFree(partials_host_);
  if (ev0_) hipEventDestroy(ev0_);
  if (ev1_) hipEventDestroy(ev1_);
  if (stream_) hipStreamDestroy(stream_);
  arena_ = nullptr;
  seed_host_ = nullptr;
  partials_host_ = nullptr;
  stream_ = nullptr;
  ev0_ = ev1_ = nullptr;
}

void Engine::build_warm_graph(int iters, int lds_bytes) {
  TraceRange range("kiosk.warm_graph");
  if (warm_exec_) hipGraphExecDestroy(warm_exec_);
  if (warm_graph_) hipGraphDestroy(warm_graph_);
  warm_exec_ = nullptr;
  warm_graph_ = nullptr;
  const size_t words = size_t(cu_count_) * kWarmRecordWords;
  if (!warm_rec_) {
    check_hip(hipMalloc(reinterpret_cast<void**>(&warm_rec_), words * 4),
              "hipMalloc(warm record)");
    check_hip(hipHostMalloc(reinterpret_cast<void**>(&warm_host_), words * 4),
              "hipHostMalloc(warm record)");
  }
  hipGraph_t graph = nullptr;
  check_hip(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal),
            "begin warm capture");
  hipError_t err = hipMemsetAsync(warm_rec_, 0, words * 4, stream_);
  if (err == hipSuccess)
    err = launch_warmstart(w1_[0], size_t(hidden_) * dim_, warm_rec_,
                           cu_count_, iters, lds_bytes, stream_);
  if (err == hipSuccess)
    err = hipMemcpyAsync(warm_host_, warm_rec_, words * 4,
                         hipMemcpyDeviceToHost, stream_);
  hipError_t end = hipStreamEndCapture(stream_, &graph);
  if (err != hipSuccess || end != hipSuccess) {
    if (graph) hipGraphDestroy(graph);
    check_hip(err != hipSuccess ? err : end, "warm-start capture");
  }
  hipGraphExec_t exec = nullptr;
  err = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  if (err != hipSuccess) {
    hipGraphDestroy(graph);
    check_hip(err, "warm graph instantiate");
  }
  warm_graph_ = graph;
  warm_exec_ = exec;
  warm_iters_ = iters;
  warm_lds_ = lds_bytes;
}

WarmStartResult Engine::warmstart(int iters, int lds_bytes) {
  if (closed_) throw std::runtime_error("engine closed");
  TraceRange range("kiosk.warmstart");
  WarmStartResult r;
  r.blocks = cu_count_;
  r.iters = iters;
  r.lds_bytes = lds_bytes;
  const long long t0 = monotonic_ns();
  if (!warm_exec_ || warm_iters_ != iters || warm_lds_ != lds_bytes)
    build_warm_graph(iters, lds_bytes);
  const size_t words = size_t(r.blocks) * kWarmRecordWords;
  check_hip(hipEventRecord(ev0_, stream_), "event");
  check_hip(hipGraphLaunch(warm_exec_, stream_), "warm graph launch");
  check_hip(hipEventRecord(ev1_, stream_), "event");
  check_hip(hipStreamSynchronize(stream_), "warmstart sync");
  std::vector<uint32_t> host(warm_host_, warm_host_ + words);
  float ms = 0;
  hipEventElapsedTime(&ms, ev0_, ev1_);
  r.kernel_us = ms * 1e3;
  r.wall_us = (monotonic_ns() - t0) / 1e3;
  std::set<unsigned> cus, xccs;
  unsigned long long tmin = ~0ull, tmax = 0;
  double checksum = 0;
  for (int b = 0; b < r.blocks; ++b) {
    const uint32_t* w = &host[size_t(b) * kWarmRecordWords];
    const unsigned hw = w[0], xcc = w[1] & 0xf;
    const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 0x1,
                   se = (hw >> 13) & 0x7;
    cus.insert((xcc << 16) | (se << 8) | (sh << 4) | cu);
    xccs.insert(xcc);
    const unsigned long long a = (static_cast<unsigned long long>(w[3]) << 32) | w[2];
    const unsigned long long z = (static_cast<unsigned long long>(w[5]) << 32) | w[4];
    if (a) tmin = std::min(tmin, a);
    tmax = std::max(tmax, z);
    float f;
    std::memcpy(&f, &w[6], 4);
    checksum += f;
  }
  r.distinct_cus = static_cast<int>(cus.size());
  r.distinct_xccs = static_cast<int>(xccs.size());
  r.span_us = tmax > tmin ? (tmax - tmin) / 100.0 : 0.0;  // 100 MHz clock
  r.checksum = checksum;
  r.cu_keys.assign(cus.begin(), cus.end());
  stage("warmstart");
  return r;
}

void Engine::enqueue_forward(int rows) {
  launch_or_throw(launch_init_uniform_bf16_devseed(
                      x_, size_t(rows) * dim_,
                      reinterpret_cast<const uint64_t*>(seed_dev_), -1.0f,
                      1.0f, stream_),
                  "input init");
  uint16_t* cur = x_;
  uint16_t* nxt = y_;
  for (int l = 0; l < layers_; ++l) {
    launch_or_throw(launch_gemm_variant(cur, w1_[l], h_, b1_[l], nullptr, rows,
                                        hidden_, dim_, EPI_BIAS_GELU,
                                        GEMM_AUTO, stream_, workspace_,
                                        workspace_bytes_),
                    "gemm1");
    launch_or_throw(launch_gemm_variant(h_, w2_[l], nxt, b2_[l], cur, rows,
                                        dim_, hidden_, EPI_BIAS_RESIDUAL,
                                        GEMM_AUTO, stream_, workspace_,
                                        workspace_bytes_),
                    "gemm2");
    std::swap(cur, nxt);
  }
  launch_or_throw(launch_partial_sums(cur, size_t(rows) * dim_, partials_,
                                      stream_),
                  "partial sums");
}

double Engine::spin(double ms) {
  if (closed_) throw std::runtime_error("engine closed");
  TraceRange range("kiosk.fault.spin");
  const long long t0 = monotonic_ns();
  check_hip(launch_spin(ms, nullptr, stream_), "launch_spin");
  check_hip(hipStreamSynchronize(stream_), "spin sync");
  return (monotonic_ns() - t0) / 1e6;
}

void Engine::prepare(int rows) {
  if (closed_) throw std::runtime_error("engine closed");
  if (rows < 1 || rows > max_rows_) {
    throw std::invalid_argument("rows out of range for this engine");
  }
  if (graphs_.count(rows)) return;
  TraceRange range("kiosk.graph_capture");
  if (graphs_.size() >= 16) {
    auto victim = graphs_.begin();
    hipGraphExecDestroy(victim->second.second);
    hipGraphDestroy(victim->second.first);
    graphs_.erase(victim);
  }
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  check_hip(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal),
            "begin capture");
  try {
    enqueue_forward(rows);
  } catch (...) {
    hipStreamEndCapture(stream_, &graph);
    if (graph) hipGraphDestroy(graph);
    throw;
  }
  check_hip(hipStreamEndCapture(stream_, &graph), "end capture");
  check_hip(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0),
            "graph instantiate");
  graphs_[rows] = std::make_pair(graph, exec);
  stage("graph_ready");
}

ForwardResult Engine::forward(int rows, int passes, unsigned long long seed) {
  if (closed_) throw std::runtime_error("engine closed");
  if (rows < 1 || rows > max_rows_) {
    throw std::invalid_argument("rows exceeds the engine's max_rows");
  }
  ForwardResult r;
  r.rows = rows;
  r.passes = std::max(1, passes);
  const long long t0 = monotonic_ns();
  prepare(rows);
  TraceRange range("kiosk.forward");
  auto exec = graphs_[rows].second;
  *seed_host_ = seed;
  check_hip(hipMemcpyAsync(seed_dev_, seed_host_, 8, hipMemcpyHostToDevice,
                           stream_),
            "seed upload");
  check_hip(hipEventRecord(ev0_, stream_), "event");
  for (int p = 0; p < r.passes; ++p) {
    check_hip(hipGraphLaunch(exec, stream_), "graph launch");
  }
  check_hip(hipEventRecord(ev1_, stream_), "event");
  check_hip(hipMemcpyAsync(partials_host_, partials_, kSumBlocks * 4,
                           hipMemcpyDeviceToHost, stream_),
            "partials download");
  check_hip(hipStreamSynchronize(stream_), "forward sync");
  float ms = 0;
  hipEventElapsedTime(&ms, ev0_, ev1_);
  double sum = 0;
  for (int b = 0; b < kSumBlocks; ++b) sum += partials_host_[b];
  r.checksum = sum;
  r.gpu_ms = ms;
  r.ms = (monotonic_ns() - t0) / 1e6;
  r.graph = true;
  return r;
}

void Engine::copy_output(unsigned long long dst, int rows) {
  if (closed_) throw std::runtime_error("engine closed");
  if (rows < 1 || rows > max_rows_) {
    throw std::invalid_argument("rows exceeds the engine's max_rows");
  }
  // the layers ping-pong x_ <-> y_ starting from x_: an even layer count
  // ends in x_ (enqueue_forward)
  const uint16_t* out = (layers_ % 2 == 0) ? x_ : y_;
  check_hip(hipMemcpyAsync(reinterpret_cast<void*>(dst), out,
                           size_t(rows) * dim_ * sizeof(uint16_t),
                           hipMemcpyDeviceToDevice, stream_),
            "output copy");
  check_hip(hipStreamSynchronize(stream_), "output sync");
}

std::map<std::string, double> Engine::info() const {
  std::map<std::string, double> out;
  size_t free_b = 0, total_b = 0;
  hipMemGetInfo(&free_b, &total_b);
  out["cu_count"] = cu_count_;
  out["hbm_free_bytes"] = static_cast<double>(free_b);
  out["hbm_total_bytes"] = static_cast<double>(total_b);
  out["arena_bytes"] = static_cast<double>(arena_bytes_);
  out["workspace_bytes"] = static_cast<double>(workspace_bytes_);
  out["graphs"] = static_cast<double>(graphs_.size());
  int clock_khz = 0;
  hipDeviceGetAttribute(&clock_khz, hipDeviceAttributeClockRate, device_);
  out["clock_khz"] = clock_khz;
  return out;
}

unsigned long long Engine::weight_ptr(int layer, int which) const {
  if (layer < 0 || layer >= layers_) throw std::out_of_range("layer");
  switch (which) {
    case 0: return reinterpret_cast<unsigned long long>(w1_[layer]);
    case 1: return reinterpret_cast<unsigned long long>(b1_[layer]);
    case 2: return reinterpret_cast<unsigned long long>(w2_[layer]);
    case 3: return reinterpret_cast<unsigned long long>(b2_[layer]);
    default: throw std::out_of_range("which");
  }
}

unsigned long long Engine::act_ptr(int which) const {
  switch (which) {
    case 0: return reinterpret_cast<unsigned long long>(x_);
    case 1: return reinterpret_cast<unsigned long long>(y_);
    case 2: return reinterpret_cast<unsigned long long>(h_);
    default: throw std::out_of_range("which");
  }
}

}  // namespace kiosk

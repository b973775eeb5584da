// RCCL membership fence (see fence.hpp).
#include "fence.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include "engine.hpp"
#include "trace.hpp"

namespace kiosk {

struct RcclApi {
  void* handle = nullptr;
  std::string path;
  decltype(&::ncclGetVersion) GetVersion = nullptr;
  decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&::ncclCommInitRankConfig) CommInitRankConfig = nullptr;
  decltype(&::ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&::ncclCommAbort) CommAbort = nullptr;
  decltype(&::ncclCommDestroy) CommDestroy = nullptr;
  decltype(&::ncclCommFinalize) CommFinalize = nullptr;
  decltype(&::ncclAllReduce) AllReduce = nullptr;
  decltype(&::ncclGetErrorString) GetErrorString = nullptr;
  decltype(&::ncclCommShrink) CommShrink = nullptr;   // optional
};

namespace {

template <typename T>
void bind(void* handle, const char* name, T& slot, bool required) {
  slot = reinterpret_cast<T>(dlsym(handle, name));
  if (!slot && required) {
    throw std::runtime_error(std::string("RCCL symbol missing: ") + name);
  }
}

// One library path: dlopen + symbol binding, or nullptr with `errors`
// extended.  A handle is never closed (an RCCL cannot be unloaded safely).
RcclApi* load_rccl_path(const std::string& path, std::string& errors) {
  void* handle = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!handle) {
    const char* e = dlerror();
    errors += path + ": " + (e ? e : "?") + "; ";
    return nullptr;
  }
  auto* api = new RcclApi();
  api->handle = handle;
  api->path = path;
  try {
    bind(handle, "ncclGetVersion", api->GetVersion, true);
    bind(handle, "ncclGetUniqueId", api->GetUniqueId, true);
    bind(handle, "ncclCommInitRankConfig", api->CommInitRankConfig, true);
    bind(handle, "ncclCommGetAsyncError", api->CommGetAsyncError, true);
    bind(handle, "ncclCommAbort", api->CommAbort, true);
    bind(handle, "ncclCommDestroy", api->CommDestroy, true);
    bind(handle, "ncclCommFinalize", api->CommFinalize, true);
    bind(handle, "ncclAllReduce", api->AllReduce, true);
    bind(handle, "ncclGetErrorString", api->GetErrorString, true);
    bind(handle, "ncclCommShrink", api->CommShrink, false);
  } catch (const std::exception& e) {
    errors += path + ": " + e.what() + "; ";
    delete api;
    return nullptr;
  }
  return api;
}

// Every library loaded so far (path -> api) and the one new communicators
// use.  The manager can move a node from one RCCL to another between
// generations (slim copy -> stock library, gpumgr/nodecomm.py): a process
// that loaded the slim copy loads the stock one beside it (RTLD_LOCAL: two
// independent copies), and a Fence keeps the api it was built with.
std::mutex g_api_mu;
std::vector<RcclApi*> g_apis;
std::atomic<RcclApi*> g_current{nullptr};
std::string g_error;

RcclApi* find_loaded(const std::string& path) {
  for (RcclApi* api : g_apis) {
    if (api->path == path) return api;
  }
  return nullptr;
}

RcclApi* load_default() {
  std::vector<std::string> candidates;
  if (const char* env = std::getenv("KIOSK_RCCL_LIB")) candidates.push_back(env);
  candidates.push_back("/opt/rocm/lib/librccl.so.1");
  candidates.push_back("librccl.so.1");
  std::string errors;
  for (const auto& path : candidates) {
    if (RcclApi* api = find_loaded(path)) return api;
    if (RcclApi* api = load_rccl_path(path, errors)) {
      g_apis.push_back(api);
      return api;
    }
  }
  g_error = "no usable RCCL library: " + errors;
  return nullptr;
}

void check_nccl(ncclResult_t res, const char* what,
                const RcclApi* api = nullptr) {
  if (res != ncclSuccess && res != ncclInProgress) {
    throw std::runtime_error(std::string(what) + ": " +
                             (api ? *api : rccl()).GetErrorString(res));
  }
}

double now_s() {
  return std::chrono::duration<double>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

const RcclApi& rccl() {
  RcclApi* api = g_current.load(std::memory_order_acquire);
  if (api) return *api;
  std::lock_guard<std::mutex> lock(g_api_mu);
  api = g_current.load(std::memory_order_relaxed);
  if (!api) {
    api = load_default();
    if (!api) throw std::runtime_error(g_error);
    g_current.store(api, std::memory_order_release);
  }
  return *api;
}

std::string rccl_use_library(const std::string& path) {
  if (path.empty()) return rccl().path;
  std::lock_guard<std::mutex> lock(g_api_mu);
  RcclApi* api = find_loaded(path);
  if (!api) {
    std::string errors;
    api = load_rccl_path(path, errors);
    if (!api) throw std::runtime_error("cannot load RCCL " + errors);
    g_apis.push_back(api);
  }
  g_current.store(api, std::memory_order_release);
  return api->path;
}

std::vector<std::string> rccl_loaded_libraries() {
  std::lock_guard<std::mutex> lock(g_api_mu);
  std::vector<std::string> out;
  for (RcclApi* api : g_apis) out.push_back(api->path);
  return out;
}

std::string rccl_library() { return rccl().path; }

int rccl_version() {
  int v = 0;
  check_nccl(rccl().GetVersion(&v), "ncclGetVersion");
  return v;
}

bool rccl_can_shrink() { return rccl().CommShrink != nullptr; }

std::string rccl_unique_id() {
  ncclUniqueId id;
  check_nccl(rccl().GetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

double rccl_dlopen() {
  const double t0 = now_s();
  rccl();
  return (now_s() - t0) * 1e3;
}

double rccl_preload() {
  const double t0 = now_s();
  rccl_version();
  (void)rccl_unique_id();
  return (now_s() - t0) * 1e3;
}

double rccl_warmup(double timeout_s) {
  const double t0 = now_s();
  Fence fence(rccl_unique_id(), 1, 0, timeout_s);
  fence.allreduce(std::vector<long long>{1});
  fence.destroy();
  return (now_s() - t0) * 1e3;
}

// Polls a non-blocking communicator until its pending operation settles.
// Never aborts: on failure, timeout or request_abort() it throws and the
// caller aborts exactly once (the communicator may be comm_ or a shrink
// child that is not owned yet).
void Fence::wait_ready(void* comm, double timeout_s, const char* what) {
  const double deadline = now_s() + timeout_s;
  while (true) {
    ncclResult_t state = ncclSuccess;
    ncclResult_t res = api_->CommGetAsyncError(
        static_cast<ncclComm_t>(comm), &state);
    if (res != ncclSuccess) state = res;
    if (state == ncclSuccess) return;
    if (state != ncclInProgress) {
      throw std::runtime_error(std::string(what) + " failed: " +
                               api_->GetErrorString(state));
    }
    if (abort_requested_.load(std::memory_order_relaxed)) {
      throw std::runtime_error(std::string(what) + " aborted on request");
    }
    if (now_s() > deadline) {
      throw std::runtime_error(std::string(what) + " timed out");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

Fence::Fence(int nranks, int rank, double timeout_s)
    : nranks_(nranks), rank_(rank), timeout_s_(timeout_s) {
  if (nranks < 1 || rank < 0 || rank >= nranks) {
    throw std::invalid_argument("bad rank / nranks");
  }
}

Fence::Fence(const std::string& unique_id, int nranks, int rank,
             double timeout_s)
    : Fence(nranks, rank, timeout_s) {
  connect(unique_id);
}

void Fence::connect(const std::string& unique_id) {
  if (unique_id.size() != sizeof(ncclUniqueId)) {
    throw std::invalid_argument("unique id must be 128 bytes");
  }
  if (comm_ || stream_) throw std::runtime_error("fence already connected");
  try {
    init(unique_id);
  } catch (...) {
    abort();     // a half-built communicator is never finalized
    destroy();   // frees the stream and buffers created so far
    throw;
  }
}

void Fence::init(const std::string& unique_id) {
  TraceRange range("kiosk.fence.init");
  const int nranks = nranks_, rank = rank_;
  const double timeout_s = timeout_s_;
  // every HIP call of this thread goes to the worker's device: with all
  // managed GPUs visible (WORKER_PIN=visible) that is not ordinal 0, and
  // the HIP current device is per thread (the node agent's is not the
  // thread that opened the device)
  if (const char* dev = std::getenv("KIOSK_DEVICE")) {
    check_hip(hipSetDevice(std::atoi(dev)), "fence hipSetDevice");
  }
  // the library in use now (rccl_use_library); kept for this
  // communicator's whole life, whatever later generations load
  api_ = &rccl();
  const RcclApi& api = *api_;
  check_hip(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking),
            "fence stream");
  check_hip(hipMalloc(reinterpret_cast<void**>(&dev_), 128 * sizeof(long long)),
            "fence buffers");
  check_hip(hipHostMalloc(reinterpret_cast<void**>(&host_),
                          64 * sizeof(long long)),
            "fence pinned");
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), sizeof(id.internal));
  ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
  config.blocking = 0;   // init must be abortable on timeout
  // (channel count: NCCL_MAX_NCHANNELS, set by the worker -- the config's
  // maxCTAs leaves RCCL's 128 channels and their ~670 MB allocated)
  config.commName = "kiosk-fence";
  ncclComm_t comm = nullptr;
  check_nccl(api.CommInitRankConfig(&comm, nranks, id, rank, &config),
             "ncclCommInitRankConfig", api_);
  comm_ = comm;
  wait_ready(comm_, timeout_s, "ncclCommInitRank");
}

Fence::~Fence() {
  try {
    destroy();
  } catch (...) {
  }
}

std::pair<std::vector<long long>, double> Fence::allreduce(
    const std::vector<long long>& values) {
  if (!comm_) throw std::runtime_error("fence communicator is closed");
  if (values.empty() || values.size() > 64) {
    throw std::invalid_argument("fence vector must have 1..64 entries");
  }
  if (stalled_) {
    throw std::runtime_error("fence has an interrupted all-reduce queued: "
                             "shrink or destroy it");
  }
  TraceRange range("kiosk.fence.allreduce");
  const size_t n = values.size();
  const double t0 = now_s();
  std::memcpy(host_, values.data(), n * sizeof(long long));
  check_hip(hipMemcpyAsync(dev_, host_, n * sizeof(long long),
                           hipMemcpyHostToDevice, stream_),
            "fence upload");
  try {
    check_nccl(api_->AllReduce(dev_, dev_ + 64, n, ncclInt64, ncclSum,
                                static_cast<ncclComm_t>(comm_), stream_),
               "ncclAllReduce", api_);
    wait_ready(comm_, timeout_s_, "ncclAllReduce enqueue");
  } catch (...) {
    abort();     // a communicator whose collective failed is never reused
    throw;
  }
  check_hip(hipMemcpyAsync(host_, dev_ + 64, n * sizeof(long long),
                           hipMemcpyDeviceToHost, stream_),
            "fence download");
  // bounded wait: a dead peer must not hang the worker forever
  const double deadline = now_s() + timeout_s_;
  while (hipStreamQuery(stream_) == hipErrorNotReady) {
    if (interrupt_requested_.exchange(false, std::memory_order_relaxed)) {
      // the manager shrinks the dead rank out: keep the communicator (the
      // kernel still waits on the peer; NCCL_SHRINK_ABORT ends it)
      stalled_ = true;
      throw FenceInterrupted("fence all-reduce interrupted for a shrink");
    }
    const bool late = now_s() > deadline;
    if (late || abort_requested_.load(std::memory_order_relaxed)) {
      abort();   // unblocks the kernel waiting on a dead peer
      throw std::runtime_error(late ? "fence all-reduce timed out"
                                    : "fence all-reduce aborted on request");
    }
    std::this_thread::yield();
  }
  check_hip(hipStreamSynchronize(stream_), "fence sync");
  std::vector<long long> out(host_, host_ + n);
  return {out, (now_s() - t0) * 1e6};
}

void Fence::shrink(const std::vector<int>& excluded, double timeout_s,
                   bool abort_parent) {
  if (!comm_) throw std::runtime_error("fence communicator is closed");
  if (!api_->CommShrink) {
    throw std::runtime_error("this RCCL has no ncclCommShrink");
  }
  std::vector<bool> gone(nranks_, false);
  for (int r : excluded) {
    if (r < 0 || r >= nranks_ || gone[r] || r == rank_) {
      throw std::invalid_argument("shrink: bad excluded rank list");
    }
    gone[r] = true;
  }
  TraceRange range("kiosk.fence.shrink");
  std::vector<int> ex(excluded);
  ncclComm_t next = nullptr;
  const int flags = abort_parent ? NCCL_SHRINK_ABORT : NCCL_SHRINK_DEFAULT;
  ncclResult_t res = api_->CommShrink(static_cast<ncclComm_t>(comm_),
                                       ex.data(), static_cast<int>(ex.size()),
                                       &next, nullptr, flags);
  if (res != ncclSuccess && res != ncclInProgress) {
    // the parent is unusable either way: a half-failed shrink is never
    // retried on it
    abort();
    throw std::runtime_error(std::string("ncclCommShrink: ") +
                             api_->GetErrorString(res));
  }
  try {
    wait_ready(next, timeout_s, "ncclCommShrink");
    if (stalled_) {
      // the interrupted all-reduce was terminated by NCCL_SHRINK_ABORT:
      // its stream work (kernel + download) must drain before the stream
      // and buffers serve the child
      const double deadline = now_s() + timeout_s;
      while (hipStreamQuery(stream_) == hipErrorNotReady) {
        if (now_s() > deadline) {
          throw std::runtime_error("interrupted all-reduce did not drain "
                                   "after ncclCommShrink");
        }
        std::this_thread::yield();
      }
    }
  } catch (...) {
    if (next) api_->CommAbort(next);   // the child is ours to abort
    abort();
    throw;
  }
  void* old = comm_;
  comm_ = next;
  stalled_ = false;
  interrupt_requested_.store(false, std::memory_order_relaxed);
  int below = 0;
  for (int r : excluded) below += (r < rank_);
  rank_ -= below;
  nranks_ -= static_cast<int>(excluded.size());
  if (abort_parent) {
    api_->CommAbort(static_cast<ncclComm_t>(old));   // a peer is gone
  } else {
    api_->CommDestroy(static_cast<ncclComm_t>(old));
  }
}

void Fence::request_interrupt() {
  interrupt_requested_.store(true, std::memory_order_relaxed);
}

void Fence::abort() {
  void* comm = comm_;
  comm_ = nullptr;   // cleared first: nothing can reach a freed communicator
  if (comm) api_->CommAbort(static_cast<ncclComm_t>(comm));
}

void Fence::request_abort() {
  abort_requested_.store(true, std::memory_order_relaxed);
}

void Fence::destroy() {
  if (comm_) {
    bool finalized = false;
    if (!abort_requested_.load(std::memory_order_relaxed) && !stalled_) {
      api_->CommFinalize(static_cast<ncclComm_t>(comm_));
      try {
        wait_ready(comm_, timeout_s_, "ncclCommFinalize");
        finalized = true;
      } catch (...) {
      }
    }
    if (finalized) {
      void* comm = comm_;
      comm_ = nullptr;
      api_->CommDestroy(static_cast<ncclComm_t>(comm));
    } else {
      abort();   // a peer is gone: finalize would wait on it
    }
  }
  // teardown: nothing useful to do with an error here
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    (void)hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
  if (dev_) {
    (void)hipFree(dev_);
    dev_ = nullptr;
  }
  if (host_) {
    (void)hipHostFree(host_);
    host_ = nullptr;
  }
}

}  // namespace kiosk

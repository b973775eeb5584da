// Host-only, multi-process stand-in for the HIP runtime calls and the RCCL
// entry points csrc/runtime/fence.cpp uses.  It lets the REAL fence code --
// Fence, RcclNodeTransport, the node agent -- run unchanged in N CPU
// processes (tools/build_native.py --fake-hip builds `_kiosk_fence_cpu`
// against this library; KIOSK_RCCL_LIB points the fence's dlopen at it),
// and under ASan / UBSan / TSan (tests/native/fence_asan_main.cpp).
//
// Semantics kept from RCCL, since they are what fence.cpp must handle:
// * the communicator is non-blocking: init / shrink / finalize report
//   ncclInProgress through ncclCommGetAsyncError until every rank joined;
// * ncclAllReduce only enqueues; the sum lands when the stream is queried
//   after every rank posted (a ShmComm in a file under FAKE_RCCL_DIR or
//   /dev/shm carries the values between processes);
// * a dead peer is NOT detected: a collective waiting on it stays pending
//   until the caller times out or aborts (ncclCommAbort drops this rank's
//   queued work, which is what unblocks the real kernel);
// * ncclCommShrink(NCCL_SHRINK_ABORT) terminates the parent's queued work
//   and builds a child over the survivors, renumbered in order.
// Every communicator and stream is a heap object: a second abort, a
// destroy after an abort, or any use after either is an ASan report.
//
// FAKE_RCCL_MODE (read at each call): ok | init_error | init_hang |
// allreduce_hang | finalize_hang.
//
// FAKE_RCCL_FAIL_MULTIRANK_FROM=<substring>: a communicator of more than one
// rank fails its init when THIS copy of the library was loaded from a path
// containing the substring (dladdr) -- a slim RCCL copy broken only for
// multi-rank P2P, so the node must move on to the stock library
// (gpumgr/nodecomm.py's library ladder), not to shared memory.
//
// What grows with the rank count on a real node (bootstrap all-gathers, IPC
// handle exchange, topology search) is modelled by FAKE_RCCL_INIT_PER_RANK_MS:
// every init settles no sooner than nranks x that after it started, so an
// 8-rank CPU rehearsal builds slower generations than a 1-rank one.  With
// NCCL_DEBUG=INFO and NCCL_DEBUG_FILE (``%h`` / ``%p`` expanded) the fake
// writes the INFO lines the node agent parses from the real library
// (parallel/rccl_info.py): ``Init COMPLETE`` with a bus id, ``Init timings``,
// the graph ``Pattern`` line and, at a communicator's first all-reduce (RCCL
// connects lazily), one ``Channel`` line per ring peer, ``via`` the
// transport named by FAKE_RCCL_TRANSPORT (default P2P/IPC).
//
// The device hold measured on MI355X (profiles/r4_collision) is modelled
// too: a process-wide "HIP runtime lock" that RCCL holds while its fat
// binary registers -- the first ncclGetUniqueId of the process, for
// FAKE_RCCL_LOAD_MS -- and while its code object loads -- the first
// communicator's init, for FAKE_RCCL_INIT_MS, on RCCL's init thread (the
// init stays ncclInProgress until then).  fake_hip_launch_kernel() takes
// that lock like hipLaunchKernel does; fake_hip_graph_launch() does not,
// like hipGraphLaunch.  The CPU mock engine launches through them, so an
// 8-process CPU test sees exactly the collision a real worker would.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>

#include <dlfcn.h>
#include <strings.h>
#include <unistd.h>

#include "runtime/shmcomm.hpp"

#define FAKE_API extern "C" __attribute__((visibility("default")))

namespace {

std::string mode() {
  const char* m = std::getenv("FAKE_RCCL_MODE");
  return m ? m : "ok";
}

struct FakeComm {
  std::unique_ptr<kiosk::ShmComm> shm;
  int rank = 0;
  int nranks = 1;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  std::chrono::steady_clock::time_point ready_at = t0;   // per-rank cost
  long load_ms = 0;            // its code-object load (first comm only)
  bool logged_init = false;
  bool logged_channels = false;
  int polls_left = 3;        // ncclInProgress this many times, then settle
  std::atomic<bool> loading{false};   // its code-object load holds the lock
  bool init_fails = false;
  bool init_hangs = false;
  bool finalize_hangs = false;
  bool finalizing = false;
};

struct Op {
  bool copy = true;
  void* dst = nullptr;
  const void* src = nullptr;
  size_t bytes = 0;
  FakeComm* comm = nullptr;   // all-reduce
  int count = 0;
  uint64_t seq = 0;
  bool posted = false;
  bool hang = false;
};

struct FakeStream {
  std::deque<Op> ops;
};

std::mutex g_mu;                       // streams, their queues, comm lifetime
std::set<FakeStream*> g_streams;
std::atomic<long> g_live_comms{0};

// the modelled HIP runtime lock (see the file comment)
std::mutex g_runtime_lock;
std::once_flag g_load_once;
std::atomic<bool> g_kernels_loaded{false};
std::atomic<int> g_loading_comms{0};   // comms whose code-object load runs

long env_ms(const char* name) {
  const char* v = std::getenv(name);
  return v ? std::atol(v) : 0;
}

std::string busid(int rank) {
  char buf[16];
  std::snprintf(buf, sizeof(buf), "%x", 0x10000 * (rank + 1));
  return buf;
}

// One INFO line to NCCL_DEBUG_FILE, in RCCL's format.
void fake_log(const std::string& text) {
  const char* level = std::getenv("NCCL_DEBUG");
  const char* pattern = std::getenv("NCCL_DEBUG_FILE");
  if (!level || !pattern || strcasecmp(level, "INFO") != 0) return;
  char host[64] = {0};
  gethostname(host, sizeof(host) - 1);
  if (char* dot = std::strchr(host, '.')) *dot = '\0';   // RCCL's %h
  std::string path;
  for (const char* p = pattern; *p; ++p) {
    if (p[0] == '%' && p[1] == 'h') {
      path += host;
      ++p;
    } else if (p[0] == '%' && p[1] == 'p') {
      path += std::to_string(getpid());
      ++p;
    } else {
      path += *p;
    }
  }
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  if (FILE* f = std::fopen(path.c_str(), "a")) {
    std::fprintf(f, "%s:%d:%d [0] NCCL INFO %s\n", host, getpid(),
                 static_cast<int>(gettid()), text.c_str());
    std::fclose(f);
  }
}

void log_init_complete(FakeComm* c) {
  using namespace std::chrono;
  const double total =
      duration<double>(steady_clock::now() - c->t0).count();
  const double kernels = c->load_ms / 1e3;
  char line[512];
  std::snprintf(line, sizeof(line),
                "ncclCommInitRankConfig_impl comm %p rank %d nranks %d "
                "cudaDev 0 nvmlDev 0 busId %s commId 0x%llx - Init COMPLETE",
                static_cast<void*>(c), c->rank, c->nranks,
                busid(c->rank).c_str(),
                static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(c)));
  fake_log(line);
  std::snprintf(line, sizeof(line),
                "Pattern 4, crossNic 0, nChannels 1, bw 40.000000/40.000000, "
                "type XGMI/PIX, sameChannels 1");
  fake_log(line);
  std::snprintf(line, sizeof(line),
                "Init timings - ncclCommInitRankConfig_impl: rank %d nranks %d "
                "total %.2f (kernels %.2f, alloc 0.00, bootstrap %.2f, "
                "allgathers 0.00, topo 0.00, graphs 0.00, connections 0.00, "
                "rest 0.00)",
                c->rank, c->nranks, total, kernels,
                std::max(0.0, total - kernels));
  fake_log(line);
}

void log_channels(FakeComm* c) {
  if (c->nranks < 2) return;
  const char* via = std::getenv("FAKE_RCCL_TRANSPORT");
  const int peer = (c->rank + 1) % c->nranks;
  char line[256];
  std::snprintf(line, sizeof(line), "Channel 00/0 : %d[%s] -> %d[%s] via %s",
                c->rank, busid(c->rank).c_str(), peer, busid(peer).c_str(),
                via && *via ? via : "P2P/IPC");
  fake_log(line);
}

void hold_runtime_lock(long ms) {
  if (ms <= 0) return;
  std::lock_guard<std::mutex> lock(g_runtime_lock);
  std::this_thread::sleep_for(std::chrono::milliseconds(ms));
}

// Runs the stream's queue in order as far as it can (g_mu held).  An
// all-reduce posts its send buffer when it reaches the front (stream
// order: after the upload copy) and completes once every rank posted.
bool progress(FakeStream* s) {
  while (!s->ops.empty()) {
    Op& op = s->ops.front();
    if (op.copy) {
      std::memcpy(op.dst, op.src, op.bytes);
      s->ops.pop_front();
      continue;
    }
    if (op.hang) return false;
    if (!op.posted) {
      op.seq = op.comm->shm->post(static_cast<const long long*>(op.src),
                                  op.count);
      op.posted = true;
    }
    if (!op.comm->shm->try_complete(op.seq, static_cast<long long*>(op.dst),
                                    op.count)) {
      return false;
    }
    s->ops.pop_front();
  }
  return true;
}

void drop_ops_of(FakeComm* c) {
  for (FakeStream* s : g_streams) {
    for (auto it = s->ops.begin(); it != s->ops.end();) {
      it = (!it->copy && it->comm == c) ? s->ops.erase(it) : std::next(it);
    }
  }
}

// this copy of the library was loaded from a path naming `needle`
bool loaded_from(const char* needle) {
  if (!needle || !*needle) return false;
  Dl_info info;
  if (!dladdr(reinterpret_cast<void*>(&loaded_from), &info) ||
      !info.dli_fname) {
    return false;
  }
  return std::strstr(info.dli_fname, needle) != nullptr;
}

thread_local int t_device = 0;

FakeComm* new_comm(std::unique_ptr<kiosk::ShmComm> shm) {
  auto* c = new FakeComm();
  c->shm = std::move(shm);
  const std::string m = mode();
  // init_error_while:<path>: inits fail while that file exists (a test
  // lets RCCL recover after the node fell back to shared memory)
  static const std::string kWhile = "init_error_while:";
  c->init_fails =
      m == "init_error" ||
      (m.compare(0, kWhile.size(), kWhile) == 0 &&
       access(m.c_str() + kWhile.size(), F_OK) == 0);
  c->init_hangs = m == "init_hang";
  c->finalize_hangs = m == "finalize_hang";
  g_live_comms++;
  return c;
}

}  // namespace

FAKE_API long fake_rccl_live_comms() { return g_live_comms.load(); }

// hipLaunchKernel: waits while RCCL holds the runtime lock
FAKE_API void fake_hip_launch_kernel() {
  std::lock_guard<std::mutex> lock(g_runtime_lock);
}
// hipGraphLaunch: never does
FAKE_API void fake_hip_graph_launch() {}

// ---- HIP (host memory stands in for HBM) ---------------------------------
// per-thread current device, like HIP's (only recorded: there is one "GPU")
FAKE_API hipError_t hipSetDevice(int device) {
  if (device < 0) return hipErrorInvalidDevice;
  t_device = device;
  return hipSuccess;
}
FAKE_API hipError_t hipGetDevice(int* device) {
  *device = t_device;
  return hipSuccess;
}
FAKE_API int fake_hip_current_device() { return t_device; }
FAKE_API hipError_t hipStreamCreateWithFlags(hipStream_t* stream,
                                             unsigned int) {
  auto* s = new FakeStream();
  std::lock_guard<std::mutex> lock(g_mu);
  g_streams.insert(s);
  *stream = reinterpret_cast<hipStream_t>(s);
  return hipSuccess;
}
FAKE_API hipError_t hipStreamDestroy(hipStream_t stream) {
  auto* s = reinterpret_cast<FakeStream*>(stream);
  std::lock_guard<std::mutex> lock(g_mu);
  g_streams.erase(s);
  delete s;
  return hipSuccess;
}
FAKE_API hipError_t hipMalloc(void** ptr, size_t size) {
  *ptr = std::calloc(1, size);
  return *ptr ? hipSuccess : hipErrorOutOfMemory;
}
FAKE_API hipError_t hipFree(void* ptr) {
  std::free(ptr);
  return hipSuccess;
}
FAKE_API hipError_t hipHostMalloc(void** ptr, size_t size, unsigned int) {
  *ptr = std::calloc(1, size);
  return *ptr ? hipSuccess : hipErrorOutOfMemory;
}
FAKE_API hipError_t hipHostFree(void* ptr) {
  std::free(ptr);
  return hipSuccess;
}
FAKE_API hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes,
                                   hipMemcpyKind, hipStream_t stream) {
  auto* s = reinterpret_cast<FakeStream*>(stream);
  std::lock_guard<std::mutex> lock(g_mu);
  if (s->ops.empty()) {
    std::memcpy(dst, src, bytes);
  } else {
    Op op;
    op.dst = dst;
    op.src = src;
    op.bytes = bytes;
    s->ops.push_back(op);
  }
  return hipSuccess;
}
FAKE_API hipError_t hipStreamQuery(hipStream_t stream) {
  std::lock_guard<std::mutex> lock(g_mu);
  return progress(reinterpret_cast<FakeStream*>(stream)) ? hipSuccess
                                                         : hipErrorNotReady;
}
FAKE_API hipError_t hipStreamSynchronize(hipStream_t stream) {
  const auto deadline =
      std::chrono::steady_clock::now() + std::chrono::seconds(10);
  while (true) {
    {
      std::lock_guard<std::mutex> lock(g_mu);
      if (progress(reinterpret_cast<FakeStream*>(stream))) return hipSuccess;
    }
    if (std::chrono::steady_clock::now() > deadline) return hipErrorUnknown;
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}
FAKE_API const char* hipGetErrorString(hipError_t) {
  return "fake hip error";
}

// ---- RCCL -------------------------------------------------------------------
FAKE_API ncclResult_t ncclGetVersion(int* version) {
  *version = 22707;
  return ncclSuccess;
}
FAKE_API ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  // the library's first use: its fat binary registers under the lock
  std::call_once(g_load_once,
                 [] { hold_runtime_lock(env_ms("FAKE_RCCL_LOAD_MS")); });
  const char* dir = std::getenv("FAKE_RCCL_DIR");
  const std::string path = kiosk::shm_unique_id(dir ? dir : "");
  std::memset(id->internal, 0, sizeof(id->internal));
  std::memcpy(id->internal, path.data(), path.size());
  return ncclSuccess;
}
FAKE_API ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks,
                                             ncclUniqueId id, int rank,
                                             ncclConfig_t*) {
  std::string path(id.internal, strnlen(id.internal, sizeof(id.internal)));
  std::unique_ptr<kiosk::ShmComm> shm;
  try {
    // like RCCL: no dead-peer detection, a 1 h bound the caller never hits
    shm.reset(new kiosk::ShmComm(path, nranks, rank, 3600.0, false));
  } catch (const std::exception&) {
    return ncclInvalidArgument;
  }
  std::call_once(g_load_once,
                 [] { hold_runtime_lock(env_ms("FAKE_RCCL_LOAD_MS")); });
  FakeComm* c = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    c = new_comm(std::move(shm));
    c->rank = rank;
    c->nranks = nranks;
    if (nranks > 1 && loaded_from(std::getenv("FAKE_RCCL_FAIL_MULTIRANK_FROM")))
      c->init_fails = true;
    c->ready_at = c->t0 + std::chrono::milliseconds(
                              env_ms("FAKE_RCCL_INIT_PER_RANK_MS") * nranks);
  }
  *comm = reinterpret_cast<ncclComm_t>(c);
  const long load_ms = env_ms("FAKE_RCCL_INIT_MS");
  if (load_ms > 0 && !g_kernels_loaded.exchange(true)) {
    // the first communicator of the process loads RCCL's code object on
    // RCCL's init thread, holding the runtime lock; the init settles after
    c->load_ms = load_ms;
    c->loading = true;
    g_loading_comms++;
    std::thread([c, load_ms] {
      hold_runtime_lock(load_ms);
      c->loading = false;
      g_loading_comms--;
    }).detach();
  }
  return ncclInProgress;
}
FAKE_API ncclResult_t ncclCommGetAsyncError(ncclComm_t comm,
                                            ncclResult_t* state) {
  auto* c = reinterpret_cast<FakeComm*>(comm);
  std::lock_guard<std::mutex> lock(g_mu);
  if (c->finalizing) {
    *state = c->finalize_hangs ? ncclInProgress : ncclSuccess;
  } else if (c->init_hangs || c->loading) {
    *state = ncclInProgress;
  } else if (c->polls_left > 0) {
    c->polls_left--;
    *state = ncclInProgress;
  } else if (c->init_fails) {
    *state = ncclInvalidUsage;
  } else if (std::chrono::steady_clock::now() < c->ready_at) {
    *state = ncclInProgress;     // bootstrap cost, growing with nranks
  } else {
    *state = c->shm->poll_ready() ? ncclSuccess : ncclInProgress;
    if (*state == ncclSuccess && !c->logged_init) {
      c->logged_init = true;
      log_init_complete(c);
    }
  }
  return ncclSuccess;
}
FAKE_API ncclResult_t ncclCommAbort(ncclComm_t comm) {
  auto* c = reinterpret_cast<FakeComm*>(comm);
  // like RCCL, an abort waits for the init thread it interrupts
  while (c->loading) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  std::lock_guard<std::mutex> lock(g_mu);
  drop_ops_of(c);                  // what unblocks the real kernel
  g_live_comms--;
  delete c;                        // a second abort is a double free
  return ncclSuccess;
}
FAKE_API ncclResult_t ncclCommFinalize(ncclComm_t comm) {
  std::lock_guard<std::mutex> lock(g_mu);
  reinterpret_cast<FakeComm*>(comm)->finalizing = true;
  return ncclInProgress;
}
FAKE_API ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  auto* c = reinterpret_cast<FakeComm*>(comm);
  while (c->loading) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  std::lock_guard<std::mutex> lock(g_mu);
  drop_ops_of(c);
  g_live_comms--;
  delete c;
  return ncclSuccess;
}
FAKE_API ncclResult_t ncclAllReduce(const void* send, void* recv,
                                    size_t count, ncclDataType_t,
                                    ncclRedOp_t, ncclComm_t comm,
                                    hipStream_t stream) {
  auto* c = reinterpret_cast<FakeComm*>(comm);
  auto* s = reinterpret_cast<FakeStream*>(stream);
  if (count < 1 || count > static_cast<size_t>(kiosk::kShmMaxValues)) {
    return ncclInvalidArgument;
  }
  Op op;
  op.copy = false;
  op.comm = c;
  op.src = send;
  op.dst = recv;
  op.count = static_cast<int>(count);
  op.hang = mode() == "allreduce_hang";   // a peer that never joins
  std::lock_guard<std::mutex> lock(g_mu);
  if (!c->logged_channels) {
    c->logged_channels = true;    // RCCL connects at the first collective
    log_channels(c);
  }
  c->polls_left = 0;
  s->ops.push_back(op);
  progress(s);
  return ncclSuccess;
}
FAKE_API const char* ncclGetErrorString(ncclResult_t) {
  return "fake rccl error";
}
FAKE_API ncclResult_t ncclCommShrink(ncclComm_t comm, int* excluded,
                                     int count, ncclComm_t* out,
                                     ncclConfig_t*, int flags) {
  auto* c = reinterpret_cast<FakeComm*>(comm);
  std::lock_guard<std::mutex> lock(g_mu);
  if (flags & NCCL_SHRINK_ABORT) drop_ops_of(c);
  std::unique_ptr<kiosk::ShmComm> child;
  try {
    child = c->shm->shrink(std::vector<int>(excluded, excluded + count));
  } catch (const std::exception&) {
    return ncclInvalidArgument;
  }
  FakeComm* next = new_comm(std::move(child));
  int below = 0;
  for (int i = 0; i < count; ++i) below += excluded[i] < c->rank;
  next->rank = c->rank - below;
  next->nranks = c->nranks - count;
  next->logged_init = true;      // a shrink logs no init of its own
  *out = reinterpret_cast<ncclComm_t>(next);
  return ncclInProgress;
}

// Host-only stand-ins for the HIP runtime calls and the RCCL entry points
// that csrc/runtime/fence.cpp uses, so the fence's failure handling (init
// errors and timeouts, aborts requested from another thread, finalize on a
// dead peer) can run under AddressSanitizer + UBSan on a CPU.  Every
// communicator is a heap object that abort / destroy delete: a second
// abort, a destroy after an abort, or any use after either is a
// heap-use-after-free / double-free that ASan reports.
//
// FAKE_RCCL_MODE: ok | init_error | init_hang | allreduce_hang |
// finalize_hang (read at each call).
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>

namespace {

struct FakeComm {
  int nranks = 1;
  int polls_left = 3;        // ncclInProgress this many times, then settle
  bool init_fails = false;
  bool init_hangs = false;
  bool finalize_hangs = false;
  bool finalizing = false;
};

std::string mode() {
  const char* m = std::getenv("FAKE_RCCL_MODE");
  return m ? m : "ok";
}

std::atomic<int> g_pending_kernels{0};   // an all-reduce that never ends
std::atomic<long> g_live_comms{0};

}  // namespace

extern "C" {

long fake_rccl_live_comms() { return g_live_comms.load(); }

// ---- HIP (host memory stands in for HBM) ---------------------------------
hipError_t hipStreamCreateWithFlags(hipStream_t* stream, unsigned int) {
  *stream = reinterpret_cast<hipStream_t>(new int(1));
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t stream) {
  delete reinterpret_cast<int*>(stream);
  return hipSuccess;
}
hipError_t hipMalloc(void** ptr, size_t size) {
  *ptr = std::calloc(1, size);
  return *ptr ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* ptr) {
  std::free(ptr);
  return hipSuccess;
}
hipError_t hipHostMalloc(void** ptr, size_t size, unsigned int) {
  *ptr = std::calloc(1, size);
  return *ptr ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void* ptr) {
  std::free(ptr);
  return hipSuccess;
}
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes,
                          hipMemcpyKind, hipStream_t) {
  std::memcpy(dst, src, bytes);
  return hipSuccess;
}
hipError_t hipStreamQuery(hipStream_t) {
  return g_pending_kernels.load() ? hipErrorNotReady : hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "fake hip error"; }

// ---- RCCL -------------------------------------------------------------------
ncclResult_t ncclGetVersion(int* version) {
  *version = 22707;
  return ncclSuccess;
}
ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id->internal, 7, sizeof(id->internal));
  return ncclSuccess;
}
ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks,
                                    ncclUniqueId, int, ncclConfig_t*) {
  auto* c = new FakeComm();
  c->nranks = nranks;
  const std::string m = mode();
  c->init_fails = m == "init_error";
  c->init_hangs = m == "init_hang";
  c->finalize_hangs = m == "finalize_hang";
  g_live_comms++;
  *comm = reinterpret_cast<ncclComm_t>(c);
  return ncclInProgress;
}
ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* state) {
  auto* c = reinterpret_cast<FakeComm*>(comm);
  if (c->finalizing && c->finalize_hangs) {
    *state = ncclInProgress;
  } else if (c->init_hangs) {
    *state = ncclInProgress;
  } else if (c->polls_left > 0) {
    c->polls_left--;
    *state = ncclInProgress;
  } else {
    *state = c->init_fails ? ncclInvalidUsage : ncclSuccess;
  }
  return ncclSuccess;
}
ncclResult_t ncclCommAbort(ncclComm_t comm) {
  auto* c = reinterpret_cast<FakeComm*>(comm);
  g_pending_kernels.store(0);
  g_live_comms--;
  delete c;                        // a second abort is a double free
  return ncclSuccess;
}
ncclResult_t ncclCommFinalize(ncclComm_t comm) {
  reinterpret_cast<FakeComm*>(comm)->finalizing = true;
  return ncclInProgress;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  g_live_comms--;
  delete reinterpret_cast<FakeComm*>(comm);
  return ncclSuccess;
}
ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count,
                           ncclDataType_t, ncclRedOp_t, ncclComm_t comm,
                           hipStream_t) {
  auto* c = reinterpret_cast<FakeComm*>(comm);
  c->polls_left = 0;
  if (mode() == "allreduce_hang") {
    g_pending_kernels.store(1);     // a peer never joins
    return ncclSuccess;
  }
  std::memcpy(recv, send, count * sizeof(long long));
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t) { return "fake rccl error"; }
ncclResult_t ncclCommShrink(ncclComm_t comm, int*, int, ncclComm_t* out,
                            ncclConfig_t*, int) {
  (void)comm;
  auto* c = new FakeComm();
  g_live_comms++;
  *out = reinterpret_cast<ncclComm_t>(c);
  return ncclInProgress;
}

}  // extern "C"

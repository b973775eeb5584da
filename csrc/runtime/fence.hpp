// RCCL membership fence.  RCCL is dlopen'ed, not linked:
// PyTorch-ROCm ships an older RCCL without ncclCommShrink and loads it into
// every process that imports torch; binding our own symbols through an
// RTLD_LOCAL handle of ROCm's RCCL 2.27 keeps the two apart while sharing
// the one HIP runtime.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace kiosk {

struct RcclApi;
const RcclApi& rccl();            // throws if no usable RCCL is found
std::string rccl_library();       // path new communicators use
// Make `path` the library new communicators use (loading it beside any
// other already loaded); "" = the default (KIOSK_RCCL_LIB, then ROCm's).
// Returns the path in use.  Communicators built earlier keep theirs.
std::string rccl_use_library(const std::string& path);
std::vector<std::string> rccl_loaded_libraries();
int rccl_version();
bool rccl_can_shrink();
std::string rccl_unique_id();     // 128 raw bytes
// One-time RCCL initialisation off the critical path (standby boot):
// loads the library, builds and destroys a 1-rank communicator on the
// current device (RCCL device code + proxy setup), returns elapsed ms.
double rccl_warmup(double timeout_s);
// The per-process one-time costs of RCCL, paid by the node agent when the
// process starts (not by its first generation): dlopen (the fat binary's
// registration, ~1.1 s of CPU, far more from a cold page cache) and the
// library init of ncclGetUniqueId.  No communicator, no device memory.
// Returns elapsed ms.
double rccl_preload();
// dlopen + symbol binding only -- no HIP call, no RCCL call: safe in a
// process that never touches the GPU and forks (the worker zygote).
// Returns elapsed ms.
double rccl_dlopen();

// A blocked collective given up on request_interrupt(): the communicator
// is NOT aborted, so the survivors can still shrink it (a peer died).
struct FenceInterrupted : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Fence {
 public:
  // Collective: every rank calls it with the same id and nranks.
  Fence(const std::string& unique_id, int nranks, int rank, double timeout_s);
  // Two-phase form: the object exists (so another thread can
  // request_abort() it) before the collective connect() blocks.
  Fence(int nranks, int rank, double timeout_s);
  void connect(const std::string& unique_id);
  ~Fence();
  Fence(const Fence&) = delete;
  Fence& operator=(const Fence&) = delete;

  // Sum-all-reduce of small int64 vectors (the 72-B membership vector).
  // Returns the result and the host-observed latency in microseconds.
  std::pair<std::vector<long long>, double> allreduce(
      const std::vector<long long>& values);
  // Collective over the surviving ranks: drop `excluded` (old rank ids).
  // `abort_parent` (NCCL_SHRINK_ABORT): first terminate what the parent
  // still runs -- an all-reduce blocked on the dead peer -- then shrink;
  // the parent is aborted, not finalized (a peer is gone).
  void shrink(const std::vector<int>& excluded, double timeout_s,
              bool abort_parent = true);
  void destroy();
  // Owner thread only: aborts the communicator once (idempotent).
  void abort();
  // Any thread: makes a blocked allreduce/init/finalize of the owner
  // thread abort and throw at its next poll (a peer died mid-collective).
  void request_abort();
  bool abort_requested() const { return abort_requested_.load(); }
  // Any thread: a blocked allreduce of the owner thread throws
  // FenceInterrupted at its next poll and leaves the communicator intact
  // for shrink() (the manager is excluding a dead rank).
  void request_interrupt();
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }
  // Owner thread: the bound of later collectives / shrinks (a first
  // generation connects under a longer one than its all-reduces use).
  void set_timeout(double timeout_s) { timeout_s_ = timeout_s; }
  double timeout() const { return timeout_s_; }

 private:
  void wait_ready(void* comm, double timeout_s, const char* what);
  void init(const std::string& unique_id);   // constructor body

  const RcclApi* api_ = nullptr;  // the library this communicator uses
  void* comm_ = nullptr;        // ncclComm_t
  hipStream_t stream_ = nullptr;
  long long* dev_ = nullptr;    // send [64] + recv [64]
  long long* host_ = nullptr;   // pinned [64]
  int nranks_ = 0;
  int rank_ = 0;
  double timeout_s_ = 60.0;
  std::atomic<bool> abort_requested_{false};
  std::atomic<bool> interrupt_requested_{false};
  bool stalled_ = false;        // an interrupted op may still be queued
};

}  // namespace kiosk

// Node-local host shared-memory communicator (the transport of
// the node membership fence when the standbys hold no GPU).
//
// The fence is a 72-byte agreement between processes on ONE node.  With
// WARM_POOL_MODE=device every slot's process already owns a HIP context, a
// hardware queue and an RCCL communicator, and the fence runs over RCCL /
// xGMI.  In the modes that hold no GPU (context / import standbys, deep
// idle) an RCCL communicator would cost ~0.8 GiB of HBM per GPU just to
// agree on 9 integers; this communicator does the same sum-all-reduce
// through a mmap'ed file under /dev/shm instead: no device state, a few
// microseconds per fence, and -- unlike RCCL -- it notices a peer process
// that died (kill(pid, 0)) instead of waiting out its timeout.
//
// Protocol: every rank owns one cache-line-aligned slot with a sequence
// number and two value buffers (double-buffered by sequence parity).  Op k
// writes buffer k&1, publishes seq = k (release), waits until every rank's
// seq >= k (acquire) and sums.  A rank posts op k+1 only after it finished
// reading op k, so buffer k&1 is never overwritten while a peer reads it.
//
// The same object is non-blocking where RCCL is (join / poll_ready, post /
// try_complete): tests/native/fake_hip_rccl.cpp builds its multi-process
// RCCL stand-in on it.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace kiosk {

constexpr int kShmMaxRanks = 64;
constexpr int kShmMaxValues = 64;

// A fresh communicator id (a path; the file appears when the first rank
// joins).  `dir` "" = $KIOSK_SHM_DIR or /dev/shm.
std::string shm_unique_id(const std::string& dir = "");

class ShmComm {
 public:
  // Joins (non-blocking): maps the segment and claims `rank`.  Throws on a
  // rank claimed twice or an nranks mismatch.
  ShmComm(const std::string& id, int nranks, int rank, double timeout_s,
          bool detect_dead_peers = true);
  ~ShmComm();
  ShmComm(const ShmComm&) = delete;
  ShmComm& operator=(const ShmComm&) = delete;

  bool poll_ready();                 // every rank joined
  void wait_ready();                 // bounded; throws on timeout / abort
  // Blocking sum-all-reduce (bounded by the timeout, abortable).
  std::vector<long long> allreduce(const std::vector<long long>& values);
  // Split form: post() publishes this rank's values for the next op,
  // try_complete() sums into `out` once every rank posted it.
  uint64_t post(const long long* values, int n);
  bool try_complete(uint64_t seq, long long* out, int n);
  // Collective over the survivors: a communicator of the ranks not in
  // `excluded` (old rank ids), renumbered in order.  Non-blocking join of
  // the child; wait_ready() on it.
  std::unique_ptr<ShmComm> shrink(const std::vector<int>& excluded);
  // Any thread: a blocked wait throws at its next poll.
  void request_abort() { abort_.store(true, std::memory_order_relaxed); }
  bool abort_requested() const {
    return abort_.load(std::memory_order_relaxed);
  }
  void close();

  int nranks() const { return nranks_; }
  int rank() const { return rank_; }
  const std::string& id() const { return id_; }

 private:
  struct Segment;
  void check_peers(uint64_t seq, const char* what);
  void wait_until(const char* what, bool (ShmComm::*done)(uint64_t),
                  uint64_t arg);
  bool joined_all(uint64_t);
  bool posted_all(uint64_t seq);
  void unlink_once();

  std::string id_;
  int nranks_ = 0;
  int rank_ = 0;
  double timeout_s_ = 30.0;
  bool detect_dead_ = true;
  Segment* seg_ = nullptr;
  int fd_ = -1;
  uint64_t seq_ = 0;
  int shrinks_ = 0;
  std::atomic<bool> abort_{false};
};

}  // namespace kiosk

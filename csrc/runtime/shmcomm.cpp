// Node-local host shared-memory communicator (see shmcomm.hpp).
#include "shmcomm.hpp"

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <thread>

namespace kiosk {

namespace {

constexpr uint32_t kMagic = 0x6b736d31;   // "ksm1"

double now_s() {
  return std::chrono::duration<double>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct alignas(64) Slot {
  std::atomic<uint64_t> seq;     // last op this rank posted
  std::atomic<int32_t> pid;      // 0 = not joined, -1 = left, else owner
  std::atomic<int32_t> joined;
  long long vals[2][kShmMaxValues];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free,
              "shared-memory atomics must be lock-free");
static_assert(std::atomic<int32_t>::is_always_lock_free,
              "shared-memory atomics must be lock-free");

}  // namespace

struct ShmComm::Segment {
  std::atomic<uint32_t> magic;
  std::atomic<int32_t> nranks;
  std::atomic<int32_t> joined;
  std::atomic<int32_t> unlinked;
  Slot slots[kShmMaxRanks];
};

std::string shm_unique_id(const std::string& dir) {
  static std::atomic<unsigned> counter{0};
  std::string base = dir;
  if (base.empty()) {
    const char* env = std::getenv("KIOSK_SHM_DIR");
    base = env && *env ? env : "/dev/shm";
    struct stat st;
    if (stat(base.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) base = "/tmp";
  }
  std::random_device rd;
  char name[96];
  std::snprintf(name, sizeof(name), "/kiosk-shm-%d-%u-%08x%08x",
                static_cast<int>(getpid()), counter.fetch_add(1),
                static_cast<unsigned>(rd()), static_cast<unsigned>(rd()));
  std::string id = base + name;
  if (id.size() >= 120) throw std::invalid_argument("shm dir path too long");
  return id;
}

ShmComm::ShmComm(const std::string& id, int nranks, int rank,
                 double timeout_s, bool detect_dead_peers)
    : id_(id), nranks_(nranks), rank_(rank), timeout_s_(timeout_s),
      detect_dead_(detect_dead_peers) {
  if (nranks < 1 || nranks > kShmMaxRanks || rank < 0 || rank >= nranks) {
    throw std::invalid_argument("shm comm: bad rank / nranks");
  }
  fd_ = ::open(id.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
  if (fd_ < 0) {
    throw std::runtime_error("shm comm: open " + id + ": " +
                             std::strerror(errno));
  }
  struct stat st;
  if (fstat(fd_, &st) != 0 ||
      (static_cast<size_t>(st.st_size) < sizeof(Segment) &&
       ftruncate(fd_, sizeof(Segment)) != 0)) {
    const int err = errno;
    ::close(fd_);
    fd_ = -1;
    throw std::runtime_error(std::string("shm comm: size: ") +
                             std::strerror(err));
  }
  void* p = mmap(nullptr, sizeof(Segment), PROT_READ | PROT_WRITE, MAP_SHARED,
                 fd_, 0);
  if (p == MAP_FAILED) {
    const int err = errno;
    ::close(fd_);
    fd_ = -1;
    throw std::runtime_error(std::string("shm comm: mmap: ") +
                             std::strerror(err));
  }
  seg_ = static_cast<Segment*>(p);
  uint32_t magic = 0;
  seg_->magic.compare_exchange_strong(magic, kMagic);
  int32_t expect = 0;
  if (!seg_->nranks.compare_exchange_strong(expect, nranks) &&
      expect != nranks) {
    close();
    throw std::runtime_error("shm comm: nranks mismatch");
  }
  Slot& mine = seg_->slots[rank];
  if (mine.joined.exchange(1) != 0) {
    seg_ = nullptr;   // the slot is someone else's: leave it untouched
    munmap(p, sizeof(Segment));
    ::close(fd_);
    fd_ = -1;
    throw std::runtime_error("shm comm: rank " + std::to_string(rank) +
                             " joined twice");
  }
  mine.pid.store(static_cast<int32_t>(getpid()), std::memory_order_relaxed);
  seq_ = mine.seq.load(std::memory_order_relaxed);
  seg_->joined.fetch_add(1, std::memory_order_acq_rel);
}

ShmComm::~ShmComm() { close(); }

void ShmComm::unlink_once() {
  if (seg_ && seg_->unlinked.exchange(1) == 0) ::unlink(id_.c_str());
}

void ShmComm::close() {
  if (!seg_) return;
  // peers still waiting on this rank see it leave (and fail fast)
  seg_->slots[rank_].pid.store(-1, std::memory_order_release);
  unlink_once();   // a generation that never completed leaves no file
  munmap(seg_, sizeof(Segment));
  seg_ = nullptr;
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

bool ShmComm::joined_all(uint64_t) {
  return seg_->joined.load(std::memory_order_acquire) >= nranks_;
}

bool ShmComm::posted_all(uint64_t seq) {
  for (int r = 0; r < nranks_; ++r) {
    if (seg_->slots[r].seq.load(std::memory_order_acquire) < seq) return false;
  }
  return true;
}

bool ShmComm::poll_ready() {
  if (!seg_) throw std::runtime_error("shm comm is closed");
  if (!joined_all(0)) return false;
  unlink_once();
  return true;
}

// Fails fast on a peer that left or whose process is gone (only for ranks
// the wait still depends on: seq below the target / not joined).
void ShmComm::check_peers(uint64_t seq, const char* what) {
  for (int r = 0; r < nranks_; ++r) {
    if (r == rank_) continue;
    Slot& s = seg_->slots[r];
    if (seq && s.seq.load(std::memory_order_acquire) >= seq) continue;
    const int32_t pid = s.pid.load(std::memory_order_acquire);
    if (pid == -1) {
      throw std::runtime_error(std::string(what) + ": peer rank " +
                               std::to_string(r) + " left");
    }
    if (detect_dead_ && pid > 0 && ::kill(pid, 0) != 0 && errno == ESRCH) {
      throw std::runtime_error(std::string(what) + ": peer rank " +
                               std::to_string(r) + " (pid " +
                               std::to_string(pid) + ") died");
    }
  }
}

void ShmComm::wait_until(const char* what, bool (ShmComm::*done)(uint64_t),
                         uint64_t arg) {
  const double t0 = now_s();
  const double deadline = t0 + timeout_s_;
  double next_check = t0 + 0.002;
  for (unsigned spin = 0;; ++spin) {
    if ((this->*done)(arg)) return;
    if (abort_.load(std::memory_order_relaxed)) {
      throw std::runtime_error(std::string(what) + " aborted on request");
    }
    if (spin < 256) {
      continue;                           // the common case: peers are close
    }
    const double t = now_s();
    if (t > deadline) {
      throw std::runtime_error(std::string(what) + " timed out");
    }
    if (t > next_check) {
      check_peers(arg, what);
      next_check = t + 0.005;
    }
    if (spin < 4096) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
}

void ShmComm::wait_ready() {
  if (!seg_) throw std::runtime_error("shm comm is closed");
  wait_until("shm comm init", &ShmComm::joined_all, 0);
  unlink_once();
}

uint64_t ShmComm::post(const long long* values, int n) {
  if (!seg_) throw std::runtime_error("shm comm is closed");
  if (n < 1 || n > kShmMaxValues) {
    throw std::invalid_argument("shm all-reduce: 1..64 values");
  }
  const uint64_t seq = ++seq_;
  Slot& mine = seg_->slots[rank_];
  std::memcpy(mine.vals[seq & 1], values, n * sizeof(long long));
  mine.seq.store(seq, std::memory_order_release);
  return seq;
}

bool ShmComm::try_complete(uint64_t seq, long long* out, int n) {
  if (!seg_) throw std::runtime_error("shm comm is closed");
  if (!posted_all(seq)) return false;
  for (int i = 0; i < n; ++i) out[i] = 0;
  for (int r = 0; r < nranks_; ++r) {
    const long long* v = seg_->slots[r].vals[seq & 1];
    for (int i = 0; i < n; ++i) out[i] += v[i];
  }
  return true;
}

std::vector<long long> ShmComm::allreduce(
    const std::vector<long long>& values) {
  const int n = static_cast<int>(values.size());
  const uint64_t seq = post(values.data(), n);
  wait_until("shm all-reduce", &ShmComm::posted_all, seq);
  std::vector<long long> out(n);
  try_complete(seq, out.data(), n);
  return out;
}

std::unique_ptr<ShmComm> ShmComm::shrink(const std::vector<int>& excluded) {
  if (!seg_) throw std::runtime_error("shm comm is closed");
  std::vector<bool> gone(nranks_, false);
  for (int r : excluded) {
    if (r < 0 || r >= nranks_ || gone[r]) {
      throw std::invalid_argument("shm shrink: bad excluded rank list");
    }
    gone[r] = true;
  }
  if (gone[rank_]) throw std::invalid_argument("shm shrink: self excluded");
  int below = 0;
  for (int r = 0; r < rank_; ++r) below += gone[r];
  const int n = nranks_ - static_cast<int>(excluded.size());
  // every survivor derives the same child id from its shrink count
  const std::string child = id_ + ".s" + std::to_string(++shrinks_);
  return std::unique_ptr<ShmComm>(
      new ShmComm(child, n, rank_ - below, timeout_s_, detect_dead_));
}

}  // namespace kiosk

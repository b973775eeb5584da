// Host-side sanitizer test of csrc/runtime/fence.cpp: its failure paths
// (init errors and timeouts, aborts requested from another thread, a peer
// that dies mid-all-reduce, shrink with NCCL_SHRINK_ABORT, a stuck
// finalize) with REAL multi-rank communicators -- each rank is a thread
// with its own Fence, the fake RCCL (csrc/fakes/fake_hip_rccl.cpp) carries
// the values through shared memory.  Built with -fsanitize=address,undefined
// or -fsanitize=thread by tests/test_fence_native_asan.py; prints one line
// per check, any sanitizer report fails the run.
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fence.hpp"

extern "C" long fake_rccl_live_comms();

namespace kiosk {
// engine.cpp's helper (the fence only needs it for HIP calls)
void check_hip(hipError_t err, const char* what) {
  if (err != hipSuccess) throw std::runtime_error(what);
}
}  // namespace kiosk

namespace {

std::atomic<int> failures{0};

void expect(bool ok, const char* what) {
  std::printf("%s %s\n", ok ? "ok" : "FAIL", what);
  std::fflush(stdout);
  if (!ok) ++failures;
}

std::string uid() { return kiosk::rccl_unique_id(); }

bool contains(const std::exception& e, const char* what) {
  return std::string(e.what()).find(what) != std::string::npos;
}

using Vec = std::vector<long long>;

// Connect `n` ranks of one communicator, one thread each; returns them.
std::vector<std::unique_ptr<kiosk::Fence>> connect_all(int n, double timeout) {
  const std::string id = uid();
  std::vector<std::unique_ptr<kiosk::Fence>> out(n);
  for (int r = 0; r < n; ++r) out[r].reset(new kiosk::Fence(n, r, timeout));
  std::vector<std::thread> threads;
  for (int r = 0; r < n; ++r) {
    threads.emplace_back([&out, &id, r] { out[r]->connect(id); });
  }
  for (auto& t : threads) t.join();
  return out;
}

// Each listed rank runs `fn(rank)` on its own thread.
void each(const std::vector<int>& ranks, const std::function<void(int)>& fn) {
  std::vector<std::thread> threads;
  for (int r : ranks) threads.emplace_back([&fn, r] { fn(r); });
  for (auto& t : threads) t.join();
}

}  // namespace

int main() {
  // 1. the good path: 2 ranks, two all-reduces, destroy (finalize + destroy)
  setenv("FAKE_RCCL_MODE", "ok", 1);
  {
    auto f = connect_all(2, 5.0);
    std::vector<Vec> got(2);
    each({0, 1}, [&](int r) {
      got[r] = f[r]->allreduce({3, r == 0, r == 1}).first;
      got[r] = f[r]->allreduce({4, 1, r}).first;
    });
    expect(got[0] == Vec({8, 2, 1}) && got[1] == got[0],
           "two-rank all-reduce sums");
    each({0, 1}, [&](int r) {
      f[r]->destroy();
      f[r]->destroy();                            // idempotent
    });
  }
  expect(fake_rccl_live_comms() == 0, "good path frees its communicators");

  // 2. init fails asynchronously: the constructor aborts exactly once
  setenv("FAKE_RCCL_MODE", "init_error", 1);
  try {
    kiosk::Fence f(uid(), 2, 1, 5.0);
    expect(false, "init error raises");
  } catch (const std::runtime_error& e) {
    expect(contains(e, "failed"), "init error raises");
  }
  expect(fake_rccl_live_comms() == 0, "failed init leaves nothing live");

  // 3. init times out (the peer never joins); the destructor runs after
  setenv("FAKE_RCCL_MODE", "ok", 1);
  try {
    kiosk::Fence f(uid(), 2, 0, 0.2);
    expect(false, "init timeout raises");
  } catch (const std::runtime_error& e) {
    expect(contains(e, "timed out"), "init timeout raises");
  }
  expect(fake_rccl_live_comms() == 0, "timed-out init leaves nothing live");

  // 4. two-phase: an abort requested before connect() aborts the init
  {
    kiosk::Fence f(2, 0, 30.0);
    f.request_abort();
    try {
      f.connect(uid());
      expect(false, "requested abort ends connect");
    } catch (const std::runtime_error& e) {
      expect(contains(e, "aborted"), "requested abort ends connect");
    }
    f.destroy();
  }
  expect(fake_rccl_live_comms() == 0, "aborted connect leaves nothing live");

  // 5. the peer dies (aborts locally) before the all-reduce: rank 0 blocks,
  //    another thread asks for the abort; then destroy must not finalize or
  //    abort again
  {
    auto f = connect_all(2, 30.0);
    f[1]->abort();                                // the dead peer
    std::thread killer([&f] {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      f[0]->request_abort();
    });
    const auto t0 = std::chrono::steady_clock::now();
    try {
      f[0]->allreduce({1, 1});
      expect(false, "blocked all-reduce aborts");
    } catch (const std::runtime_error& e) {
      const double s = std::chrono::duration<double>(
                           std::chrono::steady_clock::now() - t0).count();
      expect(s < 5.0 && contains(e, "aborted"),
             "blocked all-reduce aborts on request");
    }
    killer.join();
    f[0]->destroy();
    f[1]->destroy();
    try {
      f[0]->allreduce({1});
      expect(false, "closed fence refuses");
    } catch (const std::runtime_error&) {
      expect(true, "closed fence refuses");
    }
  }
  expect(fake_rccl_live_comms() == 0, "aborted all-reduce frees once");

  // 6. all-reduce on a dead peer times out by itself (no abort request)
  {
    auto f = connect_all(2, 0.2);
    f[1]->abort();
    try {
      f[0]->allreduce({1, 1});
      expect(false, "all-reduce timeout raises");
    } catch (const std::runtime_error& e) {
      expect(contains(e, "timed out"), "all-reduce timeout raises");
    }
  }                                               // destructors: no 2nd abort
  expect(fake_rccl_live_comms() == 0, "timed-out all-reduce frees once");

  // 7. an all-reduce the fake never completes (allreduce_hang)
  {
    auto f = connect_all(1, 0.2);
    setenv("FAKE_RCCL_MODE", "allreduce_hang", 1);
    try {
      f[0]->allreduce({1});
      expect(false, "hung all-reduce times out");
    } catch (const std::runtime_error& e) {
      expect(contains(e, "timed out"), "hung all-reduce times out");
    }
    setenv("FAKE_RCCL_MODE", "ok", 1);
  }
  expect(fake_rccl_live_comms() == 0, "hung all-reduce frees once");

  // 8. finalize that never completes (a peer is gone): destroy aborts
  {
    auto f = connect_all(2, 0.2);
    each({0, 1}, [&](int r) { f[r]->allreduce({1, 1}); });
    setenv("FAKE_RCCL_MODE", "finalize_hang", 1);
    f[0]->destroy();
    f[1]->destroy();
    setenv("FAKE_RCCL_MODE", "ok", 1);
  }
  expect(fake_rccl_live_comms() == 0, "stuck finalize is aborted once");

  // 9. a rank dies MID all-reduce: the survivors' blocked all-reduce is
  //    interrupted (not aborted), they shrink it out with NCCL_SHRINK_ABORT
  //    and keep fencing over the child communicator
  {
    auto f = connect_all(4, 10.0);
    f[2]->abort();                                // rank 2 is gone
    std::atomic<int> interrupted{0};
    std::thread manager([&f, &interrupted] {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      for (int r : {0, 1, 3}) f[r]->request_interrupt();
      (void)interrupted;
    });
    std::vector<Vec> got(4);
    each({0, 1, 3}, [&](int r) {
      try {
        f[r]->allreduce({1, r});
      } catch (const kiosk::FenceInterrupted&) {
        interrupted++;
      }
    });
    manager.join();
    expect(interrupted.load() == 3, "blocked all-reduce interrupted");
    try {
      f[0]->allreduce({1});
      expect(false, "interrupted fence refuses until shrunk");
    } catch (const std::runtime_error& e) {
      expect(contains(e, "interrupted"),
             "interrupted fence refuses until shrunk");
    }
    each({0, 1, 3}, [&](int r) {
      f[r]->shrink({2}, 5.0, true);
      got[r] = f[r]->allreduce({5, 1 << f[r]->rank()}).first;
    });
    expect(f[3]->rank() == 2 && f[3]->nranks() == 3 && f[0]->rank() == 0,
           "shrink renumbers the survivors");
    expect(got[0] == Vec({15, 7}) && got[1] == got[0] && got[3] == got[0],
           "survivors fence over the shrunk communicator");
    each({0, 1, 3}, [&](int r) { f[r]->destroy(); });
    f[2]->destroy();
  }
  expect(fake_rccl_live_comms() == 0, "shrink frees parent and child once");

  // 10. a live rank retires between fences: graceful shrink, twice
  {
    auto f = connect_all(3, 5.0);
    f[1]->destroy();                              // retired process
    each({0, 2}, [&](int r) { f[r]->shrink({1}, 5.0, true); });
    f[2]->destroy();                              // and another
    f[0]->shrink({1}, 5.0, true);
    auto solo = f[0]->allreduce({9, 1}).first;
    expect(solo == Vec({9, 1}) && f[0]->nranks() == 1,
           "repeated shrink down to one rank");
    f[0]->destroy();
  }
  expect(fake_rccl_live_comms() == 0, "repeated shrink frees everything");

  std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "PASSED",
              failures.load());
  return failures ? 1 : 0;
}

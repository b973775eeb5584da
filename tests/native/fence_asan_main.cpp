// Host-side sanitizer test of csrc/runtime/fence.cpp (the
// init-timeout / failed-enqueue paths used to abort a communicator and then
// finalize or abort it again).  Built with -fsanitize=address,undefined
// against fake_hip_rccl.cpp (KIOSK_RCCL_LIB points the fence's dlopen at
// the same fake), run by tests/test_fence_native_asan.py.  Prints one line
// per scenario; any ASan / UBSan report fails the run.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
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

int failures = 0;

void expect(bool ok, const char* what) {
  std::printf("%s %s\n", ok ? "ok" : "FAIL", what);
  if (!ok) ++failures;
}

std::string uid() { return kiosk::rccl_unique_id(); }

}  // namespace

int main() {
  // 1. the good path: init, two all-reduces, destroy (finalize + destroy)
  setenv("FAKE_RCCL_MODE", "ok", 1);
  {
    kiosk::Fence f(uid(), 1, 0, 5.0);
    auto r = f.allreduce({3, 0, 1});
    expect(r.first == std::vector<long long>({3, 0, 1}), "allreduce result");
    f.allreduce({4, 1, 0});
    f.destroy();
    f.destroy();                                  // idempotent
  }
  expect(fake_rccl_live_comms() == 0, "good path frees its communicator");

  // 2. init fails asynchronously: the constructor aborts exactly once
  setenv("FAKE_RCCL_MODE", "init_error", 1);
  try {
    kiosk::Fence f(uid(), 2, 1, 5.0);
    expect(false, "init error raises");
  } catch (const std::runtime_error& e) {
    expect(std::string(e.what()).find("failed") != std::string::npos,
           "init error raises");
  }
  expect(fake_rccl_live_comms() == 0, "failed init leaves nothing live");

  // 3. init times out (a peer died mid-init); the destructor runs after
  setenv("FAKE_RCCL_MODE", "init_hang", 1);
  try {
    kiosk::Fence f(uid(), 2, 0, 0.2);
    expect(false, "init timeout raises");
  } catch (const std::runtime_error& e) {
    expect(std::string(e.what()).find("timed out") != std::string::npos,
           "init timeout raises");
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
      expect(std::string(e.what()).find("aborted") != std::string::npos,
             "requested abort ends connect");
    }
    f.destroy();
  }
  expect(fake_rccl_live_comms() == 0, "aborted connect leaves nothing live");

  // 5. an all-reduce blocked on a dead peer, aborted from another thread;
  //    then destroy (which must not finalize or abort again)
  setenv("FAKE_RCCL_MODE", "ok", 1);
  {
    kiosk::Fence f(uid(), 2, 0, 30.0);
    setenv("FAKE_RCCL_MODE", "allreduce_hang", 1);
    std::thread killer([&f] {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      f.request_abort();
    });
    const auto t0 = std::chrono::steady_clock::now();
    try {
      f.allreduce({1, 1});
      expect(false, "blocked all-reduce aborts");
    } catch (const std::runtime_error& e) {
      const double s = std::chrono::duration<double>(
                           std::chrono::steady_clock::now() - t0).count();
      expect(s < 5.0 && std::string(e.what()).find("aborted") !=
                            std::string::npos,
             "blocked all-reduce aborts on request");
    }
    killer.join();
    f.destroy();
    try {
      f.allreduce({1});
      expect(false, "closed fence refuses");
    } catch (const std::runtime_error&) {
      expect(true, "closed fence refuses");
    }
  }
  expect(fake_rccl_live_comms() == 0, "aborted all-reduce frees once");

  // 6. all-reduce times out by itself (no abort request)
  setenv("FAKE_RCCL_MODE", "ok", 1);
  {
    kiosk::Fence f(uid(), 2, 0, 0.2);
    setenv("FAKE_RCCL_MODE", "allreduce_hang", 1);
    try {
      f.allreduce({1, 1});
      expect(false, "all-reduce timeout raises");
    } catch (const std::runtime_error& e) {
      expect(std::string(e.what()).find("timed out") != std::string::npos,
             "all-reduce timeout raises");
    }
  }                                               // destructor: no 2nd abort
  expect(fake_rccl_live_comms() == 0, "timed-out all-reduce frees once");

  // 7. finalize that never completes (a peer is gone): destroy aborts
  setenv("FAKE_RCCL_MODE", "finalize_hang", 1);
  {
    kiosk::Fence f(uid(), 2, 0, 0.2);
    f.allreduce({1, 1});
    f.destroy();
  }
  expect(fake_rccl_live_comms() == 0, "stuck finalize is aborted once");

  std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "PASSED",
              failures);
  return failures ? 1 : 0;
}

// dlopen'ed roctx (see trace.hpp).
#include "trace.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace kiosk {
namespace {

struct RoctxApi {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
};

const RoctxApi& api() {
  static RoctxApi table;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* off = std::getenv("KIOSK_ROCTX");
    if (off && std::strcmp(off, "0") == 0) return;
    // rocprofiler-sdk's roctx first (what rocprofv3 --marker-trace hooks),
    // then the legacy roctracer one
    const char* names[] = {"librocprofiler-sdk-roctx.so.1",
                           "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                           "libroctx64.so.4"};
    for (const char* name : names) {
      void* h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      RoctxApi t;
      t.push = reinterpret_cast<int (*)(const char*)>(
          dlsym(h, "roctxRangePushA"));
      t.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      t.mark = reinterpret_cast<void (*)(const char*)>(
          dlsym(h, "roctxMarkA"));
      if (t.push && t.pop) {
        table = t;
        return;
      }
      dlclose(h);
    }
  });
  return table;
}

}  // namespace

bool roctx_available() { return api().push != nullptr; }

void roctx_push(const char* name) {
  if (auto f = api().push) f(name);
}

void roctx_pop() {
  if (auto f = api().pop) f();
}

void roctx_mark(const char* name) {
  if (auto f = api().mark) f(name);
}

}  // namespace kiosk

// roctx ranges around the worker's GPU stages: warm-start,
// graph capture, inference, fence.  `rocprofv3 --marker-trace` shows them
// next to the kernel trace.  The roctx library is dlopen'ed on first use
// (never linked), so a box without it -- or KIOSK_ROCTX=0 -- costs one
// failed lookup and every call is a no-op.
#pragma once

namespace kiosk {

bool roctx_available();
void roctx_push(const char* name);
void roctx_pop();
void roctx_mark(const char* name);

// RAII range: push on construction, pop on scope exit (exceptions too).
class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctx_push(name); }
  ~TraceRange() { roctx_pop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace kiosk

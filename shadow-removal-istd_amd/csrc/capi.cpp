// Error reporting and version for the C-ABI (include/stcgan_hip.h).
#include <cstdarg>
#include <cstdio>
#include <string>

#include <hip/hip_runtime.h>

#include "../../include/stcgan_hip.h"

namespace stc {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code == 0 ? -1 : code;
}

// One-shot, thread-local instrumentation of the next main kernel launched by this thread
// (stc_time_next_main_kernel): the events bracket that kernel alone, not the split-K / split-pixel
// reduction a call may enqueue after it.  Thread-local like the error message, so concurrent
// callers on other threads are unaffected.
struct MainTimer {
  hipEvent_t begin = nullptr, end = nullptr;
};
static thread_local MainTimer g_main_timer;

void main_timer_begin(hipStream_t st) {
  if (g_main_timer.begin) (void)hipEventRecord(g_main_timer.begin, st);
}
void main_timer_end(hipStream_t st) {
  if (g_main_timer.end) (void)hipEventRecord(g_main_timer.end, st);
  g_main_timer.begin = nullptr;
  g_main_timer.end = nullptr;
}

}  // namespace stc

extern "C" int stc_time_next_main_kernel(void* ev_begin, void* ev_end) {
  if ((ev_begin == nullptr) != (ev_end == nullptr)) return stc::fail(-1, "stc_time_next_main_kernel: give both events or none");
  stc::g_main_timer.begin = (hipEvent_t)ev_begin;
  stc::g_main_timer.end = (hipEvent_t)ev_end;
  return 0;
}

extern "C" const char* stc_last_error(void) { return stc::g_last_error.c_str(); }
extern "C" int stc_version(void) { return 1; }

// Stream ordering for the host schedule (engine.wait_stream, the weight-gradient lane's fork): waiter waits for
// everything enqueued so far on src.  One call records a pooled event on src and makes waiter wait for it -- in
// place of a Python-side event (created, recorded, waited and destroyed: ~9 us of host time per fork against
// ~2 here; the train step makes ~70).  The events are never destroyed (a ring of 256 per device and thread: a
// wait already enqueued refers to the record it saw, so re-recording a pooled event later is harmless), so they
// also outlive any HIP graph capture whose edges they form.
namespace {
struct EventRing {
  int device = -1;
  hipEvent_t ev[256] = {};
  unsigned next = 0;
};
thread_local EventRing g_rings[8];
}  // namespace

extern "C" int stc_stream_wait(void* waiter, void* src) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return stc::fail((int)e, "stc_stream_wait: %s", hipGetErrorString(e));
  EventRing* r = nullptr;
  for (auto& c : g_rings)
    if (c.device == dev || c.device < 0) { r = &c; break; }
  if (!r) return stc::fail(-1, "stc_stream_wait: more than 8 devices in one thread");
  r->device = dev;
  hipEvent_t& ev = r->ev[r->next++ & 255u];
  if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess)
    return stc::fail((int)e, "stc_stream_wait: event create: %s", hipGetErrorString(e));
  if ((e = hipEventRecord(ev, (hipStream_t)src)) != hipSuccess)
    return stc::fail((int)e, "stc_stream_wait: record: %s", hipGetErrorString(e));
  if ((e = hipStreamWaitEvent((hipStream_t)waiter, ev, 0)) != hipSuccess)
    return stc::fail((int)e, "stc_stream_wait: wait: %s", hipGetErrorString(e));
  return 0;
}

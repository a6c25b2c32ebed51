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

// Error reporting and version for the C-ABI (include/stcgan_hip.h).
#include <cstdarg>
#include <cstdio>
#include <string>

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

}  // namespace stc

extern "C" const char* stc_last_error(void) { return stc::g_last_error.c_str(); }
extern "C" int stc_version(void) { return 1; }

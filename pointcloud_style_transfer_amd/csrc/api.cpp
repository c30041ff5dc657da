// Library-level entry points: version and thread-local last error.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace pcst {
static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}
}  // namespace pcst

extern "C" const char* pcst_version(void) { return "pcst 0.1.0 gfx950"; }
extern "C" const char* pcst_last_error(void) { return pcst::g_last_error; }

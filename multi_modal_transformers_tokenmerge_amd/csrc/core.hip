// Error plumbing and version of libmmt_hip.
#include <stdarg.h>

#include "common.h"

namespace mmt {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mmt

extern "C" const char* mmt_last_error(void) { return mmt::g_err; }
extern "C" int mmt_version(void) { return 1; }

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
extern "C" int mmt_version(void) { return MMT_API_VERSION; }

extern "C" int64_t mmt_workspace_size(int op, const int64_t* dims, int ndims) {
  switch (op) {
    case MMT_WS_TOME_MATCH:
      if (!dims || ndims != 3 || dims[0] <= 0 || dims[1] < 2 || dims[2] <= 0) {
        mmt::set_error("mmt_workspace_size(TOME_MATCH): dims must be {n, t, c}");
        return MMT_ERR_INVALID;
      }
      return mmt::tome_match_workspace(dims[0], dims[1], dims[2]);
    default:
      mmt::set_error("mmt_workspace_size: unknown op %d", op);
      return MMT_ERR_INVALID;
  }
}

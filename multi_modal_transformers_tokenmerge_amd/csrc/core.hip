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

// Deterministic mode on (fx non-NULL: the fixed-point shadow of the n-float gradient buffer at
// grad, zero-initialised by the caller) or off (fx NULL). Sets every unit's device state
// (synchronous; call outside stream capture).
extern "C" int mmt_set_deterministic(float* grad, long long* fx, int64_t n) {
  MMT_CHECK_ARG(!fx || (grad && n > 0), "mmt_set_deterministic: args");
  const mmt::DetState st{fx ? grad : nullptr, fx, fx ? n : 0};
  if (mmt::det_set_attention(st) || mmt::det_set_glue(st) || mmt::det_set_norm(st) ||
      mmt::det_set_stem(st)) {
    mmt::set_error("mmt_set_deterministic: hipMemcpyToSymbol failed");
    return MMT_ERR_HIP;
  }
  return MMT_OK;
}

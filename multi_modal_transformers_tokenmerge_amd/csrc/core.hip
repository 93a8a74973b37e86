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

// The device status word of common.h "device-side index checks": fault bits OR-ed by kernels,
// read and cleared by mmt_device_status.
__device__ unsigned int g_device_status;

namespace mmt {
unsigned int* fault_word() {
  static unsigned int* const p = [] {
    void* a = nullptr;
    return hipGetSymbolAddress(&a, HIP_SYMBOL(g_device_status)) == hipSuccess ? (unsigned int*)a
                                                                              : nullptr;
  }();
  return p;
}
}  // namespace mmt

extern "C" const char* mmt_last_error(void) { return mmt::g_err; }

extern "C" int mmt_device_status(mmt_stream_t stream) {
  unsigned int* w = mmt::fault_word();
  if (!w) {
    mmt::set_error("mmt_device_status: device status word unavailable (no HIP device)");
    return MMT_ERR_HIP;
  }
  hipStream_t s = mmt::as_stream(stream);
  unsigned int v = 0;
  if (hipMemcpyAsync(&v, w, sizeof v, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    mmt::set_error("mmt_device_status: %s", hipGetErrorString(hipGetLastError()));
    return MMT_ERR_HIP;
  }
  if (v == 0) return MMT_OK;
  if (hipMemsetAsync(w, 0, sizeof v, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
    mmt::set_error("mmt_device_status: clear failed: %s", hipGetErrorString(hipGetLastError()));
    return MMT_ERR_HIP;
  }
  char what[256] = "";
  static const struct { unsigned int bit; const char* name; } names[] = {
      {MMT_FAULT_TOME_INDEX, "ToMe merge: unm/src/dst index out of range"},
      {MMT_FAULT_TOME_PARTITION, "ToMe merge: unm and src do not partition the a half (index repeated)"},
      {MMT_FAULT_POS_MAP, "ToMe unmerge: pos_map entry out of range"},
      {MMT_FAULT_ROW_INDEX, "row gather / scatter: row index out of range"}};
  for (const auto& nm : names)
    if (v & nm.bit) {
      if (what[0]) strncat(what, "; ", sizeof what - strlen(what) - 1);
      strncat(what, nm.name, sizeof what - strlen(what) - 1);
    }
  mmt::set_error("device-side index check failed (status 0x%x): %s; the offending indices were "
                 "replaced by 0, so the outputs of those launches are not meaningful", v, what);
  return MMT_ERR_INVALID;
}
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

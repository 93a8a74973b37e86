// Host-side check of libmmt_hip's C-ABI dispatch under AddressSanitizer (SURVEY §5 "sanitizers";
// built by tests/asan/build_asan.sh with the host half of core.hip / tome.hip / prune.hip
// instrumented, device code not compiled: nothing here launches a kernel). Every argument check
// of the ToMe, pruning and workspace entry points is driven with invalid input — null pointers,
// shapes past the limits, misaligned strides or workspaces, unknown dtypes / ops — and must
// return MMT_ERR_INVALID with a message, never abort or touch memory it was not given; the error
// plumbing (thread-local message, truncation of long messages) and mmt_device_status without a
// GPU are exercised too. Test infrastructure only.
#include <stdio.h>
#include <string.h>

#include "mmt_api.h"

static int g_fails = 0;
#define EXPECT(cond, ...)                                        \
  do {                                                           \
    if (!(cond)) {                                               \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);       \
      fprintf(stderr, __VA_ARGS__);                              \
      fprintf(stderr, "\n");                                     \
      ++g_fails;                                                 \
    }                                                            \
  } while (0)

static void invalid(long long rc, const char* what) {
  EXPECT(rc == MMT_ERR_INVALID, "%s: rc %lld, want MMT_ERR_INVALID", what, rc);
  EXPECT(strlen(mmt_last_error()) > 0, "%s: empty mmt_last_error()", what);
}

int main() {
  EXPECT(mmt_version() == MMT_API_VERSION, "version %d", mmt_version());
  alignas(16) static char buf[1 << 16];  // stands in for device memory: never dereferenced
  void* p = buf;
  int32_t* ip = (int32_t*)buf;
  float* fp = (float*)buf;
  // ---- workspace sizes
  int64_t dims[3] = {4, 256, 64};
  const int64_t ws = mmt_workspace_size(MMT_WS_TOME_MATCH, dims, 3);
  EXPECT(ws > 0 && ws % 256 == 0, "workspace %lld", (long long)ws);
  invalid(mmt_workspace_size(MMT_WS_TOME_MATCH, dims, 2), "workspace ndims");
  invalid(mmt_workspace_size(MMT_WS_TOME_MATCH, nullptr, 3), "workspace null dims");
  invalid(mmt_workspace_size(1234, dims, 3), "workspace unknown op");
  int64_t bad[3] = {4, 1, 64};
  invalid(mmt_workspace_size(MMT_WS_TOME_MATCH, bad, 3), "workspace t < 2");
  // ---- mmt_tome_match (token_compression.py:54-112)
  invalid(mmt_tome_match(nullptr, MMT_F32, 4, 256, 1, 64, 256 * 64, 64, 0, 16, 0, ip, ip, ip,
                         nullptr, p, ws, nullptr), "match null metric");
  invalid(mmt_tome_match(p, MMT_F32, 4, 256, 1, 64, 256 * 64, 64, 0, 16, 0, ip, ip, ip, nullptr,
                         nullptr, ws, nullptr), "match null workspace");
  invalid(mmt_tome_match(p, MMT_F32, 4, 4096, 1, 64, 4096 * 64, 64, 0, 16, 0, ip, ip, ip, nullptr,
                         p, 1LL << 40, nullptr), "match t > 2048");
  invalid(mmt_tome_match(p, MMT_F32, 4, 256, 1, 1024, 256 * 1024, 1024, 0, 16, 0, ip, ip, ip,
                         nullptr, p, 1LL << 40, nullptr), "match c > 512");
  invalid(mmt_tome_match(p, MMT_F32, 4, 256, 1, 64, 256 * 64, 64, 0, 129, 0, ip, ip, ip, nullptr,
                         p, ws, nullptr), "match r > t/2");
  invalid(mmt_tome_match(p, MMT_F32, 4, 256, 1, 64, 256 * 64, 64, 0, 128, MMT_TOME_CLASS_TOKEN, ip,
                         ip, ip, nullptr, p, ws, nullptr), "match r > (t - class)/2");
  invalid(mmt_tome_match(p, MMT_F32, 4, 256, 1, 64, 256 * 64, 64, 0, 0, 0, ip, ip, ip, nullptr, p,
                         ws, nullptr), "match r == 0");
  invalid(mmt_tome_match(p, 7, 4, 256, 1, 64, 256 * 64, 64, 0, 16, 0, ip, ip, ip, nullptr, p, ws,
                         nullptr), "match dtype");
  invalid(mmt_tome_match(p, MMT_F32, 4, 256, 1, 64, 256 * 64, 64, 0, 16, 0, ip, ip, ip, nullptr, p,
                         ws - 1, nullptr), "match workspace too small");
  invalid(mmt_tome_match(p, MMT_F32, 4, 256, 1, 64, 256 * 64, 64, 0, 16, 0, ip, ip, ip, nullptr,
                         buf + 4, ws, nullptr), "match workspace misaligned");
  invalid(mmt_tome_match(p, MMT_F32, -1, 256, 1, 64, 256 * 64, 64, 0, 16, 0, ip, ip, ip, nullptr, p,
                         ws, nullptr), "match n < 0");
  // ---- merge_wavg forward / backward (token_compression.py:90-129)
  invalid(mmt_tome_merge_wavg_fwd(nullptr, MMT_F32, 2, 292, 384, 292 * 384, 384, 32, 256, 16, 0,
                                  nullptr, ip, ip, ip, p, 276 * 384, 384, fp, ip, nullptr),
          "merge null x");
  invalid(mmt_tome_merge_wavg_fwd(p, MMT_F32, 2, 292, 384, 292 * 384, 384, 40, 256, 16, 0, nullptr,
                                  ip, ip, ip, p, 276 * 384, 384, fp, ip, nullptr),
          "merge set past L");
  invalid(mmt_tome_merge_wavg_fwd(p, MMT_F32, 2, 292, 384, 292 * 384, 384, 32, 256, 129, 0,
                                  nullptr, ip, ip, ip, p, 276 * 384, 384, fp, ip, nullptr),
          "merge r > t/2");
  invalid(mmt_tome_merge_wavg_fwd(p, MMT_F32, 2, 292, 382, 292 * 382, 382, 32, 256, 16, 0, nullptr,
                                  ip, ip, ip, p, 276 * 382, 382, fp, ip, nullptr),
          "merge rows not 16-B");
  invalid(mmt_tome_merge_wavg_fwd(p, 3, 2, 292, 384, 292 * 384, 384, 32, 256, 16, 0, nullptr, ip,
                                  ip, ip, p, 276 * 384, 384, fp, ip, nullptr),
          "merge dtype");
  invalid(mmt_tome_merge_wavg_fwd(p, MMT_F32, 2, 292, 384, 292 * 384, 384, 32, 256, 16, 0, nullptr,
                                  nullptr, ip, ip, p, 276 * 384, 384, fp, ip, nullptr),
          "merge null unm with unmerged tokens");
  invalid(mmt_tome_merge_wavg_bwd(p, MMT_F32, 2, 292, 384, 276 * 384, 384, 32, 256, 16, fp, fp,
                                  nullptr, p, 292 * 384, 384, nullptr), "merge bwd null pos_map");
  invalid(mmt_tome_merge_wavg_bwd(p, MMT_BF16, 2, 292, 385, 276 * 385, 385, 32, 256, 16, fp, fp,
                                  ip, p, 292 * 385, 385, nullptr), "merge bwd rows not 16-B");
  invalid(mmt_tome_merge_wavg_bwd(p, MMT_F32, 2, 292, 384, 276 * 384, 384, 100, 256, 16, fp, fp,
                                  ip, p, 292 * 384, 384, nullptr), "merge bwd set past L");
  invalid(mmt_tome_merge_seqnorm_fwd(fp, 2, 600, 384, 600 * 384, 384, 32, 256, 16, 0, nullptr, ip,
                                     ip, ip, fp, 584 * 384, 384, fp, ip, fp, fp, 1e-6f, p,
                                     584 * 384, 384, fp, fp, nullptr), "merge+LN L - r > 512");
  invalid(mmt_tome_merge_seqnorm_fwd(fp, 2, 292, 384, 292 * 384, 384, 32, 256, 16, 0, nullptr, ip,
                                     ip, ip, fp, 276 * 384, 384, fp, ip, nullptr, fp, 1e-6f, p,
                                     276 * 384, 384, fp, fp, nullptr), "merge+LN null gamma");
  // ---- pruning (token_compression.py:15-46, compressed_attention.py:302-308)
  const int32_t starts[2] = {0, 32}, lens[2] = {32, 256}, ks[2] = {32, 200};
  const int32_t lens_bad[2] = {32, 300};
  invalid(mmt_topk_gather(p, MMT_F32, 2, 288, 384, 288 * 384, 384, fp, 288, 0, starts, lens, ks, p,
                          232 * 384, 384, ip, nullptr), "topk no sets");
  invalid(mmt_topk_gather(p, MMT_F32, 2, 288, 384, 288 * 384, 384, fp, 288, 2, starts, lens_bad,
                          ks, p, 232 * 384, 384, ip, nullptr), "topk set past L");
  invalid(mmt_topk_gather(p, MMT_F32, 2, 288, 384, 288 * 384, 384, fp, 288, 2, nullptr, lens, ks,
                          p, 232 * 384, 384, ip, nullptr), "topk null set table");
  invalid(mmt_gather_rows(p, MMT_F32, 2, 288, 384, 288 * 384, 384, nullptr, 4, p, 4 * 384, 384,
                          nullptr), "gather null idx");
  invalid(mmt_gather_rows(p, MMT_BF16, 2, 288, 383, 288 * 383, 383, ip, 4, p, 4 * 383, 383,
                          nullptr), "gather rows not 16-B");
  invalid(mmt_topk_scatter_bwd(p, 9, 2, 4, 384, 4 * 384, 384, ip, 288, p, 288 * 384, 384, nullptr),
          "scatter dtype");
  invalid(mmt_prune_importance(nullptr, 2, 6, 288, fp, nullptr), "importance null");
  // ---- error plumbing: a long message is truncated inside the thread-local buffer
  invalid(mmt_tome_match(p, MMT_F32, 4, 256, 1, 64, 256 * 64, 64, 0, 2000000000, 0, ip, ip, ip,
                         nullptr, p, ws, nullptr), "match huge r");
  EXPECT(strlen(mmt_last_error()) < 512, "error message not bounded");
  // ---- the device status word without a GPU: an error code, never a crash
  const int st = mmt_device_status(nullptr);
  EXPECT(st == MMT_OK || st == MMT_ERR_HIP, "device status rc %d", st);
  printf(g_fails ? "FAILED %d\n" : "OK\n", g_fails);
  return g_fails != 0;
}

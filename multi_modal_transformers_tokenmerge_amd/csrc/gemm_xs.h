// Activation-stationary NT GEMM (csrc/gemm_xs.hip): the launcher mmt_gemm / mmt_gemm_fp8 route to.
#pragma once
#include "common.h"

namespace mmt {

// The epilogue the activation-stationary kernel applies, in epilogue_w's order (gemm.hip):
// v = acc (* sa[m] * sb[n] for fp8) * alpha + bias[n]; relu; dropout (counter RNG pair draws of
// element (drop_row_offset + m) * N + n); + residual[m][n]; stored bf16 or fp32.
struct XsEpi {
  const float* bias = nullptr;
  int relu = 0;
  const uint32_t* rng = nullptr;  // (seed, step) device pair; NULL: no dropout
  uint32_t drop_layer = 0, drop_site = 0, keep_thresh16 = 65536u;
  float drop_scale = 1.f, alpha = 1.f;
  int64_t drop_row_offset = 0;
  const void* residual = nullptr;  // [M][ld_res], fp32 (res_f32) or bf16
  int res_f32 = 0;
  int64_t ld_res = 0;
  const float* sa = nullptr;  // fp8: per-row activation scales [M]
  const float* sb = nullptr;  // fp8: per-channel weight scales [N]
  uint32_t* relu_bits = nullptr;  // bf16: the relu-bit image (include/mmt_api.h layout), N % 256 == 0
};

// Whether the kernel takes a product: K == 384 (bf16) or 768 (fp8 bytes), N % 64 == 0, no
// residual, 16-B aligned rows / operands (bias and channel scales are DMA'd per 64-column chunk,
// so any N); a relu-bit image only for bf16 and N % 256 == 0.
bool xs_shape_ok(int M, int N, int K, bool f8, int64_t lda, int64_t ldb, int64_t ldc, const void* A,
                 const void* B, const void* C, const XsEpi& e);
// C = epi(X . W^T); X [M][lda], W [N][ldb] (elements: bf16, or e4m3 bytes when f8), C [M][ldc]
// bf16 (out_f32 0) or fp32 (1).
int xs_launch(int M, int N, int K, bool f8, const void* X, int64_t lda, const void* W, int64_t ldb,
              void* C, int64_t ldc, int out_f32, const XsEpi& e, hipStream_t stream);

}  // namespace mmt

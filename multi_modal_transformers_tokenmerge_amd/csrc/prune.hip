// Top-k token pruning for gfx950 — reference tokenizers/token_compression.py:15-46
// (compute_top_k_tokens, vmapped over the batch as in :168): per token set (start, num_tokens),
// jax.lax.top_k of the importance scores (descending; equal scores keep the lower index first;
// the float total order of lax.sort, NaN largest), indices shifted by the set start, the sets'
// index lists concatenated in the given order, then a row gather of the embeddings.
//
// One workgroup per (batch row, token set): ranks by counting in LDS (n <= 4096), then the k
// selected rows are copied with 16-byte vector accesses. The backward scatters the output
// gradient rows back (each input row is selected at most once: no atomics) and zeroes the rest.
#include <math.h>

#include "common.h"

using namespace mmt;

namespace {

constexpr int MAX_PSETS = 16;
constexpr int MAX_PN = 4096;
constexpr int PNT = 256;

struct PruneSets {
  int n_sets;
  int start[MAX_PSETS];
  int len[MAX_PSETS];
  int k[MAX_PSETS];
  int out_off[MAX_PSETS];  // first output row of the set
};

__device__ __forceinline__ uint32_t total_key(float v) {  // lax total order, NaN largest
  if (isnan(v)) return 0xffffffffu;
  uint32_t b = __float_as_uint(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

template <typename T>
__global__ __launch_bounds__(PNT) void topk_gather_kernel(const T* __restrict__ x, int D,
                                                          int64_t xs_b, int64_t xs_t,
                                                          const float* __restrict__ scores,
                                                          int64_t ss_b, PruneSets ps,
                                                          T* __restrict__ out, int64_t os_b,
                                                          int64_t os_t,
                                                          int32_t* __restrict__ idx_out, int K) {
  __shared__ uint32_t key[MAX_PN];
  __shared__ int32_t sel[MAX_PN];
  const int b = blockIdx.x, s = blockIdx.y;
  const int start = ps.start[s], n = ps.len[s], k = ps.k[s], off = ps.out_off[s];
  for (int i = threadIdx.x; i < n; i += PNT) key[i] = total_key(scores[(int64_t)b * ss_b + start + i]);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += PNT) {
    const uint32_t ki = key[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const uint32_t kj = key[j];
      rank += (kj > ki) || (kj == ki && j < i);
    }
    if (rank < k) sel[rank] = start + i;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += PNT) idx_out[(int64_t)b * K + off + i] = sel[i];
  constexpr int V = 16 / sizeof(T);
  const int nch = D / V;
  for (int e = threadIdx.x; e < k * nch; e += PNT) {
    const int row = e / nch, ch = e - row * nch;
    *reinterpret_cast<uint4*>(out + (int64_t)b * os_b + (int64_t)(off + row) * os_t + ch * V) =
        *reinterpret_cast<const uint4*>(x + (int64_t)b * xs_b + (int64_t)sel[row] * xs_t + ch * V);
  }
}

// Backward: d_x = 0 everywhere (this kernel), then d_x[b, idx[b, i]] = d_out[b, i] (the next one;
// selected rows are distinct, so plain stores suffice).
template <typename T>
__global__ void topk_zero_kernel(int D, int L, T* __restrict__ dx, int64_t xs_b, int64_t xs_t) {
  constexpr int V = 16 / sizeof(T);
  const int nch = D / V;
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)L * nch) return;
  const int row = e / nch, ch = e - (int64_t)row * nch;
  *reinterpret_cast<uint4*>(dx + (int64_t)b * xs_b + (int64_t)row * xs_t + ch * V) = make_uint4(0, 0, 0, 0);
}

template <typename T>
__global__ void topk_scatter_rows_kernel(const T* __restrict__ dout, int D, int64_t ds_b,
                                         int64_t ds_t, const int32_t* __restrict__ idx, int K,
                                         T* __restrict__ dx, int64_t xs_b, int64_t xs_t, int L,
                                         unsigned int* fault) {
  constexpr int V = 16 / sizeof(T);
  const int nch = D / V;
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)K * nch) return;
  const int i = e / nch, ch = e - (int64_t)i * nch;
  const int row = checked_index(idx[(int64_t)b * K + i], L, fault, MMT_FAULT_ROW_INDEX);
  *reinterpret_cast<uint4*>(dx + (int64_t)b * xs_b + (int64_t)row * xs_t + ch * V) =
      *reinterpret_cast<const uint4*>(dout + (int64_t)b * ds_b + (int64_t)i * ds_t + ch * V);
}

int fill_sets(PruneSets& ps, int n_sets, const int32_t* start, const int32_t* len,
              const int32_t* k, int L, int* K_total) {
  MMT_CHECK_ARG(n_sets >= 1 && n_sets <= MAX_PSETS && start && len && k,
                "mmt_topk: 1..%d token sets", MAX_PSETS);
  ps.n_sets = n_sets;
  int off = 0;
  for (int i = 0; i < n_sets; ++i) {
    MMT_CHECK_ARG(start[i] >= 0 && len[i] >= 1 && start[i] + len[i] <= L && len[i] <= MAX_PN &&
                      k[i] >= 0 && k[i] <= len[i],
                  "mmt_topk: set %d (start %d, len %d, k %d) invalid for L=%d", i, start[i],
                  len[i], k[i], L);
    ps.start[i] = start[i];
    ps.len[i] = len[i];
    ps.k[i] = k[i];
    ps.out_off[i] = off;
    off += k[i];
  }
  *K_total = off;
  return MMT_OK;
}

bool vec_ok(int dtype, int D, int64_t a, int64_t b, int64_t c, int64_t d) {
  const int v = dtype == MMT_F32 ? 4 : 8;
  return D % v == 0 && a % v == 0 && b % v == 0 && c % v == 0 && d % v == 0;
}

}  // namespace

extern "C" int mmt_topk_gather(const void* x, int dtype, int B, int L, int D, int64_t xs_b,
                               int64_t xs_t, const float* scores, int64_t ss_b, int n_sets,
                               const int32_t* set_start, const int32_t* set_len,
                               const int32_t* set_k, void* out, int64_t os_b, int64_t os_t,
                               int32_t* idx_out, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && scores && out && idx_out && B > 0 && L > 0 && D > 0, "mmt_topk_gather: args");
  MMT_CHECK_ARG(dtype == MMT_F32 || dtype == MMT_BF16, "mmt_topk_gather: dtype");
  MMT_CHECK_ARG(vec_ok(dtype, D, xs_b, xs_t, os_b, os_t), "mmt_topk_gather: D/strides not 16-B rows");
  PruneSets ps;
  int K = 0;
  int rc = fill_sets(ps, n_sets, set_start, set_len, set_k, L, &K);
  if (rc) return rc;
  dim3 grid(B, n_sets);
  hipStream_t s = as_stream(stream);
  if (dtype == MMT_F32)
    hipLaunchKernelGGL(topk_gather_kernel<float>, grid, dim3(PNT), 0, s, (const float*)x, D, xs_b,
                       xs_t, scores, ss_b, ps, (float*)out, os_b, os_t, idx_out, K);
  else
    hipLaunchKernelGGL(topk_gather_kernel<bf16_t>, grid, dim3(PNT), 0, s, (const bf16_t*)x, D,
                       xs_b, xs_t, scores, ss_b, ps, (bf16_t*)out, os_b, os_t, idx_out, K);
  MMT_CHECK_LAUNCH("mmt_topk_gather");
  return MMT_OK;
}

extern "C" int mmt_topk_scatter_bwd(const void* dout, int dtype, int B, int K, int D,
                                    int64_t ds_b, int64_t ds_t, const int32_t* idx, int L,
                                    void* dx, int64_t xs_b, int64_t xs_t, mmt_stream_t stream) {
  MMT_CHECK_ARG(dout && idx && dx && B > 0 && K >= 0 && L > 0 && D > 0, "mmt_topk_scatter_bwd: args");
  MMT_CHECK_ARG(dtype == MMT_F32 || dtype == MMT_BF16, "mmt_topk_scatter_bwd: dtype");
  MMT_CHECK_ARG(vec_ok(dtype, D, ds_b, ds_t, xs_b, xs_t), "mmt_topk_scatter_bwd: D/strides");
  const int nch = D / (dtype == MMT_F32 ? 4 : 8);
  hipStream_t s = as_stream(stream);
  const int64_t nz = (int64_t)L * nch, ns = (int64_t)K * nch;
  dim3 gz((nz + 255) / 256, B), gs((ns + 255) / 256 > 0 ? (ns + 255) / 256 : 1, B);
  if (dtype == MMT_F32) {
    hipLaunchKernelGGL(topk_zero_kernel<float>, gz, dim3(256), 0, s, D, L, (float*)dx, xs_b, xs_t);
    if (K > 0)
      hipLaunchKernelGGL(topk_scatter_rows_kernel<float>, gs, dim3(256), 0, s, (const float*)dout,
                         D, ds_b, ds_t, idx, K, (float*)dx, xs_b, xs_t, L, fault_word());
  } else {
    hipLaunchKernelGGL(topk_zero_kernel<bf16_t>, gz, dim3(256), 0, s, D, L, (bf16_t*)dx, xs_b, xs_t);
    if (K > 0)
      hipLaunchKernelGGL(topk_scatter_rows_kernel<bf16_t>, gs, dim3(256), 0, s,
                         (const bf16_t*)dout, D, ds_b, ds_t, idx, K, (bf16_t*)dx, xs_b, xs_t, L,
                         fault_word());
  }
  MMT_CHECK_LAUNCH("mmt_topk_scatter_bwd");
  return MMT_OK;
}

namespace {
template <typename T>
__global__ void gather_rows_kernel(const T* __restrict__ x, int D, int64_t xs_b, int64_t xs_t,
                                   const int32_t* __restrict__ idx, int K, T* __restrict__ out,
                                   int64_t os_b, int64_t os_t, int L, unsigned int* fault) {
  constexpr int V = 16 / sizeof(T);
  const int nch = D / V;
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)K * nch) return;
  const int i = e / nch, ch = e - (int64_t)i * nch;
  const int row = checked_index(idx[(int64_t)b * K + i], L, fault, MMT_FAULT_ROW_INDEX);
  *reinterpret_cast<uint4*>(out + (int64_t)b * os_b + (int64_t)i * os_t + ch * V) =
      *reinterpret_cast<const uint4*>(x + (int64_t)b * xs_b + (int64_t)row * xs_t + ch * V);
}

__global__ void prune_importance_kernel(const float* __restrict__ wsum, int B, int H, int L,
                                        float* __restrict__ scores) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * L) return;
  const int b = (int)(i / L), q = (int)(i - (int64_t)b * L);
  float acc = 0.f;
  // IEEE divisions (the test restates this order exactly: h ascending, / L, then / H)
  for (int h = 0; h < H; ++h) acc += __fdiv_rn(wsum[((int64_t)b * H + h) * L + q], (float)L);
  scores[i] = __fdiv_rn(acc, (float)H);
}
}  // namespace

extern "C" int mmt_prune_importance(const float* wsum, int B, int H, int L, float* scores,
                                    mmt_stream_t stream) {
  MMT_CHECK_ARG(wsum && scores && B > 0 && H > 0 && L > 0, "mmt_prune_importance: args");
  const int64_t n = (int64_t)B * L;
  hipLaunchKernelGGL(prune_importance_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     as_stream(stream), wsum, B, H, L, scores);
  MMT_CHECK_LAUNCH("mmt_prune_importance");
  return MMT_OK;
}

extern "C" int mmt_gather_rows(const void* x, int dtype, int B, int L, int D, int64_t xs_b,
                               int64_t xs_t, const int32_t* idx, int K, void* out, int64_t os_b,
                               int64_t os_t, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && idx && out && B > 0 && L > 0 && D > 0 && K >= 0, "mmt_gather_rows: args");
  MMT_CHECK_ARG(dtype == MMT_F32 || dtype == MMT_BF16, "mmt_gather_rows: dtype");
  MMT_CHECK_ARG(vec_ok(dtype, D, xs_b, xs_t, os_b, os_t), "mmt_gather_rows: D/strides not 16-B rows");
  if (K == 0) return MMT_OK;
  const int64_t ns = (int64_t)K * (D / (dtype == MMT_F32 ? 4 : 8));
  dim3 grid((ns + 255) / 256, B);
  hipStream_t s = as_stream(stream);
  if (dtype == MMT_F32)
    hipLaunchKernelGGL(gather_rows_kernel<float>, grid, dim3(256), 0, s, (const float*)x, D, xs_b,
                       xs_t, idx, K, (float*)out, os_b, os_t, L, fault_word());
  else
    hipLaunchKernelGGL(gather_rows_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, D,
                       xs_b, xs_t, idx, K, (bf16_t*)out, os_b, os_t, L, fault_word());
  MMT_CHECK_LAUNCH("mmt_gather_rows");
  return MMT_OK;
}

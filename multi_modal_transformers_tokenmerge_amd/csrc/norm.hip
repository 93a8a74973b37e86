// Sequence-axis LayerNorm, column reductions and dropout backward for gfx950.
//
// seqnorm: flax.linen.LayerNorm(reduction_axes=[1], feature_axes=[-1]) as configured by the
// reference (model_configs/attention_blocks/vanilla_decoder.yaml:5-13, used twice per block in
// attention.py:58,66): statistics over the SEQUENCE axis per (batch, feature), fast variance
// max(0, E[x^2] - E[x]^2), y = (x - mean) * (rsqrt(var + eps) * scale) + bias.
// x is (B, L, D) token-major, so a column reduction over L: each workgroup owns 64 features of
// one sample; 8 lanes x 16 B cover the 64 columns, 32 row groups stride over L (coalesced 128-B
// row segments), partial sums meet in LDS. The second pass re-reads the 64-column panel (L2-hot).
#include "common.h"

using namespace mmt;

namespace {

constexpr int CW = 64;   // columns per workgroup
constexpr int RG = 32;   // row groups
constexpr int NT = 256;  // = 8 column vectors x RG

__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = __uint_as_float(w[q] << 16);
    f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = (uint32_t)f2bf(f[2 * q]) | ((uint32_t)f2bf(f[2 * q + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Reduce NV per-thread vectors of 8 column partials over the RG row groups (LDS), result for
// column (cv*8 + e) of quantity v in red[v][cv*8+e] after the call (row group 0 slot).
template <int NV>
__device__ __forceinline__ void reduce_rows(float (*part)[8], float* red /*[NV][RG][CW]*/) {
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(v * RG + rg) * CW + cv * 8 + e] = part[v][e];
  __syncthreads();
  for (int i = threadIdx.x; i < NV * CW; i += NT) {
    const int v = i / CW, c = i % CW;
    float s = 0.f;
    for (int r = 0; r < RG; ++r) s += red[(v * RG + r) * CW + c];
    red[(v * RG) * CW + c] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(NT) void seqnorm_fwd_kernel(
    const bf16_t* __restrict__ x, int64_t xs_b, int64_t xs_t, int L, int D,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    bf16_t* __restrict__ y, int64_t ys_b, int64_t ys_t, float* __restrict__ mean_out,
    float* __restrict__ rstd_out) {
  __shared__ float red[2 * RG * CW];
  __shared__ float s_mul[CW], s_add[CW];
  const int b = blockIdx.x, c0 = blockIdx.y * CW;
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = c0 + cv * 8;
  const bool cok = col < D;
  const bf16_t* xb = x + (int64_t)b * xs_b + col;
  float part[2][8] = {};
  if (cok)
    for (int l = rg; l < L; l += RG) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(xb + (int64_t)l * xs_t), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        part[0][e] += f[e];
        part[1][e] += f[e] * f[e];
      }
    }
  reduce_rows<2>(part, red);
  if (threadIdx.x < CW && c0 + threadIdx.x < D) {
    const int c = c0 + threadIdx.x;
    const float mu = red[threadIdx.x] / L;
    const float var = fmaxf(0.f, red[RG * CW + threadIdx.x] / L - mu * mu);
    const float rs = rsqrtf(var + eps);
    const float mul = rs * gamma[c];
    s_mul[threadIdx.x] = mul;
    s_add[threadIdx.x] = beta[c] - mu * mul;  // (x - mu) * mul + beta
    mean_out[(int64_t)b * D + c] = mu;
    rstd_out[(int64_t)b * D + c] = rs;
  }
  __syncthreads();
  if (!cok) return;
  float mul[8], add[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mul[e] = s_mul[cv * 8 + e];
    add[e] = s_add[cv * 8 + e];
  }
  bf16_t* yb = y + (int64_t)b * ys_b + col;
  for (int l = rg; l < L; l += RG) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(xb + (int64_t)l * xs_t), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = f[e] * mul[e] + add[e];
    *reinterpret_cast<uint4*>(yb + (int64_t)l * ys_t) = pack8(f);
  }
}

// dx = rstd * (g - mean_L(g) - xhat * mean_L(g * xhat)),  g = dy * gamma  (+ optional addend)
// dgamma += sum_{b,l} dy * xhat ; dbeta += sum_{b,l} dy   (fp32 atomics, one per column per block)
__global__ __launch_bounds__(NT) void seqnorm_bwd_kernel(
    const bf16_t* __restrict__ dy, int64_t ds_b, int64_t ds_t, const bf16_t* __restrict__ x,
    int64_t xs_b, int64_t xs_t, int L, int D, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma, const bf16_t* addend,
    int64_t as_b, int64_t as_t, bf16_t* dx, int64_t dxs_b, int64_t dxs_t,
    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[4 * RG * CW];
  const int b = blockIdx.x, c0 = blockIdx.y * CW;
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = c0 + cv * 8;
  const bool cok = col < D;
  float mu[8], rs[8], ga[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = cok ? mean[(int64_t)b * D + col + e] : 0.f;
    rs[e] = cok ? rstd[(int64_t)b * D + col + e] : 0.f;
    ga[e] = cok ? gamma[col + e] : 0.f;
  }
  const bf16_t* xb = x + (int64_t)b * xs_b + col;
  const bf16_t* db = dy + (int64_t)b * ds_b + col;
  float part[4][8] = {};  // sum g, sum g*xhat, sum dy*xhat, sum dy
  if (cok)
    for (int l = rg; l < L; l += RG) {
      float fx[8], fd[8];
      unpack8(*reinterpret_cast<const uint4*>(xb + (int64_t)l * xs_t), fx);
      unpack8(*reinterpret_cast<const uint4*>(db + (int64_t)l * ds_t), fd);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (fx[e] - mu[e]) * rs[e];
        const float g = fd[e] * ga[e];
        part[0][e] += g;
        part[1][e] += g * xh;
        part[2][e] += fd[e] * xh;
        part[3][e] += fd[e];
      }
    }
  reduce_rows<4>(part, red);
  if (threadIdx.x < CW && c0 + threadIdx.x < D) {
    atomicAdd(dgamma + c0 + threadIdx.x, red[2 * RG * CW + threadIdx.x]);
    atomicAdd(dbeta + c0 + threadIdx.x, red[3 * RG * CW + threadIdx.x]);
  }
  if (!cok) return;
  float mg[8], mgx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mg[e] = red[cv * 8 + e] / L;
    mgx[e] = red[RG * CW + cv * 8 + e] / L;
  }
  bf16_t* dxb = dx + (int64_t)b * dxs_b + col;
  const bf16_t* ab = addend ? addend + (int64_t)b * as_b + col : nullptr;
  for (int l = rg; l < L; l += RG) {
    float fx[8], fd[8], fa[8];
    unpack8(*reinterpret_cast<const uint4*>(xb + (int64_t)l * xs_t), fx);
    unpack8(*reinterpret_cast<const uint4*>(db + (int64_t)l * ds_t), fd);
    if (ab) unpack8(*reinterpret_cast<const uint4*>(ab + (int64_t)l * as_t), fa);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (fx[e] - mu[e]) * rs[e];
      const float g = fd[e] * ga[e];
      fx[e] = rs[e] * (g - mg[e] - xh * mgx[e]) + (ab ? fa[e] : 0.f);
    }
    *reinterpret_cast<uint4*>(dxb + (int64_t)l * dxs_t) = pack8(fx);
  }
}

// out[n] += sum_m x[m][n]  and, with rng, dz = x * keep / keep_prob written to z first
// (dropout backward of a GEMM-epilogue dropout; the column sum is then the bias gradient).
constexpr int CS_ROWS = 256;
__global__ __launch_bounds__(NT) void colsum_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                    int M, int N, float* __restrict__ out,
                                                    const uint32_t* __restrict__ rng,
                                                    uint32_t layer, uint32_t site, uint32_t thresh,
                                                    float scale, int64_t row_offset,
                                                    bf16_t* __restrict__ z, int64_t ldz) {
  __shared__ float red[RG * CW];
  const int c0 = blockIdx.x * CW, r0 = blockIdx.y * CS_ROWS;
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = c0 + cv * 8;
  const bool cok = col < N;
  uint32_t key = 0;
  if (rng) key = stream_key(rng[0], rng[1], layer, site);
  float part[1][8] = {};
  if (cok)
    for (int m = r0 + rg; m < min(M, r0 + CS_ROWS); m += RG) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (int64_t)m * ldx + col), f);
      if (rng) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t ctr = (uint32_t)((row_offset + m) * (int64_t)N + col + e);
          f[e] = keep_draw(key, ctr, thresh) ? f[e] * scale : 0.f;
        }
        *reinterpret_cast<uint4*>(z + (int64_t)m * ldz + col) = pack8(f);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) part[0][e] += f[e];
    }
  if (!out) return;
  reduce_rows<1>(part, red);
  if (threadIdx.x < CW && c0 + threadIdx.x < N) atomicAdd(out + c0 + threadIdx.x, red[threadIdx.x]);
}

}  // namespace

extern "C" int mmt_seqnorm_fwd(const void* x, int64_t xs_b, int64_t xs_t, int B, int L, int D,
                               const float* gamma, const float* beta, float eps, void* y,
                               int64_t ys_b, int64_t ys_t, float* mean, float* rstd,
                               mmt_stream_t stream) {
  MMT_CHECK_ARG(x && y && gamma && beta && mean && rstd, "mmt_seqnorm_fwd: null pointer");
  MMT_CHECK_ARG(B > 0 && L > 0 && D > 0 && D % 8 == 0 && xs_t % 8 == 0 && ys_t % 8 == 0 &&
                    xs_b % 8 == 0 && ys_b % 8 == 0,
                "mmt_seqnorm_fwd: D and strides must be multiples of 8");
  dim3 grid(B, (D + CW - 1) / CW);
  hipLaunchKernelGGL(seqnorm_fwd_kernel, grid, dim3(NT), 0, as_stream(stream), (const bf16_t*)x,
                     xs_b, xs_t, L, D, gamma, beta, eps, (bf16_t*)y, ys_b, ys_t, mean, rstd);
  MMT_CHECK_LAUNCH("mmt_seqnorm_fwd");
  return MMT_OK;
}

extern "C" int mmt_seqnorm_bwd(const void* dy, int64_t ds_b, int64_t ds_t, const void* x,
                               int64_t xs_b, int64_t xs_t, int B, int L, int D, const float* mean,
                               const float* rstd, const float* gamma, const void* addend,
                               int64_t as_b, int64_t as_t, void* dx, int64_t dxs_b, int64_t dxs_t,
                               float* dgamma, float* dbeta, mmt_stream_t stream) {
  MMT_CHECK_ARG(dy && x && mean && rstd && gamma && dx && dgamma && dbeta,
                "mmt_seqnorm_bwd: null pointer");
  MMT_CHECK_ARG(B > 0 && L > 0 && D > 0 && D % 8 == 0 && ds_t % 8 == 0 && xs_t % 8 == 0 &&
                    dxs_t % 8 == 0 && (!addend || as_t % 8 == 0),
                "mmt_seqnorm_bwd: D and strides must be multiples of 8");
  dim3 grid(B, (D + CW - 1) / CW);
  hipLaunchKernelGGL(seqnorm_bwd_kernel, grid, dim3(NT), 0, as_stream(stream), (const bf16_t*)dy,
                     ds_b, ds_t, (const bf16_t*)x, xs_b, xs_t, L, D, mean, rstd, gamma,
                     (const bf16_t*)addend, as_b, as_t, (bf16_t*)dx, dxs_b, dxs_t, dgamma, dbeta);
  MMT_CHECK_LAUNCH("mmt_seqnorm_bwd");
  return MMT_OK;
}

extern "C" int mmt_colsum(const void* x, int64_t ldx, int M, int N, float* out,
                          mmt_stream_t stream) {
  MMT_CHECK_ARG(x && out && M > 0 && N > 0 && N % 8 == 0 && ldx % 8 == 0, "mmt_colsum: bad args");
  dim3 grid((N + CW - 1) / CW, (M + CS_ROWS - 1) / CS_ROWS);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(NT), 0, as_stream(stream), (const bf16_t*)x, ldx, M,
                     N, out, nullptr, 0u, 0u, 0u, 1.f, (int64_t)0, nullptr, (int64_t)0);
  MMT_CHECK_LAUNCH("mmt_colsum");
  return MMT_OK;
}

extern "C" int mmt_dropout_bwd(const void* dy, int64_t ldy, int M, int N, const uint32_t* rng,
                               uint32_t layer, uint32_t site, float keep_prob,
                               int64_t row_offset, void* dz, int64_t ldz, float* colsum,
                               mmt_stream_t stream) {
  MMT_CHECK_ARG(dy && dz && rng && M > 0 && N > 0 && N % 8 == 0 && ldy % 8 == 0 && ldz % 8 == 0,
                "mmt_dropout_bwd: bad args");
  MMT_CHECK_ARG(keep_prob > 0.f && keep_prob <= 1.f, "mmt_dropout_bwd: keep_prob");
  dim3 grid((N + CW - 1) / CW, (M + CS_ROWS - 1) / CS_ROWS);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(NT), 0, as_stream(stream), (const bf16_t*)dy, ldy, M,
                     N, colsum, rng, layer, site, keep_threshold(keep_prob), 1.f / keep_prob,
                     row_offset, (bf16_t*)dz, ldz);
  MMT_CHECK_LAUNCH("mmt_dropout_bwd");
  return MMT_OK;
}

// Small fused kernels around the hot path (gfx950): sequence assembly (token_sequencer.py
// :255-269 + readout.py:18-33 + attention.py:71-85 position embedding + image_tokenizer.py:300-307
// row/col embeddings), readout mean (diffusion.py:102), diffusion noising / Fourier features /
// loss (diffusion.py:17-143), T5 RMS-norm and embedding gather, fused AdamW over the flat
// parameter buffer, and the device-side step counter that keys every random stream.
#include <math.h>

#include <algorithm>

#include "common.h"

using namespace mmt;

namespace {

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

// row descriptor: kind << 24 | index   (kind 0 text row, 1 image row, 2 readout row)
constexpr int KIND_TEXT = 0, KIND_IMAGE = 1, KIND_READOUT = 2;

__global__ void seq_assemble_fwd_kernel(int B, int L, int D, const int32_t* __restrict__ row_src,
                                        const bf16_t* __restrict__ text, int T,
                                        const bf16_t* __restrict__ img, int NI,
                                        const int32_t* __restrict__ rtok,
                                        const int32_t* __restrict__ ctok,
                                        const float* __restrict__ row_emb,
                                        const float* __restrict__ col_emb,
                                        const float* __restrict__ readout_pe,
                                        const float* __restrict__ pe, float* __restrict__ x0) {
  const int cpr = D / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * L * cpr) return;
  const int ch = idx % cpr;
  const int l = (idx / cpr) % L;
  const int b = idx / ((int64_t)cpr * L);
  const int d0 = ch * 8;
  const int desc = row_src[l];
  const int kind = desc >> 24, j = desc & 0xffffff;
  float v[8];
  if (kind == KIND_TEXT) {
    unpack8(*reinterpret_cast<const uint4*>(text + ((int64_t)b * T + j) * D + d0), v);
  } else if (kind == KIND_IMAGE) {
    unpack8(*reinterpret_cast<const uint4*>(img + ((int64_t)b * NI + j) * D + d0), v);
    const int rt = rtok[(int64_t)b * NI + j], ct = ctok[(int64_t)b * NI + j];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += row_emb[(int64_t)rt * D + d0 + e] + col_emb[(int64_t)ct * D + d0 + e];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = readout_pe[(int64_t)j * D + d0 + e];  // zeros + embedding
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] += pe[(int64_t)l * D + d0 + e];
  float* xo = x0 + ((int64_t)b * L + l) * D + d0;
  *reinterpret_cast<float4*>(xo) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(xo + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

__global__ void seq_assemble_bwd_kernel(int B, int L, int D, const int32_t* __restrict__ row_src,
                                        const float* __restrict__ dx0, bf16_t* __restrict__ dtext,
                                        int T, bf16_t* __restrict__ dimg, int NI,
                                        const int32_t* __restrict__ rtok,
                                        const int32_t* __restrict__ ctok,
                                        float* __restrict__ drow_emb, float* __restrict__ dcol_emb,
                                        float* __restrict__ dreadout_pe) {
  const int cpr = D / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * L * cpr) return;
  const int ch = idx % cpr;
  const int l = (idx / cpr) % L;
  const int b = idx / ((int64_t)cpr * L);
  const int d0 = ch * 8;
  const int desc = row_src[l];
  const int kind = desc >> 24, j = desc & 0xffffff;
  float v[8];
  {
    const float* gp = dx0 + ((int64_t)b * L + l) * D + d0;
    const float4 a = *reinterpret_cast<const float4*>(gp), c = *reinterpret_cast<const float4*>(gp + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
  }
  if (kind == KIND_TEXT) {
    if (dtext) *reinterpret_cast<uint4*>(dtext + ((int64_t)b * T + j) * D + d0) = pack8(v);
  } else if (kind == KIND_IMAGE) {
    *reinterpret_cast<uint4*>(dimg + ((int64_t)b * NI + j) * D + d0) = pack8(v);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) grad_add(dreadout_pe + (int64_t)j * D + d0 + e, v[e]);
  }
}

// d(row_emb)[tok] += dx0[b, l(j)] over every image token (b, j) with rtok == tok (same for col).
// One workgroup = 64 columns x a slice of the image tokens; the two (Q x 64) partial tables are
// accumulated with LDS atomics and flushed with one global atomic per table entry. Measured:
// bound by the LDS float atomics (~50 M per step at B = 256); fewer, longer workgroups were slower.
constexpr int EMB_COLS = 64, EMB_SPLIT = 128;
// DET (deterministic mode): the table holds 64-bit fixed-point sums (integer LDS atomics,
// order-independent) and each entry goes to the gradient's fixed-point shadow (grad_add).
template <bool DET>
__global__ __launch_bounds__(256) void embed_grad_kernel(int B, int L, int D, int NI, int Q,
                                                         const int32_t* __restrict__ img_rows,
                                                         const float* __restrict__ dx0,
                                                         const int32_t* __restrict__ rtok,
                                                         const int32_t* __restrict__ ctok,
                                                         float* __restrict__ drow_emb,
                                                         float* __restrict__ dcol_emb) {
  extern __shared__ float tab[];  // [2][Q][EMB_COLS] (DET: long long)
  long long* tab64 = reinterpret_cast<long long*>(tab);
  const int c0 = blockIdx.x * EMB_COLS;
  for (int i = threadIdx.x; i < 2 * Q * EMB_COLS; i += blockDim.x) {
    if constexpr (DET) tab64[i] = 0;
    else tab[i] = 0.f;
  }
  __syncthreads();
  const int64_t total = (int64_t)B * NI;
  const int64_t per = (total + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = blockIdx.y * per, r1 = min(total, r0 + per);
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;  // 8 x 8 columns, 32 row groups
  const int col = c0 + cv * 8;
  if (col < D) {
    for (int64_t rr = r0 + rg; rr < r1; rr += 32) {
      const int b = rr / NI, j = rr % NI;
      const float* gp = dx0 + ((int64_t)b * L + img_rows[j]) * D + col;
      const float4 a = *reinterpret_cast<const float4*>(gp), c = *reinterpret_cast<const float4*>(gp + 4);
      const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      const int rt = rtok[rr], ct = ctok[rr];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (DET) {
          if (det_fits(v[e])) {
            const unsigned long long q = (unsigned long long)det_fixed(v[e]);
            atomicAdd(reinterpret_cast<unsigned long long*>(&tab64[rt * EMB_COLS + cv * 8 + e]), q);
            atomicAdd(reinterpret_cast<unsigned long long*>(&tab64[(Q + ct) * EMB_COLS + cv * 8 + e]), q);
          } else {  // NaN / Inf / out of the shadow's range: straight to the fp32 gradient (visible)
            atomicAdd(drow_emb + (int64_t)rt * D + col + e, v[e]);
            atomicAdd(dcol_emb + (int64_t)ct * D + col + e, v[e]);
          }
        } else {
          atomicAdd(&tab[rt * EMB_COLS + cv * 8 + e], v[e]);
          atomicAdd(&tab[(Q + ct) * EMB_COLS + cv * 8 + e], v[e]);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * Q * EMB_COLS; i += blockDim.x) {
    const int which = i / (Q * EMB_COLS), rem = i % (Q * EMB_COLS);
    const int tok = rem / EMB_COLS, cc = c0 + rem % EMB_COLS;
    float* dst = (which ? dcol_emb : drow_emb) + (int64_t)tok * D + cc;
    if constexpr (DET) {  // the fixed-point partial straight into the shadow (exact)
      const long long q = tab64[i];
      const int64_t gi = dst - g_det.base;
      if (cc < D && q != 0) {
        if (g_det.fx != nullptr && gi >= 0 && gi < g_det.n)
          atomicAdd(reinterpret_cast<unsigned long long*>(g_det.fx + gi), (unsigned long long)q);
        else
          atomicAdd(dst, (float)((double)q * (1.0 / DET_SCALE)));
      }
    } else {
      const float val = tab[i];
      if (cc < D && val != 0.f) atomicAdd(dst, val);
    }
  }
}

// Position-embedding gradients by window (mmt_patch_embed_grad). A patch in patch-row ri draws its
// row token from the window [q(ri P), q((ri + 1) P)) of patch_positions_kernel (likewise columns),
// so the image tokens of one patch row touch only that window's few table rows. One workgroup =
// one window x 64 columns x a slice of the batch: each thread keeps a register accumulator per
// window token (select + add per row, no atomics), the 32 row groups meet by shuffles and in LDS,
// and the workgroup adds its WMAX x 64 partial table with one global atomic per entry.
template <int WMAX>
__global__ __launch_bounds__(256) void embed_grad_win_kernel(
    int B, int L, int D, int I, int PPD, int Himg, int P, int Q, int splits,
    const int32_t* __restrict__ img_rows, const float* __restrict__ dx0,
    const int32_t* __restrict__ rtok, const int32_t* __restrict__ ctok, float* __restrict__ drow,
    float* __restrict__ dcol) {
  __shared__ float part[4][WMAX][EMB_COLS];
  const int w = blockIdx.x, c0 = blockIdx.y * EMB_COLS;
  const int z = blockIdx.z % 2, sp = blockIdx.z / 2;  // table (0 rows, 1 columns), batch slice
  const int NP = PPD * PPD, NI = I * NP, RPS = I * PPD;  // image tokens per sample in the window
  auto q = [&](int v) { return (int)floorf(((float)v / (float)Himg) * (float)(Q - 1)); };
  const int ws = q(w * P), wn = max(1, q((w + 1) * P) - ws);
  const int bper = (B + splits - 1) / splits, b0 = sp * bper, b1 = min(B, b0 + bper);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = c0 + cv * 8;
  const int32_t* tok = z == 0 ? rtok : ctok;
  float acc[WMAX][8];
#pragma unroll
  for (int t = 0; t < WMAX; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[t][e] = 0.f;
  if (col < D && b0 < b1) {
    const int nrows = (b1 - b0) * RPS;
    for (int r = rg; r < nrows; r += 32) {
      const int b = b0 + r / RPS, rem = r % RPS, i = rem / PPD, k = rem % PPD;
      const int p = z == 0 ? k * PPD + w : w * PPD + k;  // patch_positions_kernel: ri = p % PPD
      const int j = i * NP + p;
      const int t = tok[(int64_t)b * NI + j] - ws;
      const float* gp = dx0 + ((int64_t)b * L + img_rows[j]) * D + col;
      const float4 a = *reinterpret_cast<const float4*>(gp), c = *reinterpret_cast<const float4*>(gp + 4);
      const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
      for (int u = 0; u < WMAX; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[u][e] += t == u ? v[e] : 0.f;
    }
  }
#pragma unroll
  for (int u = 0; u < WMAX; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = acc[u][e];
      x += __shfl_xor(x, 8, 64);
      x += __shfl_xor(x, 16, 64);
      x += __shfl_xor(x, 32, 64);
      acc[u][e] = x;
    }
  if (lane < 8)
#pragma unroll
    for (int u = 0; u < WMAX; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) part[wave][u][cv * 8 + e] = acc[u][e];
  __syncthreads();
  float* table = z == 0 ? drow : dcol;
  for (int i = threadIdx.x; i < WMAX * EMB_COLS; i += blockDim.x) {
    const int u = i / EMB_COLS, cc = c0 + i % EMB_COLS;
    if (u < wn && cc < D) {
      const float val = part[0][u][i % EMB_COLS] + part[1][u][i % EMB_COLS] +
                        part[2][u][i % EMB_COLS] + part[3][u][i % EMB_COLS];
      if (val != 0.f) grad_add(table + (int64_t)(ws + u) * D + cc, val);
    }
  }
}

// e[b, :] = mean over the listed rows of x[b] ; written as bf16 into out (row stride ld_out)
__global__ void rows_mean_fwd_kernel(const float* __restrict__ x, int64_t xs_b, int64_t xs_t,
                                     int D, const int32_t* __restrict__ rows, int nrows,
                                     bf16_t* __restrict__ out, int64_t ld_out) {
  const int b = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < nrows; ++i) s += x[b * xs_b + (int64_t)rows[i] * xs_t + d];
    out[b * ld_out + d] = f2bf(s / nrows);
  }
}

// dx[b, l, :] = de[b, :] / n for listed rows (row_flag[l] >= 0), 0 otherwise (whole buffer)
__global__ void rows_mean_bwd_kernel(const bf16_t* __restrict__ de, int64_t ld_de, int B, int L,
                                     int D, const int32_t* __restrict__ row_flag, int nrows,
                                     float* __restrict__ dx) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * L * D) return;
  const int d = idx % D;
  const int l = (idx / D) % L;
  const int b = idx / ((int64_t)D * L);
  dx[idx] = row_flag[l] >= 0 ? bf2f(de[b * ld_de + d]) / nrows : 0.f;
}

// Grouped readout means (categorical.py:32-37: "batch (action timestep) embeddings -> batch action
// timestep embeddings", mean over timestep): out[b, g, :] = mean of the rows l with
// row_group[l] == g (counts[g] of them); bf16 (B, G, D). Backward: dx[b, l, :] = de[b, g(l), :] /
// counts[g], 0 for rows in no group (whole fp32 buffer).
__global__ void rows_group_mean_fwd_kernel(const float* __restrict__ x, int64_t xs_b, int64_t xs_t,
                                           int L, int D, const int32_t* __restrict__ row_group,
                                           int G, const int32_t* __restrict__ counts,
                                           bf16_t* __restrict__ out) {
  const int b = blockIdx.x, g = blockIdx.y;
  const float inv = 1.f / (float)counts[g];
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int l = 0; l < L; ++l)
      if (row_group[l] == g) s += x[b * xs_b + (int64_t)l * xs_t + d];
    out[((int64_t)b * G + g) * D + d] = f2bf(s * inv);
  }
}

__global__ void rows_group_mean_bwd_kernel(const bf16_t* __restrict__ de, int B, int L, int D,
                                           const int32_t* __restrict__ row_group, int G,
                                           const int32_t* __restrict__ counts,
                                           float* __restrict__ dx) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * L * D) return;
  const int d = idx % D;
  const int l = (idx / D) % L;
  const int b = idx / ((int64_t)D * L);
  const int g = row_group[l];
  dx[idx] = g >= 0 ? bf2f(de[((int64_t)b * G + g) * D + d]) / (float)counts[g] : 0.f;
}

// Continuous and categorical action-head losses, one wave per row of z (fp32, row stride ldz):
// kind 0 — ContinuousActionHead (continuous.py:19-26) + compute_l2_loss (octo.py:167-174), rows = B,
//   N = A: p = tanh(z / m) m (written to pred if non-NULL); loss += inv_count sum_a (p - y)^2;
//   dz = 2 (p - y)(1 - tanh^2) inv_count.
// kind 1 — CategoricalActionHead + compute_ce_loss (octo.py:187-198), rows = B*A, N = num_bins:
//   bin = jnp.digitize(y, edges) = #edges <= y (edges = linspace(-m, m, N+1)), label =
//   one_hot(bin, N) — all zero when bin >= N, the reference's off-by-one kept; loss += inv_count
//   (sum(label) logsumexp(z) - label . z); dz = (sum(label) softmax(z) - label) inv_count.
// y NULL: forward only (kind 0 writes pred). loss is accumulated atomically (zero it first).
__global__ __launch_bounds__(256) void action_head_kernel(
    int kind, const float* __restrict__ z, int64_t ldz, int R, int N, const float* __restrict__ y,
    const float* __restrict__ edges, int n_edges, float max_action, float inv_count,
    float* __restrict__ pred, float* __restrict__ loss, bf16_t* __restrict__ dz) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* zr = z + (int64_t)r * ldz;
  float row_loss = 0.f;
  if (kind == 0) {
    for (int a = lane; a < N; a += 64) {
      const float th = tanhf(zr[a] / max_action);
      const float p = th * max_action;
      if (pred) pred[(int64_t)r * N + a] = p;
      if (y) {
        const float d = p - y[(int64_t)r * N + a];
        row_loss += d * d;
        dz[(int64_t)r * N + a] = f2bf(2.f * d * (1.f - th * th) * inv_count);
      }
    }
  } else {
    const float yv = y[r];
    int bin = 0;
    for (int i = 0; i < n_edges; ++i) bin += edges[i] <= yv ? 1 : 0;
    const float has = bin < N ? 1.f : 0.f;
    float mx = -INFINITY;
    for (int c = lane; c < N; c += 64) mx = fmaxf(mx, zr[c]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float se = 0.f;
    for (int c = lane; c < N; c += 64) se += expf(zr[c] - mx);
    se = wave_sum(se);
    const float lse = mx + logf(se);
    for (int c = lane; c < N; c += 64) {
      const float lab = (c == bin) ? 1.f : 0.f;
      dz[(int64_t)r * N + c] = f2bf((has * expf(zr[c] - lse) - lab) * inv_count);
    }
    if (lane == 0 && bin < N) row_loss = lse - zr[bin];
  }
  if (!y) return;
  row_loss = wave_sum(row_loss);
  if (lane == 0) atomicAdd(loss, row_loss * inv_count);
}

// Diffusion noising + Fourier features (diffusion.py:41-51, 110-131):
//   t ~ U{0..steps-1}, eps ~ N(0, 1) (Box-Muller on the counter stream) unless injected;
//   noisy = sqrt(abar_t) a + sqrt(1 - abar_t) eps  -> cat[:, 0:A]  (bf16)
//   h = 2 pi t W^T (W: (F,) = fourier kernel (F, 1)), feats = [cos h, sin h] (bf16, 2F)
__global__ void diffusion_prep_kernel(const uint32_t* __restrict__ rng, int B, int A, int steps,
                                      int64_t sample_offset, const float* __restrict__ actions,
                                      const float* __restrict__ alpha_hats,
                                      const float* __restrict__ fw, int F,
                                      const int32_t* __restrict__ t_in,
                                      const float* __restrict__ eps_in, int32_t* __restrict__ t_out,
                                      float* __restrict__ eps_out, bf16_t* __restrict__ cat,
                                      int64_t ld_cat, bf16_t* __restrict__ feats) {
  const int b = blockIdx.x;
  __shared__ int s_t;
  if (threadIdx.x == 0) {
    int t;
    if (t_in) {
      t = t_in[b];
    } else {
      const uint32_t key = stream_key(rng[0], rng[1], 0xFFFEu, 1);
      t = (int)(((uint64_t)draw_u32(key, (uint32_t)(sample_offset + b)) * (uint32_t)steps) >> 32);
    }
    s_t = t;
    t_out[b] = t;
  }
  __syncthreads();
  const int t = s_t;
  const float ah = alpha_hats[t];
  const float a1 = sqrtf(ah), a2 = sqrtf(1.f - ah);
  for (int j = threadIdx.x; j < A; j += blockDim.x) {
    float e;
    if (eps_in) {
      e = eps_in[b * A + j];
    } else {
      const uint32_t key = stream_key(rng[0], rng[1], 0xFFFEu, 2);
      const uint32_t c = (uint32_t)((sample_offset + b) * A + j);
      const float u1 = ((draw_u32(key, 2 * c) >> 8) + 1) * (1.f / 16777216.f);  // (0, 1]
      const float u2 = (draw_u32(key, 2 * c + 1) >> 8) * (1.f / 16777216.f);
      e = sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
    }
    eps_out[b * A + j] = e;
    cat[b * ld_cat + j] = f2bf(a1 * actions[b * A + j] + a2 * e);
  }
  const float tf = (float)t;
  for (int k = threadIdx.x; k < F; k += blockDim.x) {
    const float h = 2.f * 3.141592653589793f * tf * fw[k];
    feats[(int64_t)b * 2 * F + k] = f2bf(cosf(h));
    feats[(int64_t)b * 2 * F + F + k] = f2bf(sinf(h));
  }
}

// dW[k] += sum_b 2 pi t_b (cos(h) dsin - sin(h) dcos); the batch is split over grid.y
// (FB_B samples per workgroup, fp32 atomics into dw) so the launch is not one serial loop over B.
constexpr int FB_B = 8;
__global__ void fourier_bwd_kernel(const bf16_t* __restrict__ dfeats, int B, int F,
                                   const int32_t* __restrict__ t, const float* __restrict__ fw,
                                   float* __restrict__ dw) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= F) return;
  const int b0 = blockIdx.y * FB_B;
  const float w = fw[k];
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < FB_B; ++i) {
    const int b = b0 + i;
    if (b < B) {
      const float tt = 2.f * 3.141592653589793f * (float)t[b];
      const float h = tt * w;
      const float dc = bf2f(dfeats[(int64_t)b * 2 * F + k]), ds = bf2f(dfeats[(int64_t)b * 2 * F + F + k]);
      acc += tt * (cosf(h) * ds - sinf(h) * dc);
    }
  }
  grad_add(dw + k, acc);
}

// loss = mean_b sum_j 0.5 (pred - eps)^2 (optax.l2_loss, diffusion.py:141-142);
// dpred = (pred - eps) * grad_scale / B  (bf16). One workgroup.
__global__ void diffusion_loss_kernel(const float* __restrict__ pred, int64_t ld_pred,
                                      const float* __restrict__ eps, int B, int A,
                                      float grad_scale, float* __restrict__ loss,
                                      bf16_t* __restrict__ dpred) {
  __shared__ float red[1024 / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < B * A; i += blockDim.x) {
    const int b = i / A, j = i % A;
    const float d = pred[b * ld_pred + j] - eps[i];
    s += 0.5f * d * d;
    dpred[i] = f2bf(d * grad_scale / B);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    loss[0] = t / B;
  }
}

// T5LayerNorm: y = x * rsqrt(mean(x^2) + eps) * w   (one wave per row, D % 8 == 0)
__global__ void rmsnorm_fwd_kernel(const bf16_t* __restrict__ x, int64_t rows, int D,
                                   const bf16_t* __restrict__ w, float eps, bf16_t* __restrict__ y) {
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const bf16_t* xr = x + row * D;
  float s = 0.f;
  if (D <= 1024) {
    // the row read once: both of a lane's chunks (and the weight's) loaded together, unconditional
    // (a lane past D reads chunk 0 and drops it); same sums in the same order as the loop below
    const int c0 = lane * 8, c1 = c0 + 512;
    const bool h0 = c0 < D, h1 = c1 < D;
    const uint4 u0 = *reinterpret_cast<const uint4*>(xr + (h0 ? c0 : 0));
    const uint4 u1 = *reinterpret_cast<const uint4*>(xr + (h1 ? c1 : 0));
    const uint4 w0 = *reinterpret_cast<const uint4*>(w + (h0 ? c0 : 0));
    const uint4 w1 = *reinterpret_cast<const uint4*>(w + (h1 ? c1 : 0));
    float f0[8], f1[8];
    unpack8(u0, f0);
    unpack8(u1, f1);
    if (h0)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += f0[e] * f0[e];
    if (h1)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += f1[e] * f1[e];
    s = wave_sum(s);
    const float rs = rsqrtf(s / D + eps);
    float g[8];
    if (h0) {
      unpack8(w0, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) f0[e] = f0[e] * rs * g[e];
      *reinterpret_cast<uint4*>(y + row * D + c0) = pack8(f0);
    }
    if (h1) {
      unpack8(w1, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) f1[e] = f1[e] * rs * g[e];
      *reinterpret_cast<uint4*>(y + row * D + c1) = pack8(f1);
    }
    return;
  }
  for (int c = lane * 8; c < D; c += 512) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += f[e] * f[e];
  }
  s = wave_sum(s);
  const float rs = rsqrtf(s / D + eps);
  for (int c = lane * 8; c < D; c += 512) {
    float f[8], g[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c), f);
    unpack8(*reinterpret_cast<const uint4*>(w + c), g);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = f[e] * rs * g[e];
    *reinterpret_cast<uint4*>(y + row * D + c) = pack8(f);
  }
}

__global__ void embedding_gather_kernel(const int32_t* __restrict__ ids, int64_t n, int D,
                                        const bf16_t* __restrict__ table, int vocab,
                                        bf16_t* __restrict__ out) {
  const int cpr = D / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * cpr) return;
  const int64_t r = idx / cpr;
  const int c = (idx % cpr) * 8;
  int id = ids[r];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  *reinterpret_cast<uint4*>(out + r * D + c) = *reinterpret_cast<const uint4*>(table + (int64_t)id * D + c);
}

// AdamW (optax.adamw semantics, decoupled weight decay on every parameter, bias-corrected
// moments) over the flat fp32 master buffer; writes the bf16 shadow used by the GEMMs.
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v,
                             bf16_t* __restrict__ shadow, int64_t n, const int32_t* __restrict__ state,
                             float lr, double b1d, double b2d, float eps, float wd, float grad_scale) {
  const int step = state[1] + 1;
  // the betas arrive in double (optax / torch hold them as Python floats): 1 - b and the bias
  // corrections are formed in double and rounded once (fp32 1.f - 0.999f would differ from
  // (float)0.001 by 1.3e-5 relative)
  const float b1 = (float)b1d, b2 = (float)b2d;
  const float bc1 = (float)(1.0 - pow(b1d, (double)step));
  const float bc2 = (float)(1.0 - pow(b2d, (double)step));
  const float omb1 = (float)(1.0 - b1d), omb2 = (float)(1.0 - b2d);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * grad_scale;
    const float mi = b1 * m[i] + omb1 * gi;
    const float vi = b2 * v[i] + omb2 * (gi * gi);
    m[i] = mi;
    v[i] = vi;
    const float upd = (mi / bc1) / (sqrtf(vi / bc2) + eps) + wd * p[i];
    const float pn = p[i] - lr * upd;
    p[i] = pn;
    if (shadow) shadow[i] = f2bf(pn);
  }
}

// Transposed bf16 weight shadows: dst (cols, rows) = src (rows, cols)^T for a batch of matrices
// (desc: n x {src_off, dst_off, rows, cols, first_tile} elements / tiles), 64 x 64 tiles through a
// padded LDS tile; grid-stride over all tiles. Lets every dX product run as an NT GEMM.
__global__ __launch_bounds__(256) void transpose_bf16_batched_kernel(
    const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, const int64_t* __restrict__ desc,
    int n, int64_t total_tiles) {
  __shared__ bf16_t tile[64][66];
  for (int64_t t = blockIdx.x; t < total_tiles; t += gridDim.x) {
    int m = 0;
    while (m + 1 < n && desc[5 * (m + 1) + 4] <= t) ++m;
    const int64_t so = desc[5 * m], dso = desc[5 * m + 1];
    const int rows = (int)desc[5 * m + 2], cols = (int)desc[5 * m + 3];
    const int64_t lt = t - desc[5 * m + 4];
    const int tcols = (cols + 63) / 64;
    const int r0 = (int)(lt / tcols) * 64, c0 = (int)(lt % tcols) * 64;
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
      const int rr = i >> 6, cc = i & 63;
      if (r0 + rr < rows && c0 + cc < cols) tile[rr][cc] = src[so + (int64_t)(r0 + rr) * cols + c0 + cc];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
      const int cc = i >> 6, rr = i & 63;  // dst row = source column
      if (r0 + rr < rows && c0 + cc < cols) dst[dso + (int64_t)(c0 + cc) * rows + r0 + rr] = tile[rr][cc];
    }
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ a, bf16_t* __restrict__ b, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    b[i] = f2bf(a[i]);
}

__global__ void step_advance_kernel(int32_t* state) { state[1] += 1; }


// The LDS-table embedding-gradient kernel, in its deterministic form when the mode is on.
void launch_embed_table(dim3 grid, hipStream_t s, int B, int L, int D, int NI, int Q,
                        const int32_t* img_rows, const float* dx0, const int32_t* rtok,
                        const int32_t* ctok, float* drow_emb, float* dcol_emb) {
  static const bool attr_ = (hipFuncSetAttribute((const void*)embed_grad_kernel<false>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024) == hipSuccess &&
                             hipFuncSetAttribute((const void*)embed_grad_kernel<true>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024) == hipSuccess);
  (void)attr_;
  if (g_det_host.fx)
    hipLaunchKernelGGL(embed_grad_kernel<true>, grid, dim3(256), sizeof(long long) * 2 * Q * EMB_COLS,
                       s, B, L, D, NI, Q, img_rows, dx0, rtok, ctok, drow_emb, dcol_emb);
  else
    hipLaunchKernelGGL(embed_grad_kernel<false>, grid, dim3(256), sizeof(float) * 2 * Q * EMB_COLS,
                       s, B, L, D, NI, Q, img_rows, dx0, rtok, ctok, drow_emb, dcol_emb);
}

// deterministic mode: grad += shadow x 2^-36, shadow = 0 (elementwise: the result is independent
// of every ordering)
__global__ void det_flush_kernel(float* __restrict__ grad, long long* __restrict__ fx, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const long long q = fx[i];
    if (q != 0) {
      grad[i] += (float)((double)q * (1.0 / DET_SCALE));
      fx[i] = 0;
    }
  }
}

}  // namespace

extern "C" int mmt_seq_assemble_fwd(int B, int L, int D, const int32_t* row_src, const void* text,
                                    int T, const void* img, int NI, const int32_t* rtok,
                                    const int32_t* ctok, const float* row_emb, const float* col_emb,
                                    const float* readout_pe, const float* pe, void* x0,
                                    mmt_stream_t stream) {
  MMT_CHECK_ARG(row_src && x0 && pe && D % 8 == 0 && B > 0 && L > 0, "mmt_seq_assemble_fwd: args");
  const int64_t n = (int64_t)B * L * (D / 8);
  hipLaunchKernelGGL(seq_assemble_fwd_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     as_stream(stream), B, L, D, row_src, (const bf16_t*)text, T,
                     (const bf16_t*)img, NI, rtok, ctok, row_emb, col_emb, readout_pe, pe,
                     (float*)x0);
  MMT_CHECK_LAUNCH("mmt_seq_assemble_fwd");
  return MMT_OK;
}

extern "C" int mmt_seq_assemble_bwd(int B, int L, int D, const int32_t* row_src, const void* dx0,
                                    void* dtext, int T, void* dimg, int NI, const int32_t* rtok,
                                    const int32_t* ctok, const int32_t* img_rows, int Q,
                                    float* drow_emb, float* dcol_emb, float* dreadout_pe,
                                    mmt_stream_t stream) {
  MMT_CHECK_ARG(row_src && dx0 && D % 8 == 0 && B > 0 && L > 0, "mmt_seq_assemble_bwd: args");
  // drow_emb = dcol_emb = NULL: the image tokens' gradients only (the position-embedding
  // gradients then come from mmt_patch_embed_grad)
  const bool emb = drow_emb || dcol_emb;
  MMT_CHECK_ARG(NI == 0 || !emb || (img_rows && rtok && ctok && drow_emb && dcol_emb && Q > 0 &&
                                    2 * Q * EMB_COLS * 4 <= 160 * 1024),
                "mmt_seq_assemble_bwd: image embedding arguments");
  MMT_CHECK_ARG(NI == 0 || !emb || !g_det_host.fx || 2 * Q * EMB_COLS * 8 <= 160 * 1024,
                "mmt_seq_assemble_bwd: Q too large for the deterministic table");
  const int64_t n = (int64_t)B * L * (D / 8);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(seq_assemble_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, s, B, L, D,
                     row_src, (const float*)dx0, (bf16_t*)dtext, T, (bf16_t*)dimg, NI, rtok, ctok,
                     drow_emb, dcol_emb, dreadout_pe);
  MMT_CHECK_LAUNCH("mmt_seq_assemble_bwd");
  if (NI > 0 && emb) {
    launch_embed_table(dim3((D + EMB_COLS - 1) / EMB_COLS, EMB_SPLIT), s, B, L, D, NI, Q, img_rows,
                       (const float*)dx0, rtok, ctok, drow_emb, dcol_emb);
    MMT_CHECK_LAUNCH("mmt_seq_assemble_bwd(embedding grads)");
  }
  return MMT_OK;
}

extern "C" int mmt_patch_embed_grad(int B, int L, int D, int I, int Himg, int P, int Q,
                                    const int32_t* img_rows, const void* dx0, const int32_t* rtok,
                                    const int32_t* ctok, float* drow_emb, float* dcol_emb,
                                    mmt_stream_t stream) {
  MMT_CHECK_ARG(img_rows && dx0 && rtok && ctok && drow_emb && dcol_emb && B > 0 && L > 0 &&
                    D > 0 && D % 8 == 0 && I > 0 && P > 0 && Himg >= P && Himg % P == 0 && Q > 1,
                "mmt_patch_embed_grad: args");
  const int PPD = Himg / P;
  int wmax = 1;  // widest token window (host float arithmetic = patch_positions_kernel's)
  for (int w = 0; w < PPD; ++w) {
    auto q = [&](int v) { return (int)floorf(((float)v / (float)Himg) * (float)(Q - 1)); };
    wmax = std::max(wmax, q((w + 1) * P) - q(w * P));
  }
  hipStream_t s = as_stream(stream);
  const int chunks = (D + EMB_COLS - 1) / EMB_COLS;
  const int splits = std::max(1, std::min(B, 1024 / (PPD * chunks * 2)));
  const dim3 grid(PPD, chunks, 2 * splits);
#define EGW(WM)                                                                                   \
  hipLaunchKernelGGL(embed_grad_win_kernel<WM>, grid, dim3(256), 0, s, B, L, D, I, PPD, Himg, P, \
                     Q, splits, img_rows, (const float*)dx0, rtok, ctok, drow_emb, dcol_emb)
  if (wmax <= 8) EGW(8);
  else if (wmax <= 16) EGW(16);
  else {  // wide windows: the LDS-atomic table kernel
    const int NI = I * PPD * PPD;
    MMT_CHECK_ARG(2 * Q * EMB_COLS * (g_det_host.fx ? 8 : 4) <= 160 * 1024,
                  "mmt_patch_embed_grad: Q too large%s", g_det_host.fx ? " for the deterministic table" : "");
    launch_embed_table(dim3(chunks, EMB_SPLIT), s, B, L, D, NI, Q, img_rows, (const float*)dx0, rtok,
                       ctok, drow_emb, dcol_emb);
  }
#undef EGW
  MMT_CHECK_LAUNCH("mmt_patch_embed_grad");
  return MMT_OK;
}

extern "C" int mmt_rows_mean_fwd(const void* x, int64_t xs_b, int64_t xs_t, int B, int D,
                                 const int32_t* rows, int nrows, void* out, int64_t ld_out,
                                 mmt_stream_t stream) {
  MMT_CHECK_ARG(x && rows && out && B > 0 && nrows > 0, "mmt_rows_mean_fwd: args");
  hipLaunchKernelGGL(rows_mean_fwd_kernel, dim3(B), dim3(256), 0, as_stream(stream),
                     (const float*)x, xs_b, xs_t, D, rows, nrows, (bf16_t*)out, ld_out);
  MMT_CHECK_LAUNCH("mmt_rows_mean_fwd");
  return MMT_OK;
}

extern "C" int mmt_rows_mean_bwd(const void* de, int64_t ld_de, int B, int L, int D,
                                 const int32_t* row_flag, int nrows, void* dx, mmt_stream_t stream) {
  MMT_CHECK_ARG(de && row_flag && dx && B > 0 && nrows > 0, "mmt_rows_mean_bwd: args");
  const int64_t n = (int64_t)B * L * D;
  hipLaunchKernelGGL(rows_mean_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)de, ld_de, B, L, D, row_flag, nrows, (float*)dx);
  MMT_CHECK_LAUNCH("mmt_rows_mean_bwd");
  return MMT_OK;
}

extern "C" int mmt_rows_group_mean_fwd(const void* x, int64_t xs_b, int64_t xs_t, int B, int L,
                                       int D, const int32_t* row_group, int G,
                                       const int32_t* counts, void* out, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && row_group && counts && out && B > 0 && L > 0 && D > 0 && G > 0,
                "mmt_rows_group_mean_fwd: args");
  hipLaunchKernelGGL(rows_group_mean_fwd_kernel, dim3(B, G), dim3(256), 0, as_stream(stream),
                     (const float*)x, xs_b, xs_t, L, D, row_group, G, counts, (bf16_t*)out);
  MMT_CHECK_LAUNCH("mmt_rows_group_mean_fwd");
  return MMT_OK;
}

extern "C" int mmt_rows_group_mean_bwd(const void* de, int B, int L, int D, const int32_t* row_group,
                                       int G, const int32_t* counts, void* dx, mmt_stream_t stream) {
  MMT_CHECK_ARG(de && row_group && counts && dx && B > 0 && L > 0 && D > 0 && G > 0,
                "mmt_rows_group_mean_bwd: args");
  const int64_t n = (int64_t)B * L * D;
  hipLaunchKernelGGL(rows_group_mean_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     as_stream(stream), (const bf16_t*)de, B, L, D, row_group, G, counts,
                     (float*)dx);
  MMT_CHECK_LAUNCH("mmt_rows_group_mean_bwd");
  return MMT_OK;
}

extern "C" int mmt_action_head(int kind, const float* z, int64_t ldz, int R, int N, const float* y,
                               const float* edges, int n_edges, float max_action, float inv_count,
                               float* pred, float* loss, void* dz, mmt_stream_t stream) {
  MMT_CHECK_ARG(z && R > 0 && N > 0 && ldz >= N && (kind == 0 || kind == 1),
                "mmt_action_head: args");
  MMT_CHECK_ARG(!y || (loss && dz), "mmt_action_head: a loss needs loss and dz outputs");
  MMT_CHECK_ARG(kind == 0 ? (max_action > 0.f && (y || pred)) : (y && edges && n_edges > 1),
                "mmt_action_head: kind %d arguments", kind);
  hipLaunchKernelGGL(action_head_kernel, dim3((R + 3) / 4), dim3(256), 0, as_stream(stream), kind,
                     z, ldz, R, N, y, edges, n_edges, max_action, inv_count, pred, loss,
                     (bf16_t*)dz);
  MMT_CHECK_LAUNCH("mmt_action_head");
  return MMT_OK;
}

extern "C" int mmt_transpose_bf16_batched(const void* src, void* dst, const int64_t* desc, int n,
                                          int64_t total_tiles, mmt_stream_t stream) {
  MMT_CHECK_ARG(src && dst && desc && n > 0 && total_tiles > 0, "mmt_transpose_bf16_batched: args");
  const int grid = (int)std::min<int64_t>(total_tiles, 4096);
  hipLaunchKernelGGL(transpose_bf16_batched_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)src, (bf16_t*)dst, desc, n, total_tiles);
  MMT_CHECK_LAUNCH("mmt_transpose_bf16_batched");
  return MMT_OK;
}

extern "C" int mmt_diffusion_prep(const uint32_t* rng, int B, int A, int steps,
                                  int64_t sample_offset, const float* actions,
                                  const float* alpha_hats, const float* fourier_w, int F,
                                  const int32_t* t_in, const float* eps_in, int32_t* t_out,
                                  float* eps_out, void* cat, int64_t ld_cat, void* feats,
                                  mmt_stream_t stream) {
  MMT_CHECK_ARG(actions && alpha_hats && fourier_w && t_out && eps_out && cat && feats && B > 0,
                "mmt_diffusion_prep: args");
  MMT_CHECK_ARG((t_in && eps_in) || rng, "mmt_diffusion_prep: need rng or injected (t, eps)");
  hipLaunchKernelGGL(diffusion_prep_kernel, dim3(B), dim3(256), 0, as_stream(stream), rng, B, A,
                     steps, sample_offset, actions, alpha_hats, fourier_w, F, t_in, eps_in, t_out,
                     eps_out, (bf16_t*)cat, ld_cat, (bf16_t*)feats);
  MMT_CHECK_LAUNCH("mmt_diffusion_prep");
  return MMT_OK;
}

extern "C" int mmt_fourier_bwd(const void* dfeats, int B, int F, const int32_t* t,
                               const float* fourier_w, float* dw, mmt_stream_t stream) {
  MMT_CHECK_ARG(dfeats && t && fourier_w && dw && B > 0 && F > 0, "mmt_fourier_bwd: args");
  hipLaunchKernelGGL(fourier_bwd_kernel, dim3((F + 63) / 64, (B + FB_B - 1) / FB_B), dim3(64), 0,
                     as_stream(stream),
                     (const bf16_t*)dfeats, B, F, t, fourier_w, dw);
  MMT_CHECK_LAUNCH("mmt_fourier_bwd");
  return MMT_OK;
}

extern "C" int mmt_diffusion_loss(const float* pred, int64_t ld_pred, const float* eps, int B,
                                  int A, float grad_scale, float* loss, void* dpred,
                                  mmt_stream_t stream) {
  MMT_CHECK_ARG(pred && eps && loss && dpred && B > 0 && A > 0, "mmt_diffusion_loss: args");
  hipLaunchKernelGGL(diffusion_loss_kernel, dim3(1), dim3(1024), 0, as_stream(stream), pred,
                     ld_pred, eps, B, A, grad_scale, loss, (bf16_t*)dpred);
  MMT_CHECK_LAUNCH("mmt_diffusion_loss");
  return MMT_OK;
}

extern "C" int mmt_rmsnorm_fwd(const void* x, int64_t rows, int D, const void* w, float eps,
                               void* y, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && w && y && rows > 0 && D % 8 == 0, "mmt_rmsnorm_fwd: args");
  hipLaunchKernelGGL(rmsnorm_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)x, rows, D, (const bf16_t*)w, eps, (bf16_t*)y);
  MMT_CHECK_LAUNCH("mmt_rmsnorm_fwd");
  return MMT_OK;
}

extern "C" int mmt_embedding_gather(const int32_t* ids, int64_t n, int D, const void* table,
                                    int vocab, void* out, mmt_stream_t stream) {
  MMT_CHECK_ARG(ids && table && out && n > 0 && D % 8 == 0 && vocab > 0, "mmt_embedding_gather: args");
  const int64_t t = n * (D / 8);
  hipLaunchKernelGGL(embedding_gather_kernel, dim3((t + 255) / 256), dim3(256), 0,
                     as_stream(stream), ids, n, D, (const bf16_t*)table, vocab, (bf16_t*)out);
  MMT_CHECK_LAUNCH("mmt_embedding_gather");
  return MMT_OK;
}

extern "C" int mmt_adamw(float* p, const float* g, float* m, float* v, void* shadow_bf16,
                         int64_t n, const int32_t* state, double lr, double b1, double b2,
                         double eps, double wd, float grad_scale, mmt_stream_t stream) {
  MMT_CHECK_ARG(p && g && m && v && state && n > 0, "mmt_adamw: args");
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 256 * 8);
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), p, g, m, v,
                     (bf16_t*)shadow_bf16, n, state, (float)lr, b1, b2, (float)eps, (float)wd,
                     grad_scale);
  MMT_CHECK_LAUNCH("mmt_adamw");
  return MMT_OK;
}

extern "C" int mmt_cast_f32_bf16(const float* a, void* b, int64_t n, mmt_stream_t stream) {
  MMT_CHECK_ARG(a && b && n > 0, "mmt_cast_f32_bf16: args");
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 256 * 8);
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), a,
                     (bf16_t*)b, n);
  MMT_CHECK_LAUNCH("mmt_cast_f32_bf16");
  return MMT_OK;
}

extern "C" int mmt_step_advance(int32_t* state, mmt_stream_t stream) {
  MMT_CHECK_ARG(state, "mmt_step_advance: null");
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, as_stream(stream), state);
  MMT_CHECK_LAUNCH("mmt_step_advance");
  return MMT_OK;
}

// AddPositionEmbedding (tokenizers/readout/readout.py:18-33, attention.py:71-85): out[b, l, :] =
// x[b, l, :] + pe[l, :] (fp32, float4 lanes; x may alias out). The backward is the identity for x
// and mmt_colsum over the batch for pe.
__global__ void add_pe_kernel(const float4* __restrict__ x, const float4* __restrict__ pe,
                              float4* __restrict__ out, int64_t n4, int64_t per4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 a = x[i], p = pe[i % per4];
    out[i] = make_float4(a.x + p.x, a.y + p.y, a.z + p.z, a.w + p.w);
  }
}

extern "C" int mmt_add_position_embedding(const float* x, const float* pe, float* out, int B, int L,
                                          int D, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && pe && out && B > 0 && L > 0 && D > 0 && D % 4 == 0 &&
                    (uintptr_t)x % 16 == 0 && (uintptr_t)pe % 16 == 0 && (uintptr_t)out % 16 == 0,
                "mmt_add_position_embedding: args (D %% 4 == 0, 16-B aligned)");
  const int64_t per4 = (int64_t)L * D / 4, n4 = per4 * B;
  const int64_t blocks = std::min<int64_t>((n4 + 255) / 256, 256 * 8);
  hipLaunchKernelGGL(add_pe_kernel, dim3(blocks), dim3(256), 0, as_stream(stream),
                     (const float4*)x, (const float4*)pe, (float4*)out, n4, per4);
  MMT_CHECK_LAUNCH("mmt_add_position_embedding");
  return MMT_OK;
}

namespace mmt {
int det_set_glue(const DetState& st) { return det_set_unit(st); }
}  // namespace mmt

extern "C" int mmt_det_flush(float* grad, long long* fx, int64_t n, mmt_stream_t stream) {
  MMT_CHECK_ARG(grad && fx && n >= 0, "mmt_det_flush: args");
  if (n == 0) return MMT_OK;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(det_flush_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), grad, fx, n);
  MMT_CHECK_LAUNCH("mmt_det_flush");
  return MMT_OK;
}

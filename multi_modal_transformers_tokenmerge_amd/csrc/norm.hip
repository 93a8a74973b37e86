// Sequence-axis LayerNorm, column reductions and dropout backward for gfx950.
//
// seqnorm: flax.linen.LayerNorm(reduction_axes=[1], feature_axes=[-1]) as configured by the
// reference (model_configs/attention_blocks/vanilla_decoder.yaml:5-13, used twice per block in
// attention.py:58,66): statistics over the SEQUENCE axis per (batch, feature), fast variance
// max(0, E[x^2] - E[x]^2), y = (x - mean) * (rsqrt(var + eps) * scale) + bias.
// x is (B, L, D) token-major, so a column reduction over L: each workgroup owns 64 features of
// one sample; 8 lanes x 8 elements cover the 64 columns, 32 row groups stride over L (coalesced
// row segments), partial sums meet in LDS. The second pass re-reads the panel (L2-hot).
//
// Precision: a sequence-axis LayerNorm subtracts each feature's mean over the tokens, which in
// this architecture is large next to the per-token deviations (attention outputs are averages
// over the sequence). The residual stream x and its gradient are therefore fp32 (x_dtype /
// res_dtype = MMT_F32 on the training path); y is emitted in bf16 for the MFMA GEMMs.
#include <algorithm>
#include <type_traits>

#include "common.h"

using namespace mmt;

namespace {

constexpr int CW = 64;   // columns per workgroup
constexpr int RG = 32;   // row groups
constexpr int NT = 256;  // = 8 column vectors x RG

__device__ __forceinline__ void load8(const bf16_t* p, float* f) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = __uint_as_float(w[q] << 16);
    f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ void unpack8(const uint4 u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = __uint_as_float(w[q] << 16);
    f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ void load8(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void store8(bf16_t* p, const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = (uint32_t)f2bf(f[2 * q]) | ((uint32_t)f2bf(f[2 * q + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void store8(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}

template <int NV, int NTT = NT, int CWT = CW>
__device__ __forceinline__ void reduce_rows(float (*part)[8], float* red /*[NV][RGT][CWT]*/) {
  constexpr int CVN = CWT / 8, RGT = NTT / CVN;
  const int cv = threadIdx.x % CVN, rg = threadIdx.x / CVN;
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(v * RGT + rg) * CWT + cv * 8 + e] = part[v][e];
  __syncthreads();
  for (int i = threadIdx.x; i < NV * CWT; i += NTT) {
    const int v = i / CWT, c = i % CWT;
    float s = 0.f;
    for (int r = 0; r < RGT; ++r) s += red[(v * RGT + r) * CWT + c];
    red[(v * RGT) * CWT + c] = s;
  }
  __syncthreads();
}

// RPT > 0 (fp32 x, L <= 32 RPT): one read of x — each thread keeps its RPT rows in registers
// from the statistics pass to the normalisation pass, every load unconditional (row-clamped).
template <typename TX, int RPT = 0>
__global__ __launch_bounds__(NT) void seqnorm_fwd_kernel(
    const TX* __restrict__ x, int64_t xs_b, int64_t xs_t, int L, int D,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    bf16_t* __restrict__ y, int64_t ys_b, int64_t ys_t, float* __restrict__ mean_out,
    float* __restrict__ rstd_out) {
  __shared__ float red[2 * RG * CW];
  __shared__ float s_mul[CW], s_add[CW];
  const int b = ln_sample(), c0 = ln_colblk() * CW;
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = c0 + cv * 8;
  const bool cok = col < D;
  const TX* xb = x + (int64_t)b * xs_b + col;
  float part[2][8] = {};
  constexpr int RR = RPT > 0 ? RPT : 1;
  [[maybe_unused]] float rx[RR][8];
  if constexpr (RPT > 0) {
    if (cok) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) load8(xb + (int64_t)min(rg + j * RG, L - 1) * xs_t, rx[j]);
#pragma unroll
      for (int j = 0; j < RPT; ++j)
        if (rg + j * RG < L)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            part[0][e] += rx[j][e];
            part[1][e] += rx[j][e] * rx[j][e];
          }
    }
  } else if (cok) {
    for (int l = rg; l < L; l += RG) {
      float f[8];
      load8(xb + (int64_t)l * xs_t, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        part[0][e] += f[e];
        part[1][e] += f[e] * f[e];
      }
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
    s_add[threadIdx.x] = beta[c] - mu * mul;
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
  if constexpr (RPT > 0) {
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int l = rg + j * RG;
      if (l >= L) break;
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = rx[j][e] * mul[e] + add[e];
      store8(yb + (int64_t)l * ys_t, f);
    }
  } else {
    for (int l = rg; l < L; l += RG) {
      float f[8];
      load8(xb + (int64_t)l * xs_t, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = f[e] * mul[e] + add[e];
      store8(yb + (int64_t)l * ys_t, f);
    }
  }
}

// dx = rstd * (g - mean_L(g) - xhat * mean_L(g * xhat)),  g = dy * gamma  (+ optional addend)
// dgamma += sum_{b,l} dy * xhat ; dbeta += sum_{b,l} dy   (fp32 atomics, one per column per block)
// x, addend and dx share the residual dtype TX; dy has its own (TDY).
// DZ: also the dropout backward of the block BEFORE this LayerNorm's block (its MLP-output
// dropout, site 3, applied to this dx: z = keep ? dx / keep_prob : 0 in bf16, the colsum_kernel
// arithmetic) with its column sums (that block's Dense_1 bias gradient), so the block-input
// gradient is not read again by a separate dropout pass.
struct DropZ {
  const uint32_t* rng;
  uint32_t layer, site, thresh;
  float scale;
  int64_t row_offset;
  bf16_t* z;
  int64_t zs_b, zs_t;
  float* colsum;
};
// RPT > 0 (bf16 dy, fp32 x, L <= 32 RPT): single pass over HBM — each thread keeps its RPT rows
// of x (fp32) and dy (packed bf16) in registers from the statistics pass to the gradient pass
// (the two-pass form re-reads both: 1.43x the algorithmic bytes measured at B = 512).
template <typename TDY, typename TX, bool DZ = false, int RPT = 0, int NTT = NT, int CWT = CW>
__global__ __launch_bounds__(NTT) void seqnorm_bwd_kernel(
    const TDY* __restrict__ dy, int64_t ds_b, int64_t ds_t, const TX* __restrict__ x,
    int64_t xs_b, int64_t xs_t, int L, int D, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma, const TX* addend,
    int64_t as_b, int64_t as_t, TX* dx, int64_t dxs_b, int64_t dxs_t,
    float* __restrict__ dgamma, float* __restrict__ dbeta, DropZ dz = DropZ{}) {
  constexpr int CVN = CWT / 8, RGT = NTT / CVN;  // column vectors, row groups
  __shared__ float red[4 * RGT * CWT];
  const int b = ln_sample(), c0 = ln_colblk() * CWT;
  const int cv = threadIdx.x % CVN, rg = threadIdx.x / CVN;
  const int col = c0 + cv * 8;
  const bool cok = col < D;
  float mu[8], rs[8], ga[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = cok ? mean[(int64_t)b * D + col + e] : 0.f;
    rs[e] = cok ? rstd[(int64_t)b * D + col + e] : 0.f;
    ga[e] = cok ? gamma[col + e] : 0.f;
  }
  const TX* xb = x + (int64_t)b * xs_b + col;
  const TDY* db = dy + (int64_t)b * ds_b + col;
  float part[4][8] = {};  // sum g, sum g*xhat, sum dy*xhat, sum dy
  constexpr int RR = RPT > 0 ? RPT : 1;
  [[maybe_unused]] float rx[RR][8];  // RPT: this thread's rows of x and dy, kept for pass 2
  [[maybe_unused]] uint4 rdy[RR];
  auto stat = [&](const float* fx, const float* fd) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (fx[e] - mu[e]) * rs[e];
      const float g = fd[e] * ga[e];
      part[0][e] += g;
      part[1][e] += g * xh;
      part[2][e] += fd[e] * xh;
      part[3][e] += fd[e];
    }
  };
  if constexpr (RPT > 0) {
    static_assert(std::is_same<TDY, bf16_t>::value && std::is_same<TX, float>::value, "RPT form");
    // every load unconditional (rows past L clamped, their dy zeroed: no contribution), so
    // they are all in flight together: a load under a per-row branch waits vmcnt(0) each
    if (cok) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int l = min(rg + j * RGT, L - 1);
        load8(xb + (int64_t)l * xs_t, rx[j]);
        rdy[j] = *reinterpret_cast<const uint4*>(db + (int64_t)l * ds_t);
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        if (rg + j * RGT >= L) rdy[j] = make_uint4(0u, 0u, 0u, 0u);
        float fd[8];
        unpack8(rdy[j], fd);
        stat(rx[j], fd);
      }
    }
  } else if (cok) {
    for (int l = rg; l < L; l += RGT) {
      float fx[8], fd[8];
      load8(xb + (int64_t)l * xs_t, fx);
      load8(db + (int64_t)l * ds_t, fd);
      stat(fx, fd);
    }
  }
  reduce_rows<4, NTT, CWT>(part, red);
  if (threadIdx.x < CWT && c0 + threadIdx.x < D) {
    grad_add(dgamma + c0 + threadIdx.x, red[2 * RGT * CWT + threadIdx.x]);
    grad_add(dbeta + c0 + threadIdx.x, red[3 * RGT * CWT + threadIdx.x]);
  }
  // (threads past D skip the loop but stay for the DZ reduction's barriers)
  float mg[8], mgx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mg[e] = red[cv * 8 + e] / L;
    mgx[e] = red[RGT * CWT + cv * 8 + e] / L;
  }
  TX* dxb = dx + (int64_t)b * dxs_b + col;
  const TX* ab = addend ? addend + (int64_t)b * as_b + col : nullptr;
  [[maybe_unused]] float cs[8] = {};
  [[maybe_unused]] const uint32_t key = DZ && dz.rng ? stream_key(dz.rng[0], dz.rng[1], dz.layer, dz.site) : 0u;
#pragma unroll(RPT > 0 ? RPT : 1)
  for (int j = 0, l = rg; cok && (RPT > 0 ? j < RPT : l < L); ++j, l += RGT) {
    // RPT: a fixed trip count and unconditional (row-clamped) addend loads; only the stores of
    // rows past L are skipped
    const int la = RPT > 0 ? min(l, L - 1) : l;
    float fx[8], fd[8], fa[8];
    if constexpr (RPT > 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) fx[e] = rx[j][e];
      unpack8(rdy[j], fd);
    } else {
      load8(xb + (int64_t)l * xs_t, fx);
      load8(db + (int64_t)l * ds_t, fd);
    }
    if (ab) load8(ab + (int64_t)la * as_t, fa);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (fx[e] - mu[e]) * rs[e];
      const float g = fd[e] * ga[e];
      fx[e] = rs[e] * (g - mg[e] - xh * mgx[e]) + (ab ? fa[e] : 0.f);
    }
    if (RPT > 0 && l >= L) continue;
    store8(dxb + (int64_t)l * dxs_t, fx);
    if constexpr (DZ) {
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fx[e];  // the stored (TX) value
      if (dz.rng) {
        const int64_t m = (int64_t)b * L + l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t ctr = (uint32_t)((dz.row_offset + m) * (int64_t)D + col + e);
          f[e] = keep_elem(key, ctr, dz.thresh) ? f[e] * dz.scale : 0.f;
        }
      }
      store8(dz.z + (int64_t)b * dz.zs_b + (int64_t)l * dz.zs_t + col, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += f[e];
    }
  }
  if constexpr (DZ) {
    float p1[1][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) p1[0][e] = cs[e];
    __syncthreads();  // every thread has read mg / mgx out of red
    reduce_rows<1, NTT, CWT>(p1, red);
    if (dz.colsum && threadIdx.x < CWT && c0 + threadIdx.x < D)
      grad_add(dz.colsum + c0 + threadIdx.x, red[threadIdx.x]);
  }
}

// LayerNorm_1 backward + ToMe unmerge + the attention-output dropout backward of one block, fused
// (attention_blocks/attention.py backward: ln1.bwd -> tome_merge_bwd -> dropout_bwd(site 1)).
// One workgroup = one sample x 64 columns: pass 1 as seqnorm_bwd_kernel (x1, dy1 of the merged
// sequence; dgamma / dbeta), pass 2 computes the merged-layout input gradient (+ addend) into an
// LDS panel instead of HBM, pass 3 walks the L unmerged rows: g_in = (g[orow] * s) / S (the merge
// backward's arithmetic) or a copy, stored fp32, then z = keep ? g_in / keep_prob : 0 stored bf16
// with its column sums (the out-projection bias gradient). Same expressions as the three kernels
// (this file's compilation): bit-identical g_in, z and LN gradients; the column-sum atomics
// differ in order only.
// RPT > 0 (L2 <= 32 RPT): passes 1 and 2 read x1 / dy1 once, kept in registers (as the
// RPT form of seqnorm_bwd_kernel).
constexpr int kUnmergeMax = 512;  // unmerged rows per sample of the fused form
template <int RPT = 0, int CWT = CW>
__global__ __launch_bounds__(NT) void ln_unmerge_dropout_bwd_kernel(
    const bf16_t* __restrict__ dy, int64_t ds_b, int64_t ds_t, const float* __restrict__ x,
    int64_t xs_b, int64_t xs_t, int L2, int D, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma, const float* addend,
    int64_t as_b, int64_t as_t, float* __restrict__ dgamma, float* __restrict__ dbeta, int L,
    int set_start, int t, int r, const float* __restrict__ size_in,
    const float* __restrict__ size_out, const int32_t* __restrict__ pos_map,
    float* __restrict__ g_in, int64_t gs_b, int64_t gs_t, const uint32_t* __restrict__ rng,
    uint32_t layer, uint32_t site, uint32_t thresh, float scale, int64_t row_offset,
    bf16_t* __restrict__ z, int64_t zs_b, int64_t zs_t, float* __restrict__ bias_grad,
    unsigned int* fault) {
  extern __shared__ __attribute__((aligned(16))) float dyn_f[];  // [max(L2*CWT, 4*RGT*CWT)]
  constexpr int CVN = CWT / 8, RGT = NT / CVN;  // column vectors, row groups (seqnorm_bwd_kernel)
  __shared__ int32_t u_orow[kUnmergeMax];
  __shared__ float u_s[kUnmergeMax], u_S[kUnmergeMax];
  float* red = dyn_f;
  float* panel = dyn_f;  // reused after the reduction: merged-layout gradient [L2][CWT]
  const int b = ln_sample(), c0 = ln_colblk() * CWT;
  const int cv = threadIdx.x % CVN, rg = threadIdx.x / CVN;
  const int col = c0 + cv * 8;
  const bool cok = col < D;
  for (int row = threadIdx.x; row < L; row += NT) {  // merge-backward row sources
    if (row < set_start || row >= set_start + t) {
      u_orow[row] = row < set_start ? row : row - r;
      u_s[row] = -1.f;  // copy
    } else {
      const int tok = row - set_start;
      const int q = checked_index(pos_map[(int64_t)b * t + tok], t - r,
                                  ln_colblk() == 0 ? fault : nullptr, MMT_FAULT_POS_MAP);
      u_orow[row] = set_start + q;
      u_s[row] = size_in ? size_in[(int64_t)b * t + tok] : 1.f;
      u_S[row] = size_out ? size_out[(int64_t)b * (t - r) + q] : 1.f;
    }
  }
  float mu[8], rs[8], ga[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = cok ? mean[(int64_t)b * D + col + e] : 0.f;
    rs[e] = cok ? rstd[(int64_t)b * D + col + e] : 0.f;
    ga[e] = cok ? gamma[col + e] : 0.f;
  }
  const float* xb = x + (int64_t)b * xs_b + col;
  const bf16_t* db = dy + (int64_t)b * ds_b + col;
  float part[4][8] = {};  // pass 1 (seqnorm_bwd_kernel)
  constexpr int RR = RPT > 0 ? RPT : 1;
  [[maybe_unused]] float rx[RR][8];
  [[maybe_unused]] uint4 rdy[RR];
  auto stat = [&](const float* fx, const float* fd) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (fx[e] - mu[e]) * rs[e];
      const float g = fd[e] * ga[e];
      part[0][e] += g;
      part[1][e] += g * xh;
      part[2][e] += fd[e] * xh;
      part[3][e] += fd[e];
    }
  };
  if constexpr (RPT > 0) {
    // every load unconditional (rows past L2 clamped, their dy zeroed: no contribution), so
    // they are all in flight together: a load under a per-row branch waits vmcnt(0) each
    if (cok) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int l = min(rg + j * RGT, L2 - 1);
        load8(xb + (int64_t)l * xs_t, rx[j]);
        rdy[j] = *reinterpret_cast<const uint4*>(db + (int64_t)l * ds_t);
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        if (rg + j * RGT >= L2) rdy[j] = make_uint4(0u, 0u, 0u, 0u);
        float fd[8];
        unpack8(rdy[j], fd);
        stat(rx[j], fd);
      }
    }
  } else if (cok) {
    for (int l = rg; l < L2; l += RGT) {
      float fx[8], fd[8];
      load8(xb + (int64_t)l * xs_t, fx);
      load8(db + (int64_t)l * ds_t, fd);
      stat(fx, fd);
    }
  }
  reduce_rows<4, NT, CWT>(part, red);
  if (threadIdx.x < CWT && c0 + threadIdx.x < D) {
    grad_add(dgamma + c0 + threadIdx.x, red[2 * RGT * CWT + threadIdx.x]);
    grad_add(dbeta + c0 + threadIdx.x, red[3 * RGT * CWT + threadIdx.x]);
  }
  float mg[8], mgx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mg[e] = red[cv * 8 + e] / L2;
    mgx[e] = red[RGT * CWT + cv * 8 + e] / L2;
  }
  __syncthreads();  // red is read; the panel reuses it
  const float* ab = addend ? addend + (int64_t)b * as_b + col : nullptr;
#pragma unroll(RPT > 0 ? RPT : 1)
  for (int j = 0, l = rg; cok && (RPT > 0 ? j < RPT : l < L2); ++j, l += RGT) {  // pass 2: into LDS
      const int la = RPT > 0 ? min(l, L2 - 1) : l;
      float fx[8], fd[8], fa[8];
      if constexpr (RPT > 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) fx[e] = rx[j][e];
        unpack8(rdy[j], fd);
      } else {
        load8(xb + (int64_t)l * xs_t, fx);
        load8(db + (int64_t)l * ds_t, fd);
      }
      if (ab) load8(ab + (int64_t)la * as_t, fa);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (fx[e] - mu[e]) * rs[e];
        const float g = fd[e] * ga[e];
        fx[e] = rs[e] * (g - mg[e] - xh * mgx[e]) + (ab ? fa[e] : 0.f);
      }
      if (RPT > 0 && l >= L2) continue;  // rows past L2: no panel row
      store8(panel + l * CWT + cv * 8, fx);
    }
  __syncthreads();
  // pass 3: unmerge (tome_merge_bwd_kernel), dropout backward (colsum_kernel), column sums
  const uint32_t key = rng ? stream_key(rng[0], rng[1], layer, site) : 0u;
  float cs[8] = {};
  if (cok)
    for (int row = rg; row < L; row += RGT) {
      float f[8];
      load8(panel + u_orow[row] * CWT + cv * 8, f);
      const float sv = u_s[row];
      if (sv >= 0.f) {
        const float S = u_S[row];
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = (f[e] * sv) / S;
      }
      store8(g_in + (int64_t)b * gs_b + (int64_t)row * gs_t + col, f);
      if (rng) {
        const int64_t m = (int64_t)b * L + row;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t ctr = (uint32_t)((row_offset + m) * (int64_t)D + col + e);
          f[e] = keep_elem(key, ctr, thresh) ? f[e] * scale : 0.f;
        }
      }
      store8(z + (int64_t)b * zs_b + (int64_t)row * zs_t + col, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += f[e];
    }
  __syncthreads();  // the panel is read; reduce the column sums in its place
  float part1[1][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) part1[0][e] = cs[e];
  reduce_rows<1, NT, CWT>(part1, red);
  if (bias_grad && threadIdx.x < CWT && c0 + threadIdx.x < D)
    grad_add(bias_grad + c0 + threadIdx.x, red[threadIdx.x]);
}

// out[n] += sum_m x[m][n]  and, with z != NULL, z = x * keep / keep_prob (keep = 1 when rng is
// NULL: a cast to bf16) written first — the dropout backward of a GEMM-epilogue dropout, whose
// column sum is the bias gradient.
constexpr int CS_ROWS = 256;
template <typename T>
__global__ __launch_bounds__(NT) void colsum_kernel(const T* __restrict__ x, int64_t ldx,
                                                    int M, int N, float* __restrict__ out,
                                                    const uint32_t* __restrict__ rng,
                                                    uint32_t layer, uint32_t site, uint32_t thresh,
                                                    float scale, int64_t row_offset,
                                                    bf16_t* __restrict__ z, int64_t ldz,
                                                    int rows_per) {
  __shared__ float red[RG * CW];
  const int c0 = blockIdx.x * CW, r0 = blockIdx.y * rows_per;
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = c0 + cv * 8;
  const bool cok = col < N;
  uint32_t key = 0;
  if (rng) key = stream_key(rng[0], rng[1], layer, site);
  float part[1][8] = {};
  if (cok)
    for (int m = r0 + rg; m < min(M, r0 + rows_per); m += RG) {
      float f[8];
      load8(x + (int64_t)m * ldx + col, f);
      if (rng) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t ctr = (uint32_t)((row_offset + m) * (int64_t)N + col + e);
          f[e] = keep_elem(key, ctr, thresh) ? f[e] * scale : 0.f;
        }
      }
      if (z) store8(z + (int64_t)m * ldz + col, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) part[0][e] += f[e];
    }
  if (!out) return;
  reduce_rows<1>(part, red);
  if (threadIdx.x < CW && c0 + threadIdx.x < N) grad_add(out + c0 + threadIdx.x, red[threadIdx.x]);
}

inline bool is_dt(int d) { return d == MMT_F32 || d == MMT_BF16; }

// rows per column-sum workgroup: CS_ROWS, fewer (down to RG) when that leaves the launch under
// ~512 workgroups (the bias-gradient slabs: 552 x 1536 floats gave 72 workgroups, 16 us)
inline int colsum_rows(int M, int N) {
  const int cb = (N + CW - 1) / CW;
  int r = CS_ROWS;
  while (r > RG && (int64_t)cb * ((M + r - 1) / r) < 512) r /= 2;
  return r;
}

}  // namespace

// rows per thread of the single-pass (register-resident) LayerNorm backward for L rows, 0 for the
// two-pass form (L > 320, or MMT_SNB_RPT=0)
static int snb_rpt(int L) {
  static const bool on = !getenv("MMT_SNB_RPT") || atoi(getenv("MMT_SNB_RPT")) != 0;
  if (!on) return 0;
  for (int r : {4, 6, 8, 10})
    if (L <= RG * r) return r;
  return 0;
}


extern "C" int mmt_seqnorm_fwd(const void* x, int x_dtype, int64_t xs_b, int64_t xs_t, int B,
                               int L, int D, const float* gamma, const float* beta, float eps,
                               void* y, int64_t ys_b, int64_t ys_t, float* mean, float* rstd,
                               mmt_stream_t stream) {
  MMT_CHECK_ARG(x && y && gamma && beta && mean && rstd, "mmt_seqnorm_fwd: null pointer");
  MMT_CHECK_ARG(is_dt(x_dtype), "mmt_seqnorm_fwd: x_dtype");
  MMT_CHECK_ARG(B > 0 && L > 0 && D > 0 && D % 8 == 0 && xs_t % 8 == 0 && ys_t % 8 == 0 &&
                    xs_b % 8 == 0 && ys_b % 8 == 0,
                "mmt_seqnorm_fwd: D and strides must be multiples of 8");
  const dim3 grid = ln_grid(B, (D + CW - 1) / CW);
  const int rpt = snb_rpt(L);
  if (x_dtype == MMT_F32 && rpt) {
#define SNF(R)                                                                                       \
  hipLaunchKernelGGL((seqnorm_fwd_kernel<float, R>), grid, dim3(NT), 0, as_stream(stream),          \
                     (const float*)x, xs_b, xs_t, L, D, gamma, beta, eps, (bf16_t*)y, ys_b, ys_t,    \
                     mean, rstd)
    if (rpt == 4) SNF(4);
    else if (rpt == 6) SNF(6);
    else if (rpt == 8) SNF(8);
    else SNF(10);
#undef SNF
  } else if (x_dtype == MMT_F32)
    hipLaunchKernelGGL(seqnorm_fwd_kernel<float>, grid, dim3(NT), 0, as_stream(stream),
                       (const float*)x, xs_b, xs_t, L, D, gamma, beta, eps, (bf16_t*)y, ys_b, ys_t,
                       mean, rstd);
  else
    hipLaunchKernelGGL(seqnorm_fwd_kernel<bf16_t>, grid, dim3(NT), 0, as_stream(stream),
                       (const bf16_t*)x, xs_b, xs_t, L, D, gamma, beta, eps, (bf16_t*)y, ys_b, ys_t,
                       mean, rstd);
  MMT_CHECK_LAUNCH("mmt_seqnorm_fwd");
  return MMT_OK;
}

extern "C" int mmt_seqnorm_bwd(const void* dy, int dy_dtype, int64_t ds_b, int64_t ds_t,
                               const void* x, int x_dtype, int64_t xs_b, int64_t xs_t, int B,
                               int L, int D, const float* mean, const float* rstd,
                               const float* gamma, const void* addend, int64_t as_b, int64_t as_t,
                               void* dx, int64_t dxs_b, int64_t dxs_t, float* dgamma, float* dbeta,
                               mmt_stream_t stream) {
  MMT_CHECK_ARG(dy && x && mean && rstd && gamma && dx && dgamma && dbeta,
                "mmt_seqnorm_bwd: null pointer");
  MMT_CHECK_ARG(is_dt(dy_dtype) && is_dt(x_dtype), "mmt_seqnorm_bwd: dtypes");
  MMT_CHECK_ARG(B > 0 && L > 0 && D > 0 && D % 8 == 0 && ds_t % 8 == 0 && xs_t % 8 == 0 &&
                    dxs_t % 8 == 0 && (!addend || as_t % 8 == 0),
                "mmt_seqnorm_bwd: D and strides must be multiples of 8");
  const dim3 grid = ln_grid(B, (D + CW - 1) / CW);
  hipStream_t s = as_stream(stream);
#define SNB(TDY, TX)                                                                             \
  hipLaunchKernelGGL((seqnorm_bwd_kernel<TDY, TX>), grid, dim3(NT), 0, s, (const TDY*)dy, ds_b, \
                     ds_t, (const TX*)x, xs_b, xs_t, L, D, mean, rstd, gamma, (const TX*)addend,  \
                     as_b, as_t, (TX*)dx, dxs_b, dxs_t, dgamma, dbeta)
  const int rpt = snb_rpt(L);
  if (dy_dtype == MMT_BF16 && x_dtype == MMT_F32 && rpt) {
#define SNBR(R)                                                                                     \
  hipLaunchKernelGGL((seqnorm_bwd_kernel<bf16_t, float, false, R>), grid, dim3(NT), 0, s,           \
                     (const bf16_t*)dy, ds_b, ds_t, (const float*)x, xs_b, xs_t, L, D, mean, rstd,  \
                     gamma, (const float*)addend, as_b, as_t, (float*)dx, dxs_b, dxs_t, dgamma, dbeta)
    if (rpt == 4) SNBR(4);
    else if (rpt == 6) SNBR(6);
    else if (rpt == 8) SNBR(8);
    else SNBR(10);
#undef SNBR
  } else if (dy_dtype == MMT_F32 && x_dtype == MMT_F32) SNB(float, float);
  else if (dy_dtype == MMT_BF16 && x_dtype == MMT_F32) SNB(bf16_t, float);
  else if (dy_dtype == MMT_F32 && x_dtype == MMT_BF16) SNB(float, bf16_t);
  else SNB(bf16_t, bf16_t);
#undef SNB
  MMT_CHECK_LAUNCH("mmt_seqnorm_bwd");
  return MMT_OK;
}

extern "C" int mmt_colsum(const void* x, int dtype, int64_t ldx, int M, int N, float* out,
                          mmt_stream_t stream) {
  MMT_CHECK_ARG(x && out && M > 0 && N > 0 && N % 8 == 0 && ldx % 8 == 0 && is_dt(dtype),
                "mmt_colsum: bad args");
  const int rows_per = colsum_rows(M, N);
  dim3 grid((N + CW - 1) / CW, (M + rows_per - 1) / rows_per);
  if (dtype == MMT_F32)
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(NT), 0, as_stream(stream), (const float*)x,
                       ldx, M, N, out, nullptr, 0u, 0u, 0u, 1.f, (int64_t)0, nullptr, (int64_t)0, rows_per);
  else
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(NT), 0, as_stream(stream),
                       (const bf16_t*)x, ldx, M, N, out, nullptr, 0u, 0u, 0u, 1.f, (int64_t)0,
                       nullptr, (int64_t)0, rows_per);
  MMT_CHECK_LAUNCH("mmt_colsum");
  return MMT_OK;
}

extern "C" int mmt_dropout_bwd(const void* dy, int dtype, int64_t ldy, int M, int N,
                               const uint32_t* rng, uint32_t layer, uint32_t site, float keep_prob,
                               int64_t row_offset, void* dz, int64_t ldz, float* colsum,
                               mmt_stream_t stream) {
  MMT_CHECK_ARG(dy && dz && M > 0 && N > 0 && N % 8 == 0 && ldy % 8 == 0 && ldz % 8 == 0 &&
                    is_dt(dtype),
                "mmt_dropout_bwd: bad args");
  MMT_CHECK_ARG(keep_prob > 0.f && keep_prob <= 1.f, "mmt_dropout_bwd: keep_prob");
  const int rows_per = colsum_rows(M, N);
  dim3 grid((N + CW - 1) / CW, (M + rows_per - 1) / rows_per);
  const uint32_t th = rng ? keep_threshold16(keep_prob) : 0u;
  const float sc = rng ? 1.f / keep_prob : 1.f;
  if (dtype == MMT_F32)
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(NT), 0, as_stream(stream), (const float*)dy,
                       ldy, M, N, colsum, rng, layer, site, th, sc, row_offset, (bf16_t*)dz, ldz, rows_per);
  else
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(NT), 0, as_stream(stream),
                       (const bf16_t*)dy, ldy, M, N, colsum, rng, layer, site, th, sc, row_offset,
                       (bf16_t*)dz, ldz, rows_per);
  MMT_CHECK_LAUNCH("mmt_dropout_bwd");
  return MMT_OK;
}

extern "C" int mmt_ln_unmerge_dropout_bwd(
    const void* dy, int64_t ds_b, int64_t ds_t, const float* x, int64_t xs_b, int64_t xs_t, int B,
    int L2, int D, const float* mean, const float* rstd, const float* gamma, const float* addend,
    int64_t as_b, int64_t as_t, float* dgamma, float* dbeta, int L, int set_start, int t, int r,
    const float* size_in, const float* size_out, const int32_t* pos_map, float* g_in, int64_t gs_b,
    int64_t gs_t, const uint32_t* rng, uint32_t layer, uint32_t site, float keep_prob,
    int64_t row_offset, void* z, int64_t zs_b, int64_t zs_t, float* bias_grad, mmt_stream_t stream) {
  MMT_CHECK_ARG(dy && x && mean && rstd && gamma && dgamma && dbeta && pos_map && g_in && z,
                "mmt_ln_unmerge_dropout_bwd: null pointer");
  MMT_CHECK_ARG(B > 0 && L2 > 0 && D > 0 && D % 8 == 0 && L == L2 + r && r > 0 && t >= 2 &&
                    set_start >= 0 && set_start + t <= L && L <= kUnmergeMax &&
                    L2 * CW * 4 <= 96 * 1024,
                "mmt_ln_unmerge_dropout_bwd: bad shape (L <= %d)", kUnmergeMax);
  MMT_CHECK_ARG(ds_t % 8 == 0 && xs_t % 8 == 0 && gs_t % 8 == 0 && zs_t % 8 == 0 &&
                    (!addend || as_t % 8 == 0),
                "mmt_ln_unmerge_dropout_bwd: strides must be multiples of 8");
  MMT_CHECK_ARG(!rng || (keep_prob > 0.f && keep_prob <= 1.f), "mmt_ln_unmerge_dropout_bwd: keep_prob");
  const int cwt = CW;
  const size_t dyn = sizeof(float) * (size_t)std::max(L2 * cwt, 4 * (NT / (cwt / 8)) * cwt);
  const dim3 grid = ln_grid(B, (D + cwt - 1) / cwt);
  const int rpt = snb_rpt(L2);
#define LUD(R, CWV)                                                                                 \
  do {                                                                                              \
    static const bool attr_ = (hipFuncSetAttribute((const void*)ln_unmerge_dropout_bwd_kernel<R, CWV>, \
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                                   96 * 1024), true);                               \
    (void)attr_;                                                                                    \
    hipLaunchKernelGGL((ln_unmerge_dropout_bwd_kernel<R, CWV>), grid, dim3(NT), dyn, as_stream(stream), \
                       (const bf16_t*)dy, ds_b, ds_t, x, xs_b, xs_t, L2, D, mean, rstd, gamma,      \
                       addend, as_b, as_t, dgamma, dbeta, L, set_start, t, r, size_in, size_out,    \
                       pos_map, g_in, gs_b, gs_t, rng, layer, site,                                  \
                       rng ? keep_threshold16(keep_prob) : 0u, rng ? 1.f / keep_prob : 1.f,          \
                       row_offset, (bf16_t*)z, zs_b, zs_t, bias_grad, fault_word());                \
  } while (0)
  if (rpt == 4) LUD(4, CW);
  else if (rpt == 6) LUD(6, CW);
  else if (rpt == 8) LUD(8, CW);
  else if (rpt == 10) LUD(10, CW);
  else LUD(0, CW);
#undef LUD
  MMT_CHECK_LAUNCH("mmt_ln_unmerge_dropout_bwd");
  return MMT_OK;
}

extern "C" int mmt_seqnorm_dropout_bwd(const void* dy, int64_t ds_b, int64_t ds_t, const float* x,
                                       int64_t xs_b, int64_t xs_t, int B, int L, int D,
                                       const float* mean, const float* rstd, const float* gamma,
                                       const float* addend, int64_t as_b, int64_t as_t, float* dx,
                                       int64_t dxs_b, int64_t dxs_t, float* dgamma, float* dbeta,
                                       const uint32_t* rng, uint32_t layer, uint32_t site,
                                       float keep_prob, int64_t row_offset, void* z, int64_t zs_b,
                                       int64_t zs_t, float* colsum, mmt_stream_t stream) {
  MMT_CHECK_ARG(dy && x && mean && rstd && gamma && dx && dgamma && dbeta && z,
                "mmt_seqnorm_dropout_bwd: null pointer");
  MMT_CHECK_ARG(B > 0 && L > 0 && D > 0 && D % 8 == 0 && ds_t % 8 == 0 && xs_t % 8 == 0 &&
                    dxs_t % 8 == 0 && zs_t % 8 == 0 && (!addend || as_t % 8 == 0),
                "mmt_seqnorm_dropout_bwd: D and strides must be multiples of 8");
  MMT_CHECK_ARG(!rng || (keep_prob > 0.f && keep_prob <= 1.f), "mmt_seqnorm_dropout_bwd: keep_prob");
  DropZ dz{rng, layer, site, rng ? keep_threshold16(keep_prob) : 0u, rng ? 1.f / keep_prob : 1.f,
           row_offset, (bf16_t*)z, zs_b, zs_t, colsum};
  const dim3 grid = ln_grid(B, (D + CW - 1) / CW);
  const int rpt = snb_rpt(L);
#define SDZ(R)                                                                                      \
  hipLaunchKernelGGL((seqnorm_bwd_kernel<bf16_t, float, true, R>), grid, dim3(NT), 0,               \
                     as_stream(stream), (const bf16_t*)dy, ds_b, ds_t, x, xs_b, xs_t, L, D, mean,   \
                     rstd, gamma, addend, as_b, as_t, dx, dxs_b, dxs_t, dgamma, dbeta, dz)
  if (rpt == 4) SDZ(4);
  else if (rpt == 6) SDZ(6);
  else if (rpt == 8) SDZ(8);
  else if (rpt == 10) SDZ(10);
  else SDZ(0);
#undef SDZ
  MMT_CHECK_LAUNCH("mmt_seqnorm_dropout_bwd");
  return MMT_OK;
}

namespace mmt {
int det_set_norm(const DetState& st) { return det_set_unit(st); }
}  // namespace mmt

// Blockwise-causal multi-head attention for gfx950: flash-style forward and backward.
//
// Replaces flax.linen.SelfAttention's dot_product_attention as configured by the reference
// (model_configs/attention_blocks/vanilla_decoder.yaml:19-31; mask from
// tokenizers/token_sequencer.py:313-321 repeated over heads/batch, octo.py:66-68,119):
//   logits = (q / sqrt(Dh)) . k ; where(mask, logits, finfo.min) ; softmax (fp32) ;
//   attention dropout with ONE (L, L) keep-mask broadcast over batch and heads ; . v
// The (B, H, L, L) logits are never materialised. The mask is not a tensor either: it is the
// token-set table of the layer (set ranges + a bitmask of the key sets each query set sees), so
// fully invisible key tiles are skipped. T5 mode: an additive fp32 (H, L, L) bias, scale 1.
//
// Layout: qkv rows (b, t) hold [q(H, Dh) | k(H, Dh) | v(H, Dh)] (the fused QKV GEMM output);
// o rows (b, t) hold (H, Dh); lse / delta are (B, H, L) fp32.
//
// Forward and dQ: one wave = 32 queries ON THE LANES; S^T = K . Q^T so every score of a query is
// lane-local (registers) and the row max / sum need one cross-half exchange; the S^T accumulator
// is used directly as the B operand of O^T += V^T . P^T (no LDS round trip for P).
// dK/dV: one wave = 32 keys on the lanes; S = Q . K^T and dP = dO . V^T accumulators feed
// dV^T += dO^T . P and dK^T += Q^T . dS directly. V^T, dO^T, Q^T, K^T operands come from
// row-major LDS tiles through ds_read_b64_tr_b16.
#include <math.h>

#include "common.h"

using namespace mmt;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int MAX_SETS = 16;
constexpr int KT = 64;      // keys (or queries) per LDS tile
constexpr int NT = 256;     // threads per workgroup (4 waves x 32 rows)
constexpr int MAXL = 4096;  // LDS set-id table size

struct AttnMask {
  int n_sets;
  int start[MAX_SETS];
  int len[MAX_SETS];
  uint32_t vis[MAX_SETS];  // bit k: query set s sees key set k
};

__device__ __forceinline__ int set_of(const AttnMask& m, int t) {
  int s = 0;
#pragma unroll 1
  for (int i = 0; i < m.n_sets; ++i)
    if (t >= m.start[i]) s = i;
  return s;
}

// Any visible (query, key) pair for queries [q0, q1) x keys [k0, k1)?  (workgroup-uniform)
__device__ __forceinline__ bool tile_visible(const AttnMask& m, int q0, int q1, int k0, int k1) {
  uint32_t kmask = 0;
  for (int i = 0; i < m.n_sets; ++i)
    if (m.start[i] < k1 && m.start[i] + m.len[i] > k0 && m.len[i] > 0) kmask |= 1u << i;
  for (int i = 0; i < m.n_sets; ++i)
    if (m.start[i] < q1 && m.start[i] + m.len[i] > q0 && m.len[i] > 0 && (m.vis[i] & kmask))
      return true;
  return false;
}

__device__ __forceinline__ short4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)((__attribute__((address_space(3))) void*)p));
}

// A-operand fragment of X^T (rows = d) from a row-major LDS tile X[row][d] (stride STR):
// lane (d = dbase + lane&31, h = lane>>5), element j <-> row 16s + 8(j>>2) + 4h + (j&3) (the
// k order of an accumulator used as the next MFMA's operand).
template <int STR>
__device__ __forceinline__ bf16x8 trans_frag(const bf16_t* tile, int row_base, int dbase, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4, h = lane >> 5;
  const int col = dbase + 16 * (g & 1) + 4 * p;
  const int r1 = row_base + 4 * h + q;
  const short4v a = tr_read(tile + r1 * STR + col);
  const short4v b = tr_read(tile + (r1 + 8) * STR + col);
  short8v v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// A/B-operand fragment with the contraction dim contiguous in a row-major LDS tile X[row][d]:
// lane (row = rbase + lane&31, h), element j <-> d = 16s + 8h + j.
template <int STR>
__device__ __forceinline__ bf16x8 row_frag(const bf16_t* tile, int rbase, int s, int lane) {
  return *reinterpret_cast<const bf16x8*>(tile + (rbase + (lane & 31)) * STR + 16 * s +
                                          8 * (lane >> 5));
}

// Same fragment straight from global memory (rows beyond L read as zero).
__device__ __forceinline__ bf16x8 row_frag_global(const bf16_t* rowp, bool valid, int s, int lane) {
  if (!valid) return (bf16x8){};
  return *reinterpret_cast<const bf16x8*>(rowp + 16 * s + 8 * (lane >> 5));
}

// Pack accumulator registers 8s..8s+7 to a bf16 operand fragment.
__device__ __forceinline__ bf16x8 pack_frag(const floatx16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[8 * s + j];
  return r;
}

__device__ __forceinline__ int acc_row(int reg, int lane) {
  return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
}

// Cooperative copy of a KT x DH bf16 tile (rows r0.., clipped at L) into LDS [KT][DH+8].
template <int DH>
__device__ __forceinline__ void load_rows_to_lds(bf16_t* lds, const bf16_t* base, int64_t s_t,
                                                 int r0, int L) {
  constexpr int CPR = DH / 8;  // 16-B chunks per row
  for (int c = threadIdx.x; c < KT * CPR; c += NT) {
    const int row = c / CPR, ch = c % CPR;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + row < L) v = *reinterpret_cast<const uint4*>(base + (int64_t)(r0 + row) * s_t + ch * 8);
    *reinterpret_cast<uint4*>(lds + row * (DH + 8) + ch * 8) = v;
  }
}

struct Geo {
  const bf16_t* qkv;
  int64_t s_b, s_t;  // qkv strides (elements)
  int L, H;
  float scale;
};

// =============================================================================== forward
template <int DH>
__global__ __launch_bounds__(NT) void attn_fwd_kernel(Geo g, AttnMask mask,
                                                      const uint32_t* __restrict__ drop_bits,
                                                      int drop_words, float drop_scale,
                                                      const float* __restrict__ bias,
                                                      bf16_t* __restrict__ o, int64_t o_s_b,
                                                      int64_t o_s_t, float* __restrict__ lse) {
  constexpr int STR = DH + 8;
  constexpr int NS = DH / 16;   // k-steps over the head dim
  constexpr int ND = DH / 32;   // 32-row d sub-tiles of O^T
  __shared__ __attribute__((aligned(16))) bf16_t Ks[KT * STR];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[KT * STR];
  __shared__ uint8_t kset[MAXL];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int L = g.L, D = g.H * DH;
  const int q0 = blockIdx.x * 128, q1 = min(L, q0 + 128);
  const int q = q0 + wave * 32 + (lane & 31);
  const bool qv = q < L;
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  const bf16_t* kbase = base + D + h * DH;
  const bf16_t* vbase = base + 2 * D + h * DH;
  for (int t = threadIdx.x; t < L; t += NT) kset[t] = (uint8_t)set_of(mask, t);

  bf16x8 qf[NS];
  const bf16_t* qrow = base + (int64_t)(qv ? q : 0) * g.s_t + h * DH;
#pragma unroll
  for (int s = 0; s < NS; ++s) qf[s] = row_frag_global(qrow, qv, s, lane);
  const uint32_t visq = mask.vis[set_of(mask, qv ? q : 0)];
  const float* brow = bias ? bias + ((int64_t)h * L + (qv ? q : 0)) * L : nullptr;

  floatx16 oacc[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const float sl2 = g.scale * 1.4426950408889634f;
  __syncthreads();

  for (int k0 = 0; k0 < L; k0 += KT) {
    if (!tile_visible(mask, q0, q1, k0, min(L, k0 + KT))) continue;
    load_rows_to_lds<DH>(Ks, kbase, g.s_t, k0, L);
    load_rows_to_lds<DH>(Vs, vbase, g.s_t, k0, L);
    __syncthreads();
    floatx16 sacc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[u][r] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s)
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Ks, 32 * u, s, lane),
                                                          qf[s], sacc[u], 0, 0, 0);
    }
    uint32_t dw0 = 0xffffffffu, dw1 = 0xffffffffu;
    if (drop_bits && qv) {
      dw0 = drop_bits[(int64_t)q * drop_words + (k0 >> 5)];
      if ((k0 >> 5) + 1 < drop_words) dw1 = drop_bits[(int64_t)q * drop_words + (k0 >> 5) + 1];
    }
    // scores (log2 domain), mask, running max
    float tmax = -INFINITY;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = k0 + 32 * u + acc_row(r, lane);
        float v = sacc[u][r] * sl2;
        if (brow && kk < L) v += brow[kk] * 1.4426950408889634f;
        const bool ok = kk < L && ((visq >> kset[kk < L ? kk : 0]) & 1u);
        v = ok ? v : -INFINITY;
        sacc[u][r] = v;
        tmax = fmaxf(tmax, v);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t dw = u ? dw1 : dw0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = (mn == -INFINITY) ? 0.f : exp2f(sacc[u][r] - mn);
        rs += p;
        const bool keep = (dw >> acc_row(r, lane)) & 1u;
        sacc[u][r] = keep ? p * drop_scale : 0.f;
      }
    }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = mn;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Vs, 32 * u + 16 * s, 32 * d, lane), pack_frag(sacc[u], s), oacc[d],
              0, 0, 0);
    }
    __syncthreads();
  }
  if (qv) {
    const float inv = 1.f / l;
    bf16_t* orow = o + (int64_t)b * o_s_b + (int64_t)q * o_s_t + h * DH;
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int dd = 32 * d + 8 * r4 + 4 * (lane >> 5);
        uint2 w;
        w.x = (uint32_t)f2bf(oacc[d][4 * r4] * inv) | ((uint32_t)f2bf(oacc[d][4 * r4 + 1] * inv) << 16);
        w.y = (uint32_t)f2bf(oacc[d][4 * r4 + 2] * inv) | ((uint32_t)f2bf(oacc[d][4 * r4 + 3] * inv) << 16);
        *reinterpret_cast<uint2*>(orow + dd) = w;
      }
    if (lane < 32) lse[((int64_t)b * g.H + h) * L + q] = m * 0.6931471805599453f + logf(l);
  }
}

// =============================================================================== bwd: delta
// delta[b, h, q] = sum_d dO * O  (fp32)
template <int DH>
__global__ void attn_bwd_delta_kernel(const bf16_t* __restrict__ o, int64_t o_s_b, int64_t o_s_t,
                                      const bf16_t* __restrict__ dout, int64_t d_s_b,
                                      int64_t d_s_t, int B, int L, int H,
                                      float* __restrict__ delta) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * H * L) return;
  const int q = idx % L, h = (idx / L) % H, b = idx / ((int64_t)L * H);
  const bf16_t* op = o + b * o_s_b + (int64_t)q * o_s_t + h * DH;
  const bf16_t* dp = dout + b * d_s_b + (int64_t)q * d_s_t + h * DH;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < DH; c += 8) {
    const uint4 a = *reinterpret_cast<const uint4*>(op + c);
    const uint4 d = *reinterpret_cast<const uint4*>(dp + c);
    const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc += __uint_as_float(aw[j] << 16) * __uint_as_float(dw[j] << 16);
      acc += __uint_as_float(aw[j] & 0xffff0000u) * __uint_as_float(dw[j] & 0xffff0000u);
    }
  }
  delta[idx] = acc;
}

// =============================================================================== bwd: dQ
template <int DH>
__global__ __launch_bounds__(NT) void attn_bwd_dq_kernel(Geo g, AttnMask mask,
                                                         const uint32_t* __restrict__ drop_bits,
                                                         int drop_words, float drop_scale,
                                                         const bf16_t* __restrict__ dout,
                                                         int64_t d_s_b, int64_t d_s_t,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ delta,
                                                         bf16_t* __restrict__ dqkv,
                                                         int64_t dq_s_b, int64_t dq_s_t) {
  constexpr int STR = DH + 8;
  constexpr int NS = DH / 16;
  constexpr int ND = DH / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[KT * STR];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[KT * STR];
  __shared__ uint8_t kset[MAXL];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int L = g.L, D = g.H * DH;
  const int q0 = blockIdx.x * 128, q1 = min(L, q0 + 128);
  const int q = q0 + wave * 32 + (lane & 31);
  const bool qv = q < L;
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  for (int t = threadIdx.x; t < L; t += NT) kset[t] = (uint8_t)set_of(mask, t);
  bf16x8 qf[NS], df[NS];
  const bf16_t* qrow = base + (int64_t)(qv ? q : 0) * g.s_t + h * DH;
  const bf16_t* drow = dout + (int64_t)b * d_s_b + (int64_t)(qv ? q : 0) * d_s_t + h * DH;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    qf[s] = row_frag_global(qrow, qv, s, lane);
    df[s] = row_frag_global(drow, qv, s, lane);
  }
  const uint32_t visq = mask.vis[set_of(mask, qv ? q : 0)];
  const int64_t row_bh = ((int64_t)b * g.H + h) * L;
  const float lse2 = qv ? lse[row_bh + q] * 1.4426950408889634f : INFINITY;
  const float dlt = qv ? delta[row_bh + q] : 0.f;
  const float sl2 = g.scale * 1.4426950408889634f;
  floatx16 dqacc[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) dqacc[d][r] = 0.f;
  __syncthreads();
  for (int k0 = 0; k0 < L; k0 += KT) {
    if (!tile_visible(mask, q0, q1, k0, min(L, k0 + KT))) continue;
    load_rows_to_lds<DH>(Ks, base + D + h * DH, g.s_t, k0, L);
    load_rows_to_lds<DH>(Vs, base + 2 * D + h * DH, g.s_t, k0, L);
    __syncthreads();
    uint32_t dw0 = 0xffffffffu, dw1 = 0xffffffffu;
    if (drop_bits && qv) {
      dw0 = drop_bits[(int64_t)q * drop_words + (k0 >> 5)];
      if ((k0 >> 5) + 1 < drop_words) dw1 = drop_bits[(int64_t)q * drop_words + (k0 >> 5) + 1];
    }
    floatx16 ds[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      floatx16 sacc, pacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[r] = 0.f;
        pacc[r] = 0.f;
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Ks, 32 * u, s, lane), qf[s],
                                                       sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Vs, 32 * u, s, lane), df[s],
                                                       pacc, 0, 0, 0);
      }
      const uint32_t dw = u ? dw1 : dw0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = 32 * u + acc_row(r, lane);
        const int kk = k0 + kr;
        const bool ok = kk < L && ((visq >> kset[kk < L ? kk : 0]) & 1u);
        const float p = ok ? exp2f(sacc[r] * sl2 - lse2) : 0.f;
        const float md = ((dw >> acc_row(r, lane)) & 1u) ? drop_scale : 0.f;
        ds[u][r] = p * (pacc[r] * md - dlt);
      }
    }
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          dqacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Ks, 32 * u + 16 * s, 32 * d, lane), pack_frag(ds[u], s), dqacc[d],
              0, 0, 0);
    __syncthreads();
  }
  if (qv) {
    bf16_t* orow = dqkv + (int64_t)b * dq_s_b + (int64_t)q * dq_s_t + h * DH;
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int dd = 32 * d + 8 * r4 + 4 * (lane >> 5);
        uint2 w;
        w.x = (uint32_t)f2bf(dqacc[d][4 * r4] * g.scale) |
              ((uint32_t)f2bf(dqacc[d][4 * r4 + 1] * g.scale) << 16);
        w.y = (uint32_t)f2bf(dqacc[d][4 * r4 + 2] * g.scale) |
              ((uint32_t)f2bf(dqacc[d][4 * r4 + 3] * g.scale) << 16);
        *reinterpret_cast<uint2*>(orow + dd) = w;
      }
  }
}

// =============================================================================== bwd: dK, dV
template <int DH>
__global__ __launch_bounds__(NT) void attn_bwd_dkdv_kernel(Geo g, AttnMask mask,
                                                           const uint32_t* __restrict__ drop_bits,
                                                           int drop_words, float drop_scale,
                                                           const bf16_t* __restrict__ dout,
                                                           int64_t d_s_b, int64_t d_s_t,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta,
                                                           bf16_t* __restrict__ dqkv,
                                                           int64_t dq_s_b, int64_t dq_s_t) {
  constexpr int STR = DH + 8;
  constexpr int NS = DH / 16;
  constexpr int ND = DH / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Qs[KT * STR];
  __shared__ __attribute__((aligned(16))) bf16_t Ds[KT * STR];
  __shared__ float s_lse[KT], s_dlt[KT];
  __shared__ uint32_t s_vis[KT];
  __shared__ uint32_t s_bits[KT][4];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int L = g.L, D = g.H * DH;
  const int kb0 = blockIdx.x * 128, kb1 = min(L, kb0 + 128);
  const int key = kb0 + wave * 32 + (lane & 31);
  const bool kv = key < L;
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  bf16x8 kf[NS], vf[NS];
  const bf16_t* krow = base + (int64_t)(kv ? key : 0) * g.s_t + D + h * DH;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = row_frag_global(krow, kv, s, lane);
    vf[s] = row_frag_global(krow + D, kv, s, lane);
  }
  const int kset_l = set_of(mask, kv ? key : 0);
  const int64_t row_bh = ((int64_t)b * g.H + h) * L;
  const float sl2 = g.scale * 1.4426950408889634f;
  floatx16 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dk[d][r] = 0.f;
      dv[d][r] = 0.f;
    }
  const int wbase = kb0 >> 5;  // first 32-key word of this block
  for (int q0 = 0; q0 < L; q0 += KT) {
    if (!tile_visible(mask, q0, min(L, q0 + KT), kb0, kb1)) continue;
    load_rows_to_lds<DH>(Qs, base + h * DH, g.s_t, q0, L);
    load_rows_to_lds<DH>(Ds, dout + (int64_t)b * d_s_b + h * DH, d_s_t, q0, L);
    for (int i = threadIdx.x; i < KT; i += NT) {
      const int qq = q0 + i;
      const bool ok = qq < L;
      s_lse[i] = ok ? lse[row_bh + qq] * 1.4426950408889634f : INFINITY;
      s_dlt[i] = ok ? delta[row_bh + qq] : 0.f;
      s_vis[i] = ok ? mask.vis[set_of(mask, qq)] : 0u;
    }
    for (int i = threadIdx.x; i < KT * 4; i += NT) {
      const int qi = i >> 2, w = i & 3, qq = q0 + qi;
      uint32_t bits = 0xffffffffu;
      if (drop_bits && qq < L && wbase + w < drop_words) bits = drop_bits[(int64_t)qq * drop_words + wbase + w];
      s_bits[qi][w] = bits;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {  // 32-query sub-tiles
      floatx16 sacc, pacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[r] = 0.f;
        pacc[r] = 0.f;
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Qs, 32 * u, s, lane), kf[s],
                                                       sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Ds, 32 * u, s, lane), vf[s],
                                                       pacc, 0, 0, 0);
      }
      floatx16 pd, dsv;
      const int kw = (wave * 32 + (lane & 31)) >> 5;   // word index within the block
      const int kb = (wave * 32 + (lane & 31)) & 31;   // bit within the word
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = 32 * u + acc_row(r, lane);
        const bool ok = kv && ((s_vis[qi] >> kset_l) & 1u);
        const float p = ok ? exp2f(sacc[r] * sl2 - s_lse[qi]) : 0.f;
        const float md = ((s_bits[qi][kw] >> kb) & 1u) ? drop_scale : 0.f;
        pd[r] = p * md;
        dsv[r] = p * (pacc[r] * md - s_dlt[qi]);
      }
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Ds, 32 * u + 16 * s, 32 * d, lane), pack_frag(pd, s), dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Qs, 32 * u + 16 * s, 32 * d, lane), pack_frag(dsv, s), dk[d], 0, 0, 0);
        }
    }
    __syncthreads();
  }
  if (kv) {
    bf16_t* krow_o = dqkv + (int64_t)b * dq_s_b + (int64_t)key * dq_s_t + D + h * DH;
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int dd = 32 * d + 8 * r4 + 4 * (lane >> 5);
        uint2 wk, wv;
        wk.x = (uint32_t)f2bf(dk[d][4 * r4] * g.scale) | ((uint32_t)f2bf(dk[d][4 * r4 + 1] * g.scale) << 16);
        wk.y = (uint32_t)f2bf(dk[d][4 * r4 + 2] * g.scale) | ((uint32_t)f2bf(dk[d][4 * r4 + 3] * g.scale) << 16);
        wv.x = (uint32_t)f2bf(dv[d][4 * r4]) | ((uint32_t)f2bf(dv[d][4 * r4 + 1]) << 16);
        wv.y = (uint32_t)f2bf(dv[d][4 * r4 + 2]) | ((uint32_t)f2bf(dv[d][4 * r4 + 3]) << 16);
        *reinterpret_cast<uint2*>(krow_o + dd) = wk;
        *reinterpret_cast<uint2*>(krow_o + D + dd) = wv;
      }
  }
}

// =============================================================================== dropout bits
__global__ void dropout_bits_kernel(const uint32_t* __restrict__ rng, uint32_t layer, uint32_t site,
                                    int rows, int cols, int words, uint32_t thresh,
                                    uint32_t* __restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)rows * words) return;
  const int r = idx / words, w = idx % words;
  const uint32_t key = stream_key(rng[0], rng[1], layer, site);
  uint32_t bits = 0;
  for (int j = 0; j < 32; ++j) {
    const int c = w * 32 + j;
    if (c < cols && keep_elem(key, (uint32_t)((int64_t)r * cols + c), thresh)) bits |= 1u << j;
  }
  out[idx] = bits;
}

int fill_mask(AttnMask& m, int n_sets, const int32_t* starts, const int32_t* lens,
              const uint32_t* vis, int L) {
  if (n_sets <= 0) {  // no mask: one set covering everything
    m.n_sets = 1;
    m.start[0] = 0;
    m.len[0] = L;
    m.vis[0] = 1u;
    return MMT_OK;
  }
  MMT_CHECK_ARG(n_sets <= MAX_SETS && starts && lens && vis, "attention: bad token-set table");
  m.n_sets = n_sets;
  int expect = 0;
  for (int i = 0; i < n_sets; ++i) {
    MMT_CHECK_ARG(starts[i] == expect && lens[i] >= 0, "attention: token sets must tile [0, L)");
    m.start[i] = starts[i];
    m.len[i] = lens[i];
    m.vis[i] = vis[i];
    expect += lens[i];
  }
  MMT_CHECK_ARG(expect == L, "attention: token sets cover %d of L=%d", expect, L);
  for (int i = n_sets; i < MAX_SETS; ++i) {
    m.start[i] = 1 << 30;
    m.len[i] = 0;
    m.vis[i] = 0;
  }
  return MMT_OK;
}

}  // namespace

#define ATTN_DISPATCH(DH_, ...)                                  \
  do {                                                           \
    if (Dh == 64) { constexpr int DH_ = 64; __VA_ARGS__; }       \
    else if (Dh == 128) { constexpr int DH_ = 128; __VA_ARGS__; } \
    else { MMT_CHECK_ARG(false, "attention: head dim %d unsupported (64, 128)", Dh); } \
  } while (0)

extern "C" int mmt_dropout_bits(const uint32_t* rng, uint32_t layer, uint32_t site, int rows,
                                int cols, float keep_prob, uint32_t* out, mmt_stream_t stream) {
  MMT_CHECK_ARG(rng && out && rows > 0 && cols > 0 && keep_prob > 0.f && keep_prob <= 1.f,
                "mmt_dropout_bits: bad args");
  const int words = (cols + 31) / 32;
  const int64_t n = (int64_t)rows * words;
  hipLaunchKernelGGL(dropout_bits_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     rng, layer, site, rows, cols, words, keep_threshold16(keep_prob), out);
  MMT_CHECK_LAUNCH("mmt_dropout_bits");
  return MMT_OK;
}

extern "C" int mmt_attn_fwd(const void* qkv, int64_t s_b, int64_t s_t, int B, int L, int H, int Dh,
                            float scale, int n_sets, const int32_t* set_start,
                            const int32_t* set_len, const uint32_t* set_vis,
                            const uint32_t* drop_bits, float keep_prob, const float* bias,
                            void* o, int64_t o_s_b, int64_t o_s_t, float* lse,
                            mmt_stream_t stream) {
  MMT_CHECK_ARG(qkv && o && lse, "mmt_attn_fwd: null pointer");
  MMT_CHECK_ARG(B > 0 && L > 0 && H > 0 && L <= MAXL, "mmt_attn_fwd: bad shape (L <= %d)", MAXL);
  MMT_CHECK_ARG(s_t % 8 == 0 && s_b % 8 == 0 && o_s_t % 4 == 0 && o_s_b % 4 == 0,
                "mmt_attn_fwd: strides must keep 16-B rows");
  MMT_CHECK_ARG(keep_prob > 0.f && keep_prob <= 1.f, "mmt_attn_fwd: keep_prob");
  AttnMask m;
  int rc = fill_mask(m, n_sets, set_start, set_len, set_vis, L);
  if (rc) return rc;
  Geo g{(const bf16_t*)qkv, s_b, s_t, L, H, scale};
  const int words = (L + 31) / 32;
  dim3 grid((L + 127) / 128, H, B);
  ATTN_DISPATCH(DH, hipLaunchKernelGGL(attn_fwd_kernel<DH>, grid, dim3(NT), 0, as_stream(stream),
                                       g, m, drop_bits, words, 1.f / keep_prob, bias, (bf16_t*)o,
                                       o_s_b, o_s_t, lse));
  MMT_CHECK_LAUNCH("mmt_attn_fwd");
  return MMT_OK;
}

extern "C" int mmt_attn_bwd(const void* qkv, int64_t s_b, int64_t s_t, int B, int L, int H, int Dh,
                            float scale, int n_sets, const int32_t* set_start,
                            const int32_t* set_len, const uint32_t* set_vis,
                            const uint32_t* drop_bits, float keep_prob, const void* o,
                            int64_t o_s_b, int64_t o_s_t, const void* dout, int64_t d_s_b,
                            int64_t d_s_t, const float* lse, float* delta, void* dqkv,
                            int64_t dq_s_b, int64_t dq_s_t, mmt_stream_t stream) {
  MMT_CHECK_ARG(qkv && o && dout && lse && delta && dqkv, "mmt_attn_bwd: null pointer");
  MMT_CHECK_ARG(B > 0 && L > 0 && H > 0 && L <= MAXL, "mmt_attn_bwd: bad shape");
  MMT_CHECK_ARG(s_t % 8 == 0 && d_s_t % 8 == 0 && dq_s_t % 4 == 0 && o_s_t % 8 == 0,
                "mmt_attn_bwd: strides must keep 16-B rows");
  MMT_CHECK_ARG(keep_prob > 0.f && keep_prob <= 1.f, "mmt_attn_bwd: keep_prob");
  AttnMask m;
  int rc = fill_mask(m, n_sets, set_start, set_len, set_vis, L);
  if (rc) return rc;
  Geo g{(const bf16_t*)qkv, s_b, s_t, L, H, scale};
  const int words = (L + 31) / 32;
  hipStream_t s = as_stream(stream);
  const int64_t nd = (int64_t)B * H * L;
  ATTN_DISPATCH(DH, hipLaunchKernelGGL(attn_bwd_delta_kernel<DH>, dim3((nd + 255) / 256), dim3(256),
                                       0, s, (const bf16_t*)o, o_s_b, o_s_t, (const bf16_t*)dout,
                                       d_s_b, d_s_t, B, L, H, delta));
  dim3 grid((L + 127) / 128, H, B);
  ATTN_DISPATCH(DH, hipLaunchKernelGGL(attn_bwd_dq_kernel<DH>, grid, dim3(NT), 0, s, g, m, drop_bits,
                                       words, 1.f / keep_prob, (const bf16_t*)dout, d_s_b, d_s_t,
                                       lse, delta, (bf16_t*)dqkv, dq_s_b, dq_s_t));
  ATTN_DISPATCH(DH, hipLaunchKernelGGL(attn_bwd_dkdv_kernel<DH>, grid, dim3(NT), 0, s, g, m,
                                       drop_bits, words, 1.f / keep_prob, (const bf16_t*)dout,
                                       d_s_b, d_s_t, lse, delta, (bf16_t*)dqkv, dq_s_b, dq_s_t));
  MMT_CHECK_LAUNCH("mmt_attn_bwd");
  return MMT_OK;
}

// ToMe (token merging) kernels for gfx950.
//
//   tome_match  — bipartite soft matching, reference tokenizers/token_compression.py:54-112
//   tome_merge  — merge_wavg fwd (token_compression.py:90-129) fused with the sequence gather
//   tome_unmerge— its backward (weighted gather)
//
// This file is compiled with -ffp-contract=off: the canonical arithmetic of DESIGN.md
// ("ToMe canonical arithmetic") is spelled out with explicit __fmaf_rn / __fsqrt_rn / __fdiv_rn
// and separate multiply / add roundings, so the int32 index outputs are bit-exact with
// oracle/tome_ref.c and the fp32 merge is bit-exact too.
#include <math.h>

#include "common.h"

using namespace mmt;

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

// jnp.argmax semantics: NaN is the maximum (first NaN wins), otherwise strict '>' with the lower
// index winning ties.
__device__ __forceinline__ bool argmax_better(float v, int j, float bv, int bj) {
  if (isnan(bv)) return isnan(v) && j < bj;
  if (isnan(v)) return true;
  return v > bv || (v == bv && j < bj);
}

// Total order used by lax.sort on floats (NaNs canonicalised and sorted last, -0 < +0).
__device__ __forceinline__ uint32_t sort_key(float v) {
  if (isnan(v)) return 0xffffffffu;
  uint32_t b = __float_as_uint(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ void ld8f(const bf16_t* p, float* f) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = __uint_as_float(w[q] << 16);
    f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld8f(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// m[0..7] += the 8 metric elements at p of every head, h ascending (fp32 adds, the canonical
// order). Loads go out 8 heads at a time from clamped addresses (branch-free, so all of them are
// in flight before the first add; a per-head load + add loop waited for every load in turn).
template <typename T>
__device__ __forceinline__ void head_sum(const T* p, int heads, int64_t s_h, float* m) {
  for (int h0 = 0; h0 < heads; h0 += 8) {
    float f[8][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) ld8f(p + (int64_t)min(h0 + u, heads - 1) * s_h, f[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (h0 + u < heads)
#pragma unroll
        for (int q = 0; q < 8; ++q) m[q] = m[q] + f[u][q];
  }
}

// The matching runs as three launches// The matching runs as three launches (all on the caller's stream, workspace from the caller):
//   norm  : m = sum_h metric (fp32, h ascending), m / ||m||_2 with ||m|| = sqrt of a sequential
//           fmaf chain over c (no eps, token_compression.py:72) -> A^ [n][ta][c], B^ [n][tb][c]
//           (the reference's a = m[::2], b = m[1::2], :73), every token row in parallel;
//   score : S = A^ B^T as k-ordered fmaf chains (:75), class/distill -inf (:77-80), first-index
//           argmax per a row (:82-83) -> node_max / node_idx [n][ta]; one workgroup per
//           (32 a rows, sample), the b rows streamed through LDS 4 tiles at a time;
//   rank  : edge_idx = argsort(node_max)[::-1] (:84) as a rank count, src/unm/dst (:86-88).
// Workspace: n*t*c fp32 (A^, B^) + n*ta (node_max fp32) + n*ta (node_idx int32).
constexpr int NORM_NT = 256;
constexpr int SCORE_NT = 256;
constexpr int RANK_NT = 512;

// Vector path: LPR lanes per token row, lane q of a row owns c-chunk q (8 elements). The norm's
// fmaf chain walks the chunks in order: chunk q continues from the partial sum of chunk q-1,
// passed along the row's lanes by a shuffle.
template <typename T, int LPR>
__global__ __launch_bounds__(NORM_NT) void tome_norm_vec_kernel(
    const T* __restrict__ metric, int n, int t, int heads, int c, int64_t s_n, int64_t s_t,
    int64_t s_h, float* __restrict__ An, float* __restrict__ Bn) {
  const int lane = threadIdx.x & 63;
  const int lr = lane % LPR, rbase = lane - lr;
  const int64_t row = ((int64_t)blockIdx.x * NORM_NT + threadIdx.x) / LPR;  // global token row
  const bool live = row < (int64_t)n * t;
  const int b = live ? (int)(row / t) : 0, tok = live ? (int)(row - (int64_t)b * t) : 0;
  const int nch = c / 8;
  const bool mine = live && lr < nch;
  float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (mine) head_sum(metric + (int64_t)b * s_n + (int64_t)tok * s_t + lr * 8, heads, s_h, m);
  float ss = 0.f;
  for (int j = 0; j < nch; ++j) {
    if (lr == j) {
#pragma unroll
      for (int q = 0; q < 8; ++q) ss = __fmaf_rn(m[q], m[q], ss);
    }
    ss = __shfl(ss, rbase + j, 64);
  }
  if (!mine) return;
  const float nrm = __fsqrt_rn(ss);
  const int ta = (t + 1) / 2, tb = t / 2;
  float* o = (tok & 1) ? Bn + ((int64_t)b * tb + (tok >> 1)) * c : An + ((int64_t)b * ta + (tok >> 1)) * c;
  o += lr * 8;
  float v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = __fdiv_rn(m[q], nrm);
  *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// Scalar path (any c, any strides): one thread per token row, two passes over its output row.
template <typename T>
__global__ __launch_bounds__(NORM_NT) void tome_norm_scalar_kernel(
    const T* __restrict__ metric, int n, int t, int heads, int c, int64_t s_n, int64_t s_t,
    int64_t s_h, float* __restrict__ An, float* __restrict__ Bn) {
  const int64_t row = (int64_t)blockIdx.x * NORM_NT + threadIdx.x;
  if (row >= (int64_t)n * t) return;
  const int b = (int)(row / t), tok = (int)(row - (int64_t)b * t);
  const int ta = (t + 1) / 2, tb = t / 2;
  float* o = (tok & 1) ? Bn + ((int64_t)b * tb + (tok >> 1)) * c : An + ((int64_t)b * ta + (tok >> 1)) * c;
  const T* p = metric + (int64_t)b * s_n + (int64_t)tok * s_t;
  float ss = 0.f;
  for (int k = 0; k < c; ++k) {
    float acc = 0.f;
    for (int h = 0; h < heads; ++h) acc = acc + ld_f32(p + (int64_t)h * s_h + k);
    o[k] = acc;
    ss = __fmaf_rn(acc, acc, ss);
  }
  const float nrm = __fsqrt_rn(ss);
  for (int k = 0; k < c; ++k) o[k] = __fdiv_rn(o[k], nrm);
}

__device__ __forceinline__ void keep_best(float v, int j, float& best, int& bidx) {
  if (j >= 0 && (bidx < 0 || argmax_better(v, j, best, bidx))) {
    best = v;
    bidx = j;
  }
}

// Stage rows [r0, r0 + 32) of a normalised half (rows >= nrows zero) into LDS [32][c+1].
__device__ __forceinline__ void stage_tile(const float* __restrict__ src, int r0, int nrows, int c,
                                           float* __restrict__ dst, int tid, int nthr) {
  const int cs = c + 1;
  const int per = 32 * c;
  for (int e = tid; e < per; e += nthr) {
    const int rr = e / c, k = e - rr * c;
    dst[rr * cs + k] = (r0 + rr < nrows) ? src[(int64_t)(r0 + rr) * c + k] : 0.f;
  }
}

template <bool MFMA>
__global__ __launch_bounds__(SCORE_NT) void tome_score_kernel(const float* __restrict__ An,
                                                              const float* __restrict__ Bn, int t,
                                                              int c, int flags, int nb_tiles,
                                                              float* __restrict__ nmax,
                                                              int32_t* __restrict__ nidx) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int it = blockIdx.x, b = blockIdx.y;
  const int ta = (t + 1) / 2, tb = t / 2;
  const int cs = c + 1;
  const int n_jt = (tb + 31) / 32;
  float* As = smem;                          // [32][cs]
  float* Bs = As + 32 * cs;                  // [nb_tiles][32][cs]
  float* pb = Bs + nb_tiles * 32 * cs;       // partials [8][32]
  int* pi = (int*)(pb + 8 * 32);
  const float* Ab = An + (int64_t)b * ta * c;
  const float* Bb = Bn + (int64_t)b * tb * c;
  const bool cls = flags & MMT_TOME_CLASS_TOKEN;
  const bool dis = flags & MMT_TOME_DISTILL_TOKEN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  stage_tile(Ab, it * 32, ta, c, As, threadIdx.x, SCORE_NT);
  float best = 0.f;
  int bidx = -1;
  for (int g = 0; g < n_jt; g += nb_tiles) {
    __syncthreads();  // previous group's reads of Bs are done (and As is staged)
    for (int w = 0; w < nb_tiles && g + w < n_jt; ++w)
      stage_tile(Bb, (g + w) * 32, tb, c, Bs + w * 32 * cs, threadIdx.x, SCORE_NT);
    __syncthreads();
    if (MFMA) {
      // S^T tile (32 b rows x 32 a cols) = b^ . a^T with v_mfma_f32_32x32x2_f32, whose result
      // is a k-ordered fmaf chain (f32 in / f32 accumulate, one rounding per step): a row on the
      // lane, b rows in the 16 accumulator registers, the argmax over j lane-local.
      const int jt = g + wave;
      if (wave < nb_tiles && jt < n_jt) {
        const int i = it * 32 + (lane & 31);
        const float* bp = As + (lane & 31) * cs + (lane >> 5);
        const float* ap = Bs + wave * 32 * cs + (lane & 31) * cs + (lane >> 5);
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        for (int s = 0; s < c / 2; ++s)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[2 * s], bp[2 * s], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int jj = jt * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
          if (jj >= tb) continue;
          float v = acc[q];
          if ((cls && i == 0) || (dis && jj == 0)) v = -INFINITY;
          keep_best(v, jj, best, bidx);
        }
      }
    } else {
      // VALU: thread (a row tid & 31, slice tid >> 5 of 8) walks the group's b rows with stride 8.
      const int ar = threadIdx.x & 31, sl = threadIdx.x >> 5;
      const int i = it * 32 + ar;
      const float* ap = As + ar * cs;
      const int rows = min(nb_tiles * 32, tb - g * 32);
      for (int jr = sl; jr < rows; jr += 8) {
        const float* bq = Bs + jr * cs;
        float acc = 0.f;
        for (int k = 0; k < c; ++k) acc = __fmaf_rn(ap[k], bq[k], acc);
        const int jj = g * 32 + jr;
        if ((cls && i == 0) || (dis && jj == 0)) acc = -INFINITY;
        keep_best(acc, jj, best, bidx);
      }
    }
  }
  // combine (argmax_better is a total order with index tie-break: order-free)
  if (MFMA) {
    const float ov = __shfl_xor(best, 32, 64);
    const int oi = __shfl_xor(bidx, 32, 64);
    keep_best(ov, oi, best, bidx);
    if (lane < 32) {
      pb[wave * 32 + lane] = best;
      pi[wave * 32 + lane] = bidx;
    }
  } else {
    pb[(threadIdx.x >> 5) * 32 + (threadIdx.x & 31)] = best;
    pi[(threadIdx.x >> 5) * 32 + (threadIdx.x & 31)] = bidx;
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int nparts = MFMA ? SCORE_NT / 64 : SCORE_NT / 32;
    float bb = 0.f;
    int bi = -1;
    for (int w = 0; w < nparts; ++w) keep_best(pb[w * 32 + threadIdx.x], pi[w * 32 + threadIdx.x], bb, bi);
    const int i = it * 32 + threadIdx.x;
    if (i < ta) {
      nmax[(int64_t)b * ta + i] = bb;
      nidx[(int64_t)b * ta + i] = bi;
    }
  }
}

// Fused match, one 1024-thread workgroup per sample, when both normalised halves fit in LDS (t <=
// 512 at c = 64; every OCTO-small/base layer): (1) the per-token head sums and normalisation (the
// arithmetic of tome_norm_vec_kernel) are written straight into LDS; (2) the (a tile, b tile)
// pairs are spread over the 16 waves, each running the k-ordered f32 MFMA chain and first-index
// argmax of tome_score_kernel, partial maxima per (b tile, a row) in LDS, combined per a row
// (argmax_better is a total order: the combination order does not matter); (3) the rank sort of
// tome_rank_kernel and the src / dst / unm outputs. K is read from the QKV buffer once; nothing
// round-trips through HBM and the three launches become one.
constexpr int FUSED_NT = 1024;
__host__ __device__ __forceinline__ size_t fused_match_lds(int t, int c) {
  const int ta = (t + 1) / 2, tb = t / 2;
  const int pa = (ta + 31) / 32 * 32, pbr = (tb + 31) / 32 * 32;
  return sizeof(float) * (size_t)(pa + pbr) * (c + 1)   // normalised halves
         + (size_t)(pbr / 32) * pa * 8                  // partial (max, idx) per (b tile, a row)
         + (size_t)ta * 12;                             // node max / idx / rank slot
}
template <typename T, int LPR>
__global__ __launch_bounds__(FUSED_NT) void tome_match_fused_kernel(
    const T* __restrict__ metric, int t, int heads, int c, int64_t s_n, int64_t s_t, int64_t s_h,
    int r, int flags, int32_t* __restrict__ unm_idx, int32_t* __restrict__ src_idx,
    int32_t* __restrict__ dst_idx, float* __restrict__ node_max_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x;
  const int ta = (t + 1) / 2, tb = t / 2, cs = c + 1;
  const int pa = (ta + 31) / 32 * 32, pbr = (tb + 31) / 32 * 32;
  const int n_at = pa / 32, n_bt = pbr / 32;
  float* As = smem;                                   // [pa][cs]
  float* Bs = As + pa * cs;                           // [pbr][cs]
  float* pmax = Bs + pbr * cs;                        // [n_bt][pa]
  int* pidx = reinterpret_cast<int*>(pmax + n_bt * pa);
  float* nm = reinterpret_cast<float*>(pidx + n_bt * pa);   // [ta]
  int* ni = reinterpret_cast<int*>(nm + ta);                // [ta]
  uint32_t* keys = reinterpret_cast<uint32_t*>(ni + ta);    // [ta] (reused as edge[] after)
  for (int e = threadIdx.x; e < (pa - ta) * cs; e += FUSED_NT) As[ta * cs + e] = 0.f;
  for (int e = threadIdx.x; e < (pbr - tb) * cs; e += FUSED_NT) Bs[tb * cs + e] = 0.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // (1) head sum + L2 normalisation into LDS
  const int lr = lane % LPR, rbase = lane - lr;
  const int nch = c / 8;
  const T* mb = metric + (int64_t)b * s_n;
  for (int r0 = 0; r0 < t; r0 += FUSED_NT / LPR) {  // uniform trip count: the shuffles below
    const int tok = r0 + threadIdx.x / LPR;
    const bool mine = tok < t && lr < nch;
    float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (mine) head_sum(mb + (int64_t)tok * s_t + lr * 8, heads, s_h, m);
    float ss = 0.f;
    for (int j = 0; j < nch; ++j) {
      if (lr == j) {
#pragma unroll
        for (int q = 0; q < 8; ++q) ss = __fmaf_rn(m[q], m[q], ss);
      }
      ss = __shfl(ss, rbase + j, 64);
    }
    if (mine) {
      const float nrm = __fsqrt_rn(ss);
      float* o = ((tok & 1) ? Bs : As) + (tok >> 1) * cs + lr * 8;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = __fdiv_rn(m[q], nrm);
    }
  }
  __syncthreads();
  // (2) scores: (a tile, b tile) pairs over the waves
  const bool cls = flags & MMT_TOME_CLASS_TOKEN;
  const bool dis = flags & MMT_TOME_DISTILL_TOKEN;
  for (int pr = wave; pr < n_at * n_bt; pr += FUSED_NT / 64) {
    const int at = pr % n_at, jt = pr / n_at;
    const int i = at * 32 + (lane & 31);
    const float* bp = As + i * cs + (lane >> 5);
    const float* ap = Bs + (jt * 32 + (lane & 31)) * cs + (lane >> 5);
    floatx16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    // operands read 8 k-steps ahead of their MFMAs (one LDS latency per group, not per step)
    int s2 = 0;
    for (; s2 + 8 <= c / 2; s2 += 8) {
      float av[8], bv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        av[u] = ap[2 * (s2 + u)];
        bv[u] = bp[2 * (s2 + u)];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
    }
    for (; s2 < c / 2; ++s2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[2 * s2], bp[2 * s2], acc, 0, 0, 0);
    float best = 0.f;
    int bidx = -1;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int jj = jt * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
      if (jj >= tb) continue;
      float v = acc[q];
      if ((cls && i == 0) || (dis && jj == 0)) v = -INFINITY;
      keep_best(v, jj, best, bidx);
    }
    const float ov = __shfl_xor(best, 32, 64);
    const int oi = __shfl_xor(bidx, 32, 64);
    keep_best(ov, oi, best, bidx);
    if (lane < 32) {
      pmax[jt * pa + i] = best;
      pidx[jt * pa + i] = bidx;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ta; i += FUSED_NT) {
    float bb = 0.f;
    int bi = -1;
    for (int jt = 0; jt < n_bt; ++jt) keep_best(pmax[jt * pa + i], pidx[jt * pa + i], bb, bi);
    nm[i] = bb;
    ni[i] = bi;
    keys[i] = sort_key(bb);
  }
  __syncthreads();
  // (3) descending total-order rank, ties -> higher index first (tome_rank_kernel); 8 lanes per
  // row each count over an eighth of the keys, summed with xor shuffles (uniform trip count)
  int* edge = pidx;  // the partials are consumed
  for (int i0 = 0; i0 < ta; i0 += FUSED_NT / 8) {
    const int i = i0 + (threadIdx.x >> 3), part = threadIdx.x & 7;
    const uint32_t kv = i < ta ? keys[i] : 0u;
    int rank = 0;
    if (i < ta)
      for (int j = part; j < ta; j += 8) {
        const uint32_t kw = keys[j];
        rank += (kw > kv) || (kw == kv && j > i);
      }
    rank += __shfl_xor(rank, 1, 64);
    rank += __shfl_xor(rank, 2, 64);
    rank += __shfl_xor(rank, 4, 64);
    if (i < ta && part == 0) edge[rank] = i;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < ta; k += FUSED_NT) {
    const int e = edge[k];
    if (k < r) {
      src_idx[(int64_t)b * r + k] = e;
      dst_idx[(int64_t)b * r + k] = ni[e];
    } else {
      unm_idx[(int64_t)b * (ta - r) + (k - r)] = e;
    }
    if (node_max_out) node_max_out[(int64_t)b * ta + k] = nm[k];
  }
}

// Scores for the sets too large for the fused kernel (t > 512 at c = 64: the OCTO-base 512-px
// image set, t = 1024 ... 672): the b half B^ of one sample resident in LDS (its [pbr][c + 1]
// image, 133 KB at t = 1024), AG 32-row a tiles per 1024-thread workgroup. tome_score_kernel
// re-staged the b rows 4 tiles at a time with one scalar load per element (a latency chain per
// group, 63 us for 16 samples at t = 1024) and ran one wave per b tile; here the staging is one
// burst of 16-B loads per thread and the 16 waves split AG x (16 / AG): wave (g, u) takes a tile g
// against b tiles u, u + 16 / AG, ... with the k-ordered f32 MFMA chain and first-index argmax of
// tome_score_kernel (the same per-(a row, b tile) chain and the same total-order combine, so
// node_max / node_idx are identical). Workgroups of one sample run on one XCD (xcd_remap over
// the flattened grid), which then reads that sample's B^ once from HBM.
constexpr int SBIG_NT = 1024;
constexpr int SB = 10;  // 16-B staging loads in flight per thread (the image at t = 1024: 9)
__host__ __device__ __forceinline__ size_t score_big_lds(int t, int c, int ag) {
  const int tb = t / 2, pbr = (tb + 31) / 32 * 32;
  return sizeof(float) * ((size_t)(pbr + 32 * ag) * (c + 1) + 2 * 16 * 32);
}
template <int AG>
__global__ __launch_bounds__(SBIG_NT) void tome_score_big_kernel(const float* __restrict__ An,
                                                                 const float* __restrict__ Bn,
                                                                 int t, int c, int flags, int wps,
                                                                 float* __restrict__ nmax,
                                                                 int32_t* __restrict__ nidx) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int WPG = 16 / AG;  // waves per a tile
  const int ta = (t + 1) / 2, tb = t / 2, cs = c + 1;
  const int pbr = (tb + 31) / 32 * 32, n_bt = pbr / 32;
  const int wi = xcd_remap(blockIdx.x, gridDim.x);
  const int b = wi / wps, a0 = (wi - b * wps) * AG * 32;  // first a row of this workgroup
  float* Bs = smem;                   // [pbr][cs]
  float* As = Bs + pbr * cs;          // [32 AG][cs]
  float* pmax = As + 32 * AG * cs;    // [16 waves][32]
  int* pidx = reinterpret_cast<int*>(pmax + 16 * 32);
  const float* Bb = Bn + (int64_t)b * tb * c;
  const float* Ab = An + (int64_t)b * ta * c;
  // stage: 16-B loads of the rows (rows past tb / ta: zeros), scalar LDS stores into the padded
  // image (c + 1 floats per row: conflict-free column reads)
  // (SB loads per thread issued before any store, from clamped addresses: one latency for the
  // whole image; a load-store loop waited for each load in turn)
  const int c4 = c / 4, tot = (pbr + 32 * AG) * c4;
  for (int e0 = 0; e0 < tot; e0 += SB * SBIG_NT) {
    float4 v[SB];
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const int e = min(e0 + k * SBIG_NT + (int)threadIdx.x, tot - 1);
      const int row = e / c4, q = e - row * c4;
      const bool isb = row < pbr;
      const int rr = isb ? min(row, tb - 1) : min(a0 + row - pbr, ta - 1);
      v[k] = *reinterpret_cast<const float4*>((isb ? Bb : Ab) + (int64_t)rr * c + 4 * q);
    }
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const int e = e0 + k * SBIG_NT + (int)threadIdx.x;
      if (e >= tot) break;
      const int row = e / c4, q = e - row * c4;
      const bool isb = row < pbr;
      const int rr = isb ? row : row - pbr;
      const bool live = isb ? rr < tb : a0 + rr < ta;
      float* d = (isb ? Bs : As) + rr * cs + 4 * q;
      d[0] = live ? v[k].x : 0.f;
      d[1] = live ? v[k].y : 0.f;
      d[2] = live ? v[k].z : 0.f;
      d[3] = live ? v[k].w : 0.f;
    }
  }
  __syncthreads();
  const bool cls = flags & MMT_TOME_CLASS_TOKEN;
  const bool dis = flags & MMT_TOME_DISTILL_TOKEN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = wave / WPG, u = wave - g * WPG;
  const int i = a0 + g * 32 + (lane & 31);
  const float* bp = As + (g * 32 + (lane & 31)) * cs + (lane >> 5);
  float best = 0.f;
  int bidx = -1;
  for (int jt = u; jt < n_bt; jt += WPG) {
    const float* ap = Bs + (jt * 32 + (lane & 31)) * cs + (lane >> 5);
    floatx16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    int s2 = 0;
    for (; s2 + 8 <= c / 2; s2 += 8) {
      float av[8], bv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        av[k] = ap[2 * (s2 + k)];
        bv[k] = bp[2 * (s2 + k)];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[k], bv[k], acc, 0, 0, 0);
    }
    for (; s2 < c / 2; ++s2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[2 * s2], bp[2 * s2], acc, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int jj = jt * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
      if (jj >= tb) continue;
      float v = acc[q];
      if ((cls && i == 0) || (dis && jj == 0)) v = -INFINITY;
      keep_best(v, jj, best, bidx);
    }
  }
  const float ov = __shfl_xor(best, 32, 64);
  const int oi = __shfl_xor(bidx, 32, 64);
  keep_best(ov, oi, best, bidx);
  if (lane < 32) {
    pmax[wave * 32 + lane] = best;
    pidx[wave * 32 + lane] = bidx;
  }
  __syncthreads();
  if (threadIdx.x < 32 * AG) {
    const int gg = threadIdx.x >> 5, l = threadIdx.x & 31;
    float bb = 0.f;
    int bi = -1;
    for (int w = 0; w < WPG; ++w) keep_best(pmax[(gg * WPG + w) * 32 + l], pidx[(gg * WPG + w) * 32 + l], bb, bi);
    const int ii = a0 + threadIdx.x;
    if (ii < ta) {
      nmax[(int64_t)b * ta + ii] = bb;
      nidx[(int64_t)b * ta + ii] = bi;
    }
  }
}

// Rank sort of the unfused path, several workgroups per sample: workgroup (sample, y) loads
// every key of the sample into LDS and ranks rows [128 y, 128 y + 128), 8 lanes per row (each
// counting over an eighth of the keys, 4 keys per LDS read, summed by xor shuffles), and writes
// each row's outputs at its rank directly (src / dst for ranks < r, unm otherwise: a rank is a
// row's final position, so no workgroup needs another's). tome_rank_kernel (one workgroup per
// sample, one thread per row walking all ta keys) is VALU-bound at O(ta^2) per CU: 17 us at
// ta = 512 for any number of samples.
constexpr int RANK8_NT = 1024, RANK8_ROWS = RANK8_NT / 8;
__global__ __launch_bounds__(RANK8_NT) void tome_rank8_kernel(const float* __restrict__ nmax,
                                                              const int32_t* __restrict__ nidx,
                                                              int ta, int r,
                                                              int32_t* __restrict__ unm_idx,
                                                              int32_t* __restrict__ src_idx,
                                                              int32_t* __restrict__ dst_idx,
                                                              float* __restrict__ node_max_out) {
  __shared__ __attribute__((aligned(16))) uint32_t keys[1024 + 32];
  const int n = blockIdx.y;
  const float* nm = nmax + (int64_t)n * ta;
  const int tap = (ta + 31) & ~31;  // padding keys 0: never counted (every live key is >= 1: a
                                    // NaN maps to 0xffffffff, a negative value's bits b to ~b,
                                    // which is 0 only for b = 0xffffffff, a NaN, the rest to b | 2^31)
  for (int i = threadIdx.x; i < tap; i += RANK8_NT) keys[i] = i < ta ? sort_key(nm[i]) : 0u;
  __syncthreads();
  const int i = blockIdx.x * RANK8_ROWS + (threadIdx.x >> 3), part = threadIdx.x & 7;
  const uint32_t kv = i < ta ? keys[i] : 0u;
  int rank = 0;
  if (i < ta)
#pragma unroll 4
    for (int j4 = 4 * part; j4 < tap; j4 += 32) {
      const uint4 kw = *reinterpret_cast<const uint4*>(keys + j4);
      rank += (kw.x > kv) || (kw.x == kv && j4 > i);
      rank += (kw.y > kv) || (kw.y == kv && j4 + 1 > i);
      rank += (kw.z > kv) || (kw.z == kv && j4 + 2 > i);
      rank += (kw.w > kv) || (kw.w == kv && j4 + 3 > i);
    }
  rank += __shfl_xor(rank, 1, 64);
  rank += __shfl_xor(rank, 2, 64);
  rank += __shfl_xor(rank, 4, 64);
  if (i < ta && part == 0) {
    if (rank < r) {
      src_idx[(int64_t)n * r + rank] = i;
      dst_idx[(int64_t)n * r + rank] = nidx[(int64_t)n * ta + i];
    } else {
      unm_idx[(int64_t)n * (ta - r) + (rank - r)] = i;
    }
    if (node_max_out) node_max_out[(int64_t)n * ta + i] = nm[i];
  }
}

__global__ __launch_bounds__(RANK_NT) void tome_rank_kernel(const float* __restrict__ nmax,
                                                            const int32_t* __restrict__ nidx,
                                                            int ta, int r,
                                                            int32_t* __restrict__ unm_idx,
                                                            int32_t* __restrict__ src_idx,
                                                            int32_t* __restrict__ dst_idx,
                                                            float* __restrict__ node_max_out) {
  __shared__ uint32_t keys[1024];
  __shared__ int32_t edge[1024];
  const int n = blockIdx.x;
  const float* nm = nmax + (int64_t)n * ta;
  for (int i = threadIdx.x; i < ta; i += RANK_NT) keys[i] = sort_key(nm[i]);
  __syncthreads();
  // descending total-order key, ties -> higher index first (stable ascending sort, reversed)
  for (int i = threadIdx.x; i < ta; i += RANK_NT) {
    const uint32_t kv = keys[i];
    int rank = 0;
    for (int j = 0; j < ta; ++j) {
      const uint32_t kw = keys[j];
      rank += (kw > kv) || (kw == kv && j > i);
    }
    edge[rank] = i;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < ta; k += RANK_NT) {
    const int e = edge[k];
    if (k < r) {
      src_idx[(int64_t)n * r + k] = e;
      dst_idx[(int64_t)n * r + k] = nidx[(int64_t)n * ta + e];
    } else {
      unm_idx[(int64_t)n * (ta - r) + (k - r)] = e;
    }
    if (node_max_out) node_max_out[(int64_t)n * ta + k] = nm[k];
  }
}

// ------------------------------------------------------------------ merge fwd / bwd
template <typename T>
struct Vec;
template <>
struct Vec<bf16_t> {
  static constexpr int N = 8;  // 16 B per lane
  typedef uint4 raw;
  __device__ static void load(const bf16_t* p, float* f) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f[2 * q] = __uint_as_float(w[q] << 16);
      f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  }
  __device__ static void store(bf16_t* p, const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      w[q] = (uint32_t)f2bf(f[2 * q]) | ((uint32_t)f2bf(f[2 * q + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <>
struct Vec<float> {
  static constexpr int N = 4;
  typedef float4 raw;
  __device__ static void load(const float* p, float* f) {
    const float4 u = *reinterpret_cast<const float4*>(p);
    f[0] = u.x;
    f[1] = u.y;
    f[2] = u.z;
    f[3] = u.w;
  }
  __device__ static void store(float* p, const float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  }
};

// Set-local output row q -> (primary set token, dst index j or -1 for an unmerged a token).
__device__ __forceinline__ void merged_row_source(int q, int ta, int r, bool dis,
                                                  const int32_t* unm, int* tok, int* j) {
  const int nu = ta - r;
  int ui = -1, dj = -1;
  if (!dis) {
    if (q < nu) ui = q;
    else dj = q - nu;
  } else {  // [unm[:1], dst[:1], unm[1:], dst[1:]]  (token_compression.py:103-105)
    if (q == 0) ui = 0;
    else if (q == 1) dj = 0;
    else if (q < 1 + nu) ui = q - 1;
    else dj = q - nu;
  }
  if (ui >= 0) {
    *tok = 2 * unm[ui];
    *j = -1;
  } else {
    *tok = 2 * dj + 1;
    *j = dj;
  }
}

// The merge maps of sample n into LDS, range-checked (common.h "device-side index checks"): unm /
// src in [0, ta), dst in [0, ta_b); an a token named twice by unm + src (not a partition of the a
// half: a broken matcher, e.g. a rank with ties) is recorded too — its pos_map would keep a
// hole that the backward would read. Ends with a barrier.
constexpr int kSeenWords = (1024 + 512 + 31) / 32;  // ta <= nu + r <= 1024 + 512
__device__ __forceinline__ void load_merge_maps(int n, int t, int r, const int32_t* __restrict__ unm_g,
                                                const int32_t* __restrict__ src_g,
                                                const int32_t* __restrict__ dst_g, int32_t* s_unm,
                                                int32_t* s_src, int32_t* s_dst, uint32_t* s_seen,
                                                unsigned int* fault) {
  const int ta = (t + 1) / 2, tb = t / 2, nu = ta - r;
  for (int k = threadIdx.x; k < kSeenWords; k += blockDim.x) s_seen[k] = 0;
  __syncthreads();
  auto mark = [&](int v) {
    const uint32_t bit = 1u << (v & 31);
    if (atomicOr(&s_seen[v >> 5], bit) & bit) record_fault(fault, MMT_FAULT_TOME_PARTITION);
  };
  for (int k = threadIdx.x; k < nu; k += blockDim.x) {
    const int v = checked_index(unm_g[(int64_t)n * nu + k], ta, fault, MMT_FAULT_TOME_INDEX);
    s_unm[k] = v;
    mark(v);
  }
  for (int k = threadIdx.x; k < r; k += blockDim.x) {
    const int v = checked_index(src_g[(int64_t)n * r + k], ta, fault, MMT_FAULT_TOME_INDEX);
    s_src[k] = v;
    mark(v);
    s_dst[k] = checked_index(dst_g[(int64_t)n * r + k], tb, fault, MMT_FAULT_TOME_INDEX);
  }
  __syncthreads();
}

// Forward merge, one block = kMergeRows output rows of one sample. Phase 1 resolves every output
// row (primary source row, size weight, divisor, and the list of src tokens scattered into it,
// in increasing i = the reference's sequential scatter order) into LDS; phase 2 streams the
// (row, 16-B chunk) items of the block with all primary loads of a 4-item group issued before
// any use, so many loads are in flight per thread (HBM-bound gather).
constexpr int kMergeRows = 8;
constexpr int kMergeSeg = 8;  // src tokens listed per row in LDS (more: scan the dst list)

template <typename T>
__global__ __launch_bounds__(256) void tome_merge_fwd_kernel(
    const T* __restrict__ x, int L, int D, int64_t xs_n, int64_t xs_t, int set_start, int t, int r,
    int flags, const float* __restrict__ size_in, const int32_t* __restrict__ unm_g,
    const int32_t* __restrict__ src_g, const int32_t* __restrict__ dst_g, T* __restrict__ out,
    int64_t os_n, int64_t os_t, float* __restrict__ size_out, int32_t* __restrict__ pos_map,
    unsigned int* fault) {
  __shared__ int32_t s_unm[1024];
  __shared__ int32_t s_src[512];
  __shared__ int32_t s_dst[512];
  __shared__ uint32_t s_seen[kSeenWords];
  __shared__ int32_t m_prim[kMergeRows], m_cnt[kMergeRows], m_j[kMergeRows];
  __shared__ float m_sp[kMergeRows], m_S[kMergeRows];
  __shared__ int32_t m_list[kMergeRows][kMergeSeg];
  __shared__ float m_ss[kMergeRows][kMergeSeg];
  const int n = blockIdx.x;
  const int ta = (t + 1) / 2;
  const bool dis = flags & MMT_TOME_DISTILL_TOKEN;
  const bool plain = flags & MMT_TOME_PLAIN_SUM;      // merge(x, "sum") without the size weights
  const bool scatter = !(flags & MMT_TOME_NO_SCATTER);  // merge(x, mode != "sum"): dst unchanged
  load_merge_maps(n, t, r, unm_g, src_g, dst_g, s_unm, s_src, s_dst, s_seen, fault);
  const float* sb = size_in ? size_in + (int64_t)n * t : nullptr;
  const int Lout = L - r;
  const int row0 = blockIdx.y * kMergeRows;
  const int nrows = min(kMergeRows, Lout - row0);
  if (threadIdx.x < nrows) {  // phase 1: one thread per output row
    const int ri = threadIdx.x, o = row0 + ri;
    if (o < set_start || o >= set_start + t - r) {  // plain copy of a non-merged token
      m_prim[ri] = o < set_start ? o : o + r;
      m_j[ri] = -2;
      m_cnt[ri] = 0;
    } else {
      const int q = o - set_start;
      int tok, j;
      merged_row_source(q, ta, r, dis, s_unm, &tok, &j);
      m_prim[ri] = set_start + tok;
      m_sp[ri] = (sb && !plain) ? sb[tok] : 1.f;
      // sizes: S = s_primary + sum_i s_src_i in increasing i (sequential scatter-add, :100-101)
      float S = sb ? sb[tok] : 1.f;
      int cnt = 0;
      if (j >= 0 && scatter) {
        for (int i = 0; i < r; ++i) {
          if (s_dst[i] != j) continue;
          const int st = 2 * s_src[i];
          S = S + (sb ? sb[st] : 1.f);
          if (cnt < kMergeSeg) {
            m_list[ri][cnt] = set_start + st;
            m_ss[ri][cnt] = (sb && !plain) ? sb[st] : 1.f;
          }
          ++cnt;
        }
      }
      m_j[ri] = (j >= 0 && scatter) ? j : -1;
      m_cnt[ri] = cnt;
      m_S[ri] = S;
      if (size_out) size_out[(int64_t)n * (t - r) + q] = S;
      if (pos_map) {
        int32_t* pm = pos_map + (int64_t)n * t;
        pm[tok] = q;
        if (j >= 0 && scatter)
          for (int i = 0; i < r; ++i)
            if (s_dst[i] == j) pm[2 * s_src[i]] = q;
      }
    }
  }
  __syncthreads();
  constexpr int V = Vec<T>::N;
  const int nchunk = D / V;
  const T* xb = x + (int64_t)n * xs_n;
  T* ob = out + (int64_t)n * os_n;
  const int total = nrows * nchunk;
  constexpr int G = 4;  // items per thread whose loads are issued together
  for (int base = 0; base < total; base += G * 256) {
    float v[G][V];
    int ri[G], ch[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {  // clamped (always valid) addresses: loads issue unconditionally
      const int idx = min(base + u * 256 + (int)threadIdx.x, total - 1);
      ri[u] = idx / nchunk;
      ch[u] = idx - ri[u] * nchunk;
      Vec<T>::load(xb + (int64_t)m_prim[ri[u]] * xs_t + ch[u] * V, v[u]);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (base + u * 256 + (int)threadIdx.x >= total) break;
      const int rr = ri[u];
      const int64_t ooff = (int64_t)(row0 + rr) * os_t + ch[u] * V;
      const int jr = m_j[rr];
      if (jr == -2) {  // copy row
        Vec<T>::store(ob + ooff, v[u]);
        continue;
      }
      float acc[V];
      const float sp = m_sp[rr];
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = v[u][e] * sp;
      const int cnt = m_cnt[rr];
      if (cnt <= kMergeSeg) {
        for (int k = 0; k < cnt; ++k) {
          float w[V];
          Vec<T>::load(xb + (int64_t)m_list[rr][k] * xs_t + ch[u] * V, w);
          const float ss = m_ss[rr][k];
#pragma unroll
          for (int e = 0; e < V; ++e) acc[e] = acc[e] + w[e] * ss;
        }
      } else {
        for (int i = 0; i < r; ++i) {
          if (s_dst[i] != jr) continue;
          const int st = 2 * s_src[i];
          const float ss = (sb && !plain) ? sb[st] : 1.f;
          float w[V];
          Vec<T>::load(xb + (int64_t)(set_start + st) * xs_t + ch[u] * V, w);
#pragma unroll
          for (int e = 0; e < V; ++e) acc[e] = acc[e] + w[e] * ss;
        }
      }
      if (!plain) {
        const float S = m_S[rr];
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = __fdiv_rn(acc[e], S);
      }
      Vec<T>::store(ob + ooff, acc);
    }
  }
}

// Backward merge: g_in[row] = g_out[pos(row)] * s_tok / S_pos for set tokens (a weighted
// gather), a copy elsewhere. One block = kMergeRows input rows; (row, chunk) items streamed
// with 4 loads in flight per thread.
template <typename T>
__global__ __launch_bounds__(256) void tome_merge_bwd_kernel(
    const T* __restrict__ g_out, int L, int D, int64_t go_s_n, int64_t go_s_t, int set_start,
    int t, int r, const float* __restrict__ size_in, const float* __restrict__ size_out,
    const int32_t* __restrict__ pos_map, T* __restrict__ g_in, int64_t gi_s_n, int64_t gi_s_t,
    unsigned int* fault) {
  __shared__ int32_t m_orow[kMergeRows];
  __shared__ float m_s[kMergeRows], m_S[kMergeRows];
  __shared__ int32_t m_copy[kMergeRows];
  const int n = blockIdx.x;
  const int row0 = blockIdx.y * kMergeRows;
  const int nrows = min(kMergeRows, L - row0);
  if (threadIdx.x < nrows) {
    const int ri = threadIdx.x, row = row0 + ri;
    if (row < set_start || row >= set_start + t) {
      m_orow[ri] = row < set_start ? row : row - r;
      m_copy[ri] = 1;
    } else {
      const int tok = row - set_start;
      const int q = checked_index(pos_map[(int64_t)n * t + tok], t - r, fault, MMT_FAULT_POS_MAP);
      m_orow[ri] = set_start + q;
      m_s[ri] = size_in ? size_in[(int64_t)n * t + tok] : 1.f;
      m_S[ri] = size_out ? size_out[(int64_t)n * (t - r) + q] : 1.f;  // NULL: plain sum
      m_copy[ri] = 0;
    }
  }
  __syncthreads();
  constexpr int V = Vec<T>::N;
  const int nchunk = D / V;
  const T* gb = g_out + (int64_t)n * go_s_n;
  T* ib = g_in + (int64_t)n * gi_s_n;
  const int total = nrows * nchunk;
  constexpr int G = 4;
  for (int base = 0; base < total; base += G * 256) {
    float v[G][V];
    int ri[G], ch[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int idx = min(base + u * 256 + (int)threadIdx.x, total - 1);
      ri[u] = idx / nchunk;
      ch[u] = idx - ri[u] * nchunk;
      Vec<T>::load(gb + (int64_t)m_orow[ri[u]] * go_s_t + ch[u] * V, v[u]);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (base + u * 256 + (int)threadIdx.x >= total) break;
      const int rr = ri[u];
      if (!m_copy[rr]) {
        const float s = m_s[rr], S = m_S[rr];
#pragma unroll
        for (int e = 0; e < V; ++e) v[u][e] = (v[u][e] * s) / S;
      }
      Vec<T>::store(ib + (int64_t)(row0 + rr) * gi_s_t + ch[u] * V, v[u]);
    }
  }
}

bool g_match_use_mfma = true;

int pow2_at_least(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

}  // namespace

namespace mmt {
int64_t tome_match_workspace(int64_t n, int64_t t, int64_t c) {
  const int64_t ta = (t + 1) / 2;
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  return al(n * ta * c * 4) + al(n * (t / 2) * c * 4) + al(n * ta * 4) + al(n * ta * 4);
}
}  // namespace mmt

extern "C" void mmt_tome_set_match_path(int use_mfma) { g_match_use_mfma = use_mfma != 0; }

extern "C" int mmt_tome_match(const void* metric, int dtype, int n, int t, int heads, int c,
                              int64_t s_n, int64_t s_t, int64_t s_h, int r, int flags,
                              int32_t* unm_idx, int32_t* src_idx, int32_t* dst_idx,
                              float* node_max, void* workspace, int64_t ws_bytes,
                              mmt_stream_t stream) {
  MMT_CHECK_ARG(metric && (unm_idx || (t + 1) / 2 == r) && src_idx && dst_idx && workspace,
                "mmt_tome_match: null pointer");  // unm may be NULL when every A token merges
  MMT_CHECK_ARG(n > 0 && t >= 2 && heads >= 1 && c >= 1, "mmt_tome_match: bad shape n=%d t=%d", n, t);
  MMT_CHECK_ARG(t <= 2048 && c <= 512, "mmt_tome_match: t=%d c=%d beyond 2048 / 512", t, c);
  const int prot = ((flags & MMT_TOME_CLASS_TOKEN) ? 1 : 0) + ((flags & MMT_TOME_DISTILL_TOKEN) ? 1 : 0);
  MMT_CHECK_ARG(r > 0 && r <= (t - prot) / 2,
                "mmt_tome_match: r=%d must be clamped to 1..(t-protected)//2=%d", r, (t - prot) / 2);
  MMT_CHECK_ARG(dtype == MMT_F32 || dtype == MMT_BF16, "mmt_tome_match: dtype %d", dtype);
  const int64_t need = tome_match_workspace(n, t, c);
  MMT_CHECK_ARG(ws_bytes >= need && (uintptr_t)workspace % 16 == 0,
                "mmt_tome_match: workspace %lld B < %lld B (mmt_workspace_size) or not 16-B aligned",
                (long long)ws_bytes, (long long)need);
  const int ta = (t + 1) / 2, tb = t / 2;
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  char* w = (char*)workspace;
  float* An = (float*)w;
  float* Bn = (float*)(w + al((int64_t)n * ta * c * 4));
  float* nmax = (float*)((char*)Bn + al((int64_t)n * tb * c * 4));
  int32_t* nidx = (int32_t*)((char*)nmax + al((int64_t)n * ta * 4));
  hipStream_t s = as_stream(stream);
  const int vw = dtype == MMT_BF16 ? 8 : 4;  // elements per 16 B
  const bool vec = (c % 8 == 0) && (s_n % vw == 0) && (s_t % vw == 0) && (s_h % vw == 0) &&
                   ((uintptr_t)metric % 16 == 0);
  const size_t fused_lds = fused_match_lds(t, c);
  if (vec && g_match_use_mfma && fused_lds <= 160 * 1024 && c / 8 <= 64) {
    // one launch: norm + score + rank with both halves in LDS
    const int lpr = pow2_at_least(c / 8);
#define FUSED(T, LPR)                                                                            \
  do {                                                                                           \
    static const bool attr_ = (hipFuncSetAttribute((const void*)tome_match_fused_kernel<T, LPR>, \
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024), true);    \
    (void)attr_;                                                                                 \
    hipLaunchKernelGGL((tome_match_fused_kernel<T, LPR>), dim3(n), dim3(FUSED_NT), fused_lds, s, \
                       (const T*)metric, t, heads, c, s_n, s_t, s_h, r, flags, unm_idx, src_idx, \
                       dst_idx, node_max);                                                       \
  } while (0)
#define FUSED_ALL(T)                                  \
  switch (lpr) {                                      \
    case 1: FUSED(T, 1); break;                       \
    case 2: FUSED(T, 2); break;                       \
    case 4: FUSED(T, 4); break;                       \
    case 8: FUSED(T, 8); break;                       \
    case 16: FUSED(T, 16); break;                     \
    case 32: FUSED(T, 32); break;                     \
    default: FUSED(T, 64); break;                     \
  }
    if (dtype == MMT_F32) { FUSED_ALL(float) } else { FUSED_ALL(bf16_t) }
#undef FUSED_ALL
#undef FUSED
    MMT_CHECK_LAUNCH("mmt_tome_match(fused)");
    return MMT_OK;
  }
  // 1. per-token head sum + L2 normalisation
  const int64_t rows = (int64_t)n * t;
  if (vec) {
    const int lpr = pow2_at_least(c / 8);
#define NORMV(T, LPR)                                                                          \
  hipLaunchKernelGGL((tome_norm_vec_kernel<T, LPR>), dim3((rows * LPR + NORM_NT - 1) / NORM_NT), \
                     dim3(NORM_NT), 0, s, (const T*)metric, n, t, heads, c, s_n, s_t, s_h, An, Bn)
#define NORMV_ALL(T)                                  \
  switch (lpr) {                                      \
    case 1: NORMV(T, 1); break;                       \
    case 2: NORMV(T, 2); break;                       \
    case 4: NORMV(T, 4); break;                       \
    case 8: NORMV(T, 8); break;                       \
    case 16: NORMV(T, 16); break;                     \
    case 32: NORMV(T, 32); break;                     \
    default: NORMV(T, 64); break;                     \
  }
    if (dtype == MMT_F32) { NORMV_ALL(float) } else { NORMV_ALL(bf16_t) }
#undef NORMV_ALL
#undef NORMV
  } else {
    const dim3 grid((rows + NORM_NT - 1) / NORM_NT);
    if (dtype == MMT_F32)
      hipLaunchKernelGGL(tome_norm_scalar_kernel<float>, grid, dim3(NORM_NT), 0, s,
                         (const float*)metric, n, t, heads, c, s_n, s_t, s_h, An, Bn);
    else
      hipLaunchKernelGGL(tome_norm_scalar_kernel<bf16_t>, grid, dim3(NORM_NT), 0, s,
                         (const bf16_t*)metric, n, t, heads, c, s_n, s_t, s_h, An, Bn);
  }
  MMT_CHECK_LAUNCH("mmt_tome_match(norm)");
  // 2. scores + per-a-row argmax: with the whole b half resident in LDS when it fits (t <= 1024
  //    at c = 64), otherwise as many 32-row b tiles per LDS group as fit (<= 4); 3. rank
  const int n_at = (ta + 31) / 32;
  if (g_match_use_mfma && c % 4 == 0 && score_big_lds(t, c, 1) <= 160 * 1024) {
    const bool two = (int64_t)n * n_at > 256 && score_big_lds(t, c, 2) <= 160 * 1024;
    const int wps = two ? (n_at + 1) / 2 : n_at;
#define SBIG(AG)                                                                                  \
  do {                                                                                            \
    static const bool attr_ = (hipFuncSetAttribute((const void*)tome_score_big_kernel<AG>,       \
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024), true);     \
    (void)attr_;                                                                                  \
    hipLaunchKernelGGL(tome_score_big_kernel<AG>, dim3(n * wps), dim3(SBIG_NT),                   \
                       score_big_lds(t, c, AG), s, An, Bn, t, c, flags, wps, nmax, nidx);        \
  } while (0)
    if (two) SBIG(2); else SBIG(1);
#undef SBIG
    MMT_CHECK_LAUNCH("mmt_tome_match(score big)");
    hipLaunchKernelGGL(tome_rank8_kernel, dim3((ta + RANK8_ROWS - 1) / RANK8_ROWS, n), dim3(RANK8_NT), 0, s,
                       nmax, nidx, ta, r, unm_idx, src_idx, dst_idx, node_max);
    MMT_CHECK_LAUNCH("mmt_tome_match(rank)");
    return MMT_OK;
  }
  const int cs = c + 1;
  const size_t tile = sizeof(float) * 32 * cs;
  const size_t fixed = tile + sizeof(float) * 8 * 32 * 2;
  int nbt = (int)((160 * 1024 - fixed) / tile);
  nbt = nbt > 4 ? 4 : nbt;
  MMT_CHECK_ARG(nbt >= 1, "mmt_tome_match: c=%d too large for the LDS tiles", c);
  const size_t smem = fixed + nbt * tile;
  const bool mfma = g_match_use_mfma && (c % 2 == 0);
  const dim3 sgrid((ta + 31) / 32, n);
#define SCORE(M)                                                                              \
  do {                                                                                        \
    static const bool attr_ = (hipFuncSetAttribute((const void*)tome_score_kernel<M>,        \
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024), true); \
    (void)attr_;                                                                              \
    hipLaunchKernelGGL(tome_score_kernel<M>, sgrid, dim3(SCORE_NT), smem, s, An, Bn, t, c,    \
                       flags, nbt, nmax, nidx);                                               \
  } while (0)
  if (mfma) SCORE(true); else SCORE(false);
#undef SCORE
  MMT_CHECK_LAUNCH("mmt_tome_match(score)");
  // 3. rank sort -> src / dst / unm
  hipLaunchKernelGGL(tome_rank_kernel, dim3(n), dim3(RANK_NT), 0, s, nmax, nidx, ta, r, unm_idx,
                     src_idx, dst_idx, node_max);
  MMT_CHECK_LAUNCH("mmt_tome_match(rank)");
  return MMT_OK;
}

static int check_vec(int dtype, int D, int64_t a, int64_t b, int64_t c2, int64_t d) {
  const int V = dtype == MMT_BF16 ? 8 : 4;
  return D % V == 0 && a % V == 0 && b % V == 0 && c2 % V == 0 && d % V == 0;
}

// ToMe merge fused with the following sequence-axis LayerNorm forward (attention.py:66 after
// tome_attention.py:249-256): one workgroup = one sample x 64 columns. The output rows' sources
// are resolved once per workgroup (as phase 1 of tome_merge_fwd_kernel, for all Lout rows);
// pass 1 merges its columns with the merge kernel's exact arithmetic (this file is compiled
// without FMA contraction: bit-identical merged rows), stores them and accumulates the LN sums;
// pass 2 re-reads the just-written rows and writes y (bf16). Saves the LN's separate read of the
// merged sequence and a launch. fp32 residual stream, Lout <= kFusedRows.
// RPT > 0 (Lout <= 32 RPT): every thread first issues the primary-row loads of all its RPT output
// rows (row-clamped, unconditional: a load under a per-row branch waits vmcnt(0) each), keeps the
// merged rows in registers and writes y from them (no re-read of the merged rows).
constexpr int kFusedRows = 512, kFRG = 32;
template <int RPT = 0>
__global__ __launch_bounds__(256) void tome_merge_seqnorm_fwd_kernel(
    const float* __restrict__ x, int L, int D, int64_t xs_n, int64_t xs_t, int set_start, int t,
    int r, int flags, const float* __restrict__ size_in, const int32_t* __restrict__ unm_g,
    const int32_t* __restrict__ src_g, const int32_t* __restrict__ dst_g, float* __restrict__ out,
    int64_t os_n, int64_t os_t, float* __restrict__ size_out, int32_t* __restrict__ pos_map,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    bf16_t* __restrict__ y, int64_t ys_n, int64_t ys_t, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, unsigned int* fault) {
  // LDS sized for the rows this instantiation handles (RPT > 0: Lout <= 32 RPT; nu, r <= Lout),
  // and the pass-1 reduction scratch aliases the source lists (dead by then, behind a barrier):
  // 35-52 KB per workgroup instead of 68 KB, three or four workgroups per CU instead of two
  constexpr int MR = RPT > 0 ? 32 * RPT : kFusedRows;
  __shared__ int32_t s_unm[RPT > 0 ? MR : 1024];
  __shared__ int32_t s_src[RPT > 0 ? MR : 512];
  __shared__ int32_t s_dst[RPT > 0 ? MR : 512];
  __shared__ uint32_t s_seen[kSeenWords];
  __shared__ int32_t m_prim[MR], m_cnt[MR], m_j[MR];
  __shared__ float m_sp[MR], m_S[MR];
  constexpr int LIST_B = MR * kMergeSeg * 8, RED_B = 2 * kFRG * 64 * 4;
  __shared__ __attribute__((aligned(16))) char m_lists[LIST_B > RED_B ? LIST_B : RED_B];
  int32_t (*m_list)[kMergeSeg] = reinterpret_cast<int32_t (*)[kMergeSeg]>(m_lists);
  float (*m_ss)[kMergeSeg] = reinterpret_cast<float (*)[kMergeSeg]>(m_lists + MR * kMergeSeg * 4);
  float* red = reinterpret_cast<float*>(m_lists);
  __shared__ float s_mul[64], s_add[64];
  const int n = ln_sample(), c0 = ln_colblk() * 64;
  const int ta = (t + 1) / 2;
  const bool dis = flags & MMT_TOME_DISTILL_TOKEN;
  const bool plain = flags & MMT_TOME_PLAIN_SUM;
  const bool scatter = !(flags & MMT_TOME_NO_SCATTER);
  const bool lead = ln_colblk() == 0;  // writes the sizes and the position map
  load_merge_maps(n, t, r, unm_g, src_g, dst_g, s_unm, s_src, s_dst, s_seen, lead ? fault : nullptr);
  const float* sb = size_in ? size_in + (int64_t)n * t : nullptr;
  const int Lout = L - r;
  for (int o = threadIdx.x; o < Lout; o += blockDim.x) {  // phase 1 (tome_merge_fwd_kernel)
    if (o < set_start || o >= set_start + t - r) {
      m_prim[o] = o < set_start ? o : o + r;
      m_j[o] = -2;
      m_cnt[o] = 0;
    } else {
      const int q = o - set_start;
      int tok, j;
      merged_row_source(q, ta, r, dis, s_unm, &tok, &j);
      m_prim[o] = set_start + tok;
      m_sp[o] = (sb && !plain) ? sb[tok] : 1.f;
      float S = sb ? sb[tok] : 1.f;
      int cnt = 0;
      if (j >= 0 && scatter) {
        for (int i = 0; i < r; ++i) {
          if (s_dst[i] != j) continue;
          const int st = 2 * s_src[i];
          S = S + (sb ? sb[st] : 1.f);
          if (cnt < kMergeSeg) {
            m_list[o][cnt] = set_start + st;
            m_ss[o][cnt] = (sb && !plain) ? sb[st] : 1.f;
          }
          ++cnt;
        }
      }
      m_j[o] = (j >= 0 && scatter) ? j : -1;
      m_cnt[o] = cnt;
      m_S[o] = S;
      if (lead && size_out) size_out[(int64_t)n * (t - r) + q] = S;
      if (lead && pos_map) {
        int32_t* pm = pos_map + (int64_t)n * t;
        pm[tok] = q;
        if (j >= 0 && scatter)
          for (int i = 0; i < r; ++i)
            if (s_dst[i] == j) pm[2 * s_src[i]] = q;
      }
    }
  }
  __syncthreads();
  // pass 1: 8 column vectors x 32 row groups, 8 columns per thread (as seqnorm_fwd_kernel)
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = c0 + cv * 8;
  const bool cok = col < D;
  const float* xb = x + (int64_t)n * xs_n + col;
  float* ob = out + (int64_t)n * os_n + col;
  float part[2][8] = {};
  // the merge of output row o into v (tome_merge_fwd_kernel's arithmetic), v holding its
  // primary row on entry; then its store and LN sums
  auto merge_row = [&](int o, float* v) {
    const int jr = m_j[o];
    if (jr != -2) {
      const float sp = m_sp[o];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] * sp;
      const int cnt = m_cnt[o];
      if (cnt <= kMergeSeg) {
        for (int k = 0; k < cnt; ++k) {
          float w[8];
          Vec<float>::load(xb + (int64_t)m_list[o][k] * xs_t, w);
          Vec<float>::load(xb + (int64_t)m_list[o][k] * xs_t + 4, w + 4);
          const float ss = m_ss[o][k];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] + w[e] * ss;
        }
      } else {
        for (int i = 0; i < r; ++i) {
          if (s_dst[i] != jr) continue;
          const int st = 2 * s_src[i];
          const float ss = (sb && !plain) ? sb[st] : 1.f;
          float w[8];
          Vec<float>::load(xb + (int64_t)(set_start + st) * xs_t, w);
          Vec<float>::load(xb + (int64_t)(set_start + st) * xs_t + 4, w + 4);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] + w[e] * ss;
        }
      }
      if (!plain) {
        const float S = m_S[o];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = __fdiv_rn(v[e], S);
      }
    }
    Vec<float>::store(ob + (int64_t)o * os_t, v);
    Vec<float>::store(ob + (int64_t)o * os_t + 4, v + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      part[0][e] += v[e];
      part[1][e] = __builtin_fmaf(v[e], v[e], part[1][e]);
    }
  };
  constexpr int RR = RPT > 0 ? RPT : 1;
  [[maybe_unused]] float rv[RR][8];
  if constexpr (RPT > 0) {
    if (cok) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int o = min(rg + j * kFRG, Lout - 1);
        Vec<float>::load(xb + (int64_t)m_prim[o] * xs_t, rv[j]);
        Vec<float>::load(xb + (int64_t)m_prim[o] * xs_t + 4, rv[j] + 4);
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j)
        if (rg + j * kFRG < Lout) merge_row(rg + j * kFRG, rv[j]);
    }
  } else if (cok) {
    for (int o = rg; o < Lout; o += kFRG) {
      float v[8];
      Vec<float>::load(xb + (int64_t)m_prim[o] * xs_t, v);
      Vec<float>::load(xb + (int64_t)m_prim[o] * xs_t + 4, v + 4);
      merge_row(o, v);
    }
  }
  __syncthreads();  // every merge_row has read the source lists that red overwrites
#pragma unroll
  for (int vv = 0; vv < 2; ++vv)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(vv * kFRG + rg) * 64 + cv * 8 + e] = part[vv][e];
  __syncthreads();
  if (threadIdx.x < 64 && c0 + threadIdx.x < D) {
    float s1 = 0.f, s2 = 0.f;
    for (int g = 0; g < kFRG; ++g) {
      s1 += red[g * 64 + threadIdx.x];
      s2 += red[(kFRG + g) * 64 + threadIdx.x];
    }
    const int c = c0 + threadIdx.x;
    // the arithmetic of seqnorm_fwd_kernel as compiled there (norm.hip contracts to these fmas):
    // bit-identical statistics and outputs to merge followed by mmt_seqnorm_fwd
    const float mu = s1 / Lout;
    const float var = fmaxf(0.f, __builtin_fmaf(-mu, mu, s2 / Lout));
    const float rs = rsqrtf(var + eps);
    const float mul = rs * gamma[c];
    s_mul[threadIdx.x] = mul;
    s_add[threadIdx.x] = __builtin_fmaf(-mu, mul, beta[c]);
    mean_out[(int64_t)n * D + c] = mu;
    rstd_out[(int64_t)n * D + c] = rs;
  }
  __syncthreads();
  if (!cok) return;
  float mul[8], add[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mul[e] = s_mul[cv * 8 + e];
    add[e] = s_add[cv * 8 + e];
  }
  bf16_t* yb = y + (int64_t)n * ys_n + col;
#pragma unroll(RPT > 0 ? RPT : 1)
  for (int j = 0, o = rg; o < Lout && (RPT == 0 || j < RPT); ++j, o += kFRG) {
    float f[8];
    if constexpr (RPT > 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = rv[j][e];
    } else {
      Vec<float>::load(ob + (int64_t)o * os_t, f);
      Vec<float>::load(ob + (int64_t)o * os_t + 4, f + 4);
    }
    uint32_t wds[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float a = __builtin_fmaf(f[2 * q], mul[2 * q], add[2 * q]);
      const float b = __builtin_fmaf(f[2 * q + 1], mul[2 * q + 1], add[2 * q + 1]);
      wds[q] = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
    }
    *reinterpret_cast<uint4*>(yb + (int64_t)o * ys_t) = make_uint4(wds[0], wds[1], wds[2], wds[3]);
  }
}

extern "C" int mmt_tome_merge_seqnorm_fwd(const float* x, int n, int L, int D, int64_t x_s_n,
                                          int64_t x_s_t, int set_start, int t, int r, int flags,
                                          const float* size_in, const int32_t* unm_idx,
                                          const int32_t* src_idx, const int32_t* dst_idx,
                                          float* x_out, int64_t o_s_n, int64_t o_s_t,
                                          float* size_out, int32_t* pos_map, const float* gamma,
                                          const float* beta, float eps, void* y, int64_t y_s_n,
                                          int64_t y_s_t, float* mean, float* rstd,
                                          mmt_stream_t stream) {
  MMT_CHECK_ARG(x && x_out && (unm_idx || (t + 1) / 2 == r) && src_idx && dst_idx && gamma && beta &&
                    y && mean && rstd,
                "mmt_tome_merge_seqnorm_fwd: null pointer");
  MMT_CHECK_ARG(n > 0 && L > 0 && D > 0 && D % 8 == 0 && t >= 2 && set_start >= 0 &&
                    set_start + t <= L && L - r <= kFusedRows,
                "mmt_tome_merge_seqnorm_fwd: bad shape (L - r <= %d)", kFusedRows);
  MMT_CHECK_ARG(r > 0 && r <= t / 2 && (t + 1) / 2 - r <= 1024 && r <= 512,
                "mmt_tome_merge_seqnorm_fwd: bad r=%d for t=%d", r, t);
  MMT_CHECK_ARG(x_s_t % 8 == 0 && x_s_n % 8 == 0 && o_s_t % 8 == 0 && o_s_n % 8 == 0 &&
                    y_s_t % 8 == 0 && y_s_n % 8 == 0,
                "mmt_tome_merge_seqnorm_fwd: strides must be multiples of 8");
  const dim3 grid = ln_grid(n, (D + 63) / 64);
  const int Lo = L - r;
  static const bool rpt_on = !getenv("MMT_SNB_RPT") || atoi(getenv("MMT_SNB_RPT")) != 0;
  const int rpt = !rpt_on ? 0 : Lo <= 128 ? 4 : Lo <= 192 ? 6 : Lo <= 256 ? 8 : Lo <= 320 ? 10 : 0;
#define TMS(R) hipLaunchKernelGGL((tome_merge_seqnorm_fwd_kernel<R>), grid, dim3(256), 0, as_stream(stream), ARGS_)
  unsigned int* const fault = fault_word();
#define ARGS_ x, L, D, x_s_n, x_s_t, set_start, t, r, flags, size_in, unm_idx, src_idx, dst_idx, x_out, o_s_n, o_s_t, size_out, pos_map, gamma, beta, eps, (bf16_t*)y, y_s_n, y_s_t, mean, rstd, fault
  if (rpt == 4) TMS(4);
  else if (rpt == 6) TMS(6);
  else if (rpt == 8) TMS(8);
  else if (rpt == 10) TMS(10);
  else TMS(0);
#undef ARGS_
#undef TMS
  MMT_CHECK_LAUNCH("mmt_tome_merge_seqnorm_fwd");
  return MMT_OK;
}

extern "C" int mmt_tome_merge_wavg_fwd(const void* x, int dtype, int n, int L, int D, int64_t x_s_n,
                                       int64_t x_s_t, int set_start, int t, int r, int flags,
                                       const float* size_in, const int32_t* unm_idx,
                                       const int32_t* src_idx, const int32_t* dst_idx, void* x_out,
                                       int64_t o_s_n, int64_t o_s_t, float* size_out,
                                       int32_t* pos_map, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && x_out && (unm_idx || (t + 1) / 2 == r) && src_idx && dst_idx,
                "mmt_tome_merge_wavg_fwd: null pointer");
  MMT_CHECK_ARG(n > 0 && L > 0 && D > 0 && t >= 2 && set_start >= 0 && set_start + t <= L,
                "mmt_tome_merge_wavg_fwd: bad shape");
  MMT_CHECK_ARG(r > 0 && r <= t / 2 && (t + 1) / 2 - r <= 1024 && r <= 512,
                "mmt_tome_merge_wavg_fwd: bad r=%d for t=%d", r, t);
  MMT_CHECK_ARG(dtype == MMT_F32 || dtype == MMT_BF16, "mmt_tome_merge_wavg_fwd: dtype");
  MMT_CHECK_ARG(check_vec(dtype, D, x_s_n, x_s_t, o_s_n, o_s_t),
                "mmt_tome_merge_wavg_fwd: D and strides must be multiples of 16 bytes");
  dim3 grid(n, (L - r + kMergeRows - 1) / kMergeRows);
  hipStream_t s = as_stream(stream);
  unsigned int* const fault = fault_word();
  if (dtype == MMT_F32)
    hipLaunchKernelGGL(tome_merge_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)x, L, D,
                       x_s_n, x_s_t, set_start, t, r, flags, size_in, unm_idx, src_idx, dst_idx,
                       (float*)x_out, o_s_n, o_s_t, size_out, pos_map, fault);
  else
    hipLaunchKernelGGL(tome_merge_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, L,
                       D, x_s_n, x_s_t, set_start, t, r, flags, size_in, unm_idx, src_idx,
                       dst_idx, (bf16_t*)x_out, o_s_n, o_s_t, size_out, pos_map, fault);
  MMT_CHECK_LAUNCH("mmt_tome_merge_wavg_fwd");
  return MMT_OK;
}

extern "C" int mmt_tome_merge_wavg_bwd(const void* g_out, int dtype, int n, int L, int D,
                                       int64_t go_s_n, int64_t go_s_t, int set_start, int t, int r,
                                       const float* size_in, const float* size_out,
                                       const int32_t* pos_map, void* g_in, int64_t gi_s_n,
                                       int64_t gi_s_t, mmt_stream_t stream) {
  MMT_CHECK_ARG(g_out && g_in && pos_map, "mmt_tome_merge_wavg_bwd: null pointer");
  MMT_CHECK_ARG(n > 0 && L > 0 && D > 0 && t >= 2 && set_start >= 0 && set_start + t <= L &&
                    r > 0 && r <= t / 2,
                "mmt_tome_merge_wavg_bwd: bad shape");
  MMT_CHECK_ARG(dtype == MMT_F32 || dtype == MMT_BF16, "mmt_tome_merge_wavg_bwd: dtype");
  MMT_CHECK_ARG(check_vec(dtype, D, go_s_n, go_s_t, gi_s_n, gi_s_t),
                "mmt_tome_merge_wavg_bwd: D and strides must be multiples of 16 bytes");
  dim3 grid(n, (L + kMergeRows - 1) / kMergeRows);
  hipStream_t s = as_stream(stream);
  unsigned int* const fault = fault_word();
  if (dtype == MMT_F32)
    hipLaunchKernelGGL(tome_merge_bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)g_out, L,
                       D, go_s_n, go_s_t, set_start, t, r, size_in, size_out, pos_map,
                       (float*)g_in, gi_s_n, gi_s_t, fault);
  else
    hipLaunchKernelGGL(tome_merge_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)g_out,
                       L, D, go_s_n, go_s_t, set_start, t, r, size_in, size_out, pos_map,
                       (bf16_t*)g_in, gi_s_n, gi_s_t, fault);
  MMT_CHECK_LAUNCH("mmt_tome_merge_wavg_bwd");
  return MMT_OK;
}

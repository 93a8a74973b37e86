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

struct MatchSmem {
  int ta, tb, ta_pad, tb_pad, cs;
};

constexpr int MATCH_NT = 512;  // 8 waves per batch row

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

// One workgroup (8 waves) per batch row. LDS: a^ [ta_pad][c+1], b^ [tb_pad][c+1] fp32, per-a-row
// node arrays and per-(b tile, a row) argmax partials [PJ][ta_pad].
template <typename T, bool MFMA>
__global__ __launch_bounds__(MATCH_NT) void tome_match_kernel(const T* __restrict__ metric, int t,
                                                              int heads, int c, int64_t s_n,
                                                              int64_t s_t, int64_t s_h, int r,
                                                              int flags, int vec,
                                                              int32_t* __restrict__ unm_idx,
                                                              int32_t* __restrict__ src_idx,
                                                              int32_t* __restrict__ dst_idx,
                                                              float* __restrict__ node_max_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int n = blockIdx.x;
  const int ta = (t + 1) / 2, tb = t / 2;
  const int ta_pad = (ta + 31) & ~31, tb_pad = (tb + 31) & ~31;
  const int n_it = ta_pad / 32, n_jt = tb_pad / 32;
  const int PJ = n_jt > 4 ? n_jt : 4;
  const int cs = c + 1;
  float* A = smem;                    // normalised even tokens (the reference's a = m[::2])
  float* Bm = A + ta_pad * cs;        // normalised odd tokens  (b = m[1::2])
  float* nmax = Bm + tb_pad * cs;     // node_max [ta_pad]
  int* nidx = (int*)(nmax + ta_pad);  // node_idx [ta_pad]
  int* edge = nidx + ta_pad;          // edge_idx [ta_pad]
  float* pbest = (float*)(edge + ta_pad);  // argmax partials [PJ][ta_pad]
  int* pidx = (int*)(pbest + PJ * ta_pad);

  const T* base = metric + (int64_t)n * s_n;
  const bool cls = flags & MMT_TOME_CLASS_TOKEN;
  const bool dis = flags & MMT_TOME_DISTILL_TOKEN;
  const int rows_total = ta_pad + tb_pad;

  // Phase 1a: metric = sum over heads (fp32, h ascending). Pad rows = 0. Vector path: 8
  // contiguous c per work item, 16-B loads per head.
  for (int i = threadIdx.x; i < PJ * ta_pad; i += blockDim.x) pidx[i] = -1;
  const int cw = vec ? 8 : 1;
  const int cchunks = c / cw;
  for (int e = threadIdx.x; e < rows_total * cchunks; e += blockDim.x) {
    const int row = e / cchunks, k = (e - row * cchunks) * cw;
    int tok;
    float* dstp;
    if (row < ta_pad) {
      tok = (row < ta) ? 2 * row : -1;
      dstp = A + row * cs + k;
    } else {
      const int j = row - ta_pad;
      tok = (j < tb) ? 2 * j + 1 : -1;
      dstp = Bm + j * cs + k;
    }
    if (vec) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (tok >= 0) {
        const T* p = base + (int64_t)tok * s_t + k;
        for (int h = 0; h < heads; ++h) {
          float f[8];
          ld8f(p + (int64_t)h * s_h, f);
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] = acc[q] + f[q];
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) dstp[q] = acc[q];
    } else {
      float acc = 0.f;
      if (tok >= 0) {
        const T* p = base + (int64_t)tok * s_t + k;
        for (int h = 0; h < heads; ++h) acc = acc + ld_f32(p + (int64_t)h * s_h);
      }
      *dstp = acc;
    }
  }
  __syncthreads();

  // Phase 1b: m / ||m||_2 per row; ||m|| = sqrt of a sequential fmaf chain over c (no eps,
  // token_compression.py:72).
  for (int row = threadIdx.x; row < rows_total; row += blockDim.x) {
    const bool is_a = row < ta_pad;
    const int lr = is_a ? row : row - ta_pad;
    if (lr >= (is_a ? ta : tb)) continue;
    float* rp = (is_a ? A : Bm) + lr * cs;
    float ss = 0.f;
    for (int k = 0; k < c; ++k) ss = __fmaf_rn(rp[k], rp[k], ss);
    const float nrm = __fsqrt_rn(ss);
    for (int k = 0; k < c; ++k) rp[k] = __fdiv_rn(rp[k], nrm);
  }
  __syncthreads();

  // Phase 2: scores = a^ b^T (fmaf chain over c ascending); per (b tile, a row) argmax partials.
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  if (MFMA) {
    // S^T tile (32 b rows x 32 a cols) = b^ . a^T with v_mfma_f32_32x32x2_f32, whose result is a
    // k-ordered fmaf chain (f32 in / f32 accumulate, one rounding per step). a row i is on the
    // lane, b rows in the 16 accumulator registers: the argmax over j is lane-local. The
    // (a tile, b tile) pairs are spread over the 8 waves.
    for (int pr = wave; pr < n_it * n_jt; pr += nwaves) {
      const int it = pr / n_jt, jt = pr - it * n_jt;
      const int i = it * 32 + (lane & 31);
      const float* bp = A + (it * 32 + (lane & 31)) * cs + (lane >> 5);
      const float* ap = Bm + (jt * 32 + (lane & 31)) * cs + (lane >> 5);
      floatx16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.f;
      for (int s = 0; s < c / 2; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[2 * s], bp[2 * s], acc, 0, 0, 0);
      float best = 0.f;
      int bidx = -1;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int jj = jt * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
        if (jj >= tb) continue;
        float v = acc[q];
        if ((cls && i == 0) || (dis && jj == 0)) v = -INFINITY;
        if (bidx < 0 || argmax_better(v, jj, best, bidx)) {
          best = v;
          bidx = jj;
        }
      }
      const float ov = __shfl_xor(best, 32, 64);
      const int oi = __shfl_xor(bidx, 32, 64);
      if (oi >= 0 && (bidx < 0 || argmax_better(ov, oi, best, bidx))) {
        best = ov;
        bidx = oi;
      }
      if (lane < 32 && i < ta) {
        pbest[jt * ta_pad + i] = best;
        pidx[jt * ta_pad + i] = bidx;
      }
    }
  } else {
    // VALU path: (a row, one of PJ slices of the b rows) per thread, sequential __fmaf_rn.
    const int cwj = (tb + PJ - 1) / PJ;
    for (int e = threadIdx.x; e < ta * PJ; e += blockDim.x) {
      const int i = e / PJ, jc = e - i * PJ;
      const float* ap = A + i * cs;
      float best = 0.f;
      int bidx = -1;
      const int j1 = min(tb, (jc + 1) * cwj);
      for (int j = jc * cwj; j < j1; ++j) {
        const float* bq = Bm + j * cs;
        float acc = 0.f;
        for (int k = 0; k < c; ++k) acc = __fmaf_rn(ap[k], bq[k], acc);
        if ((cls && i == 0) || (dis && j == 0)) acc = -INFINITY;
        if (bidx < 0 || argmax_better(acc, j, best, bidx)) {
          best = acc;
          bidx = j;
        }
      }
      pbest[jc * ta_pad + i] = best;
      pidx[jc * ta_pad + i] = bidx;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ta; i += blockDim.x) {  // combine the partials (order-free)
    float best = 0.f;
    int bidx = -1;
    for (int jc = 0; jc < PJ; ++jc) {
      const int oi = pidx[jc * ta_pad + i];
      const float ov = pbest[jc * ta_pad + i];
      if (oi >= 0 && (bidx < 0 || argmax_better(ov, oi, best, bidx))) {
        best = ov;
        bidx = oi;
      }
    }
    nmax[i] = best;
    nidx[i] = bidx;
  }
  __syncthreads();

  // Phase 3: edge_idx = argsort(node_max)[::-1] (stable ascending sort, reversed) as a rank
  // count: descending total-order key, ties -> higher index first (token_compression.py:84).
  for (int i = threadIdx.x; i < ta; i += blockDim.x) {
    const uint32_t kv = sort_key(nmax[i]);
    int rank = 0;
    for (int j = 0; j < ta; ++j) {
      const uint32_t kw = sort_key(nmax[j]);
      rank += (kw > kv) || (kw == kv && j > i);
    }
    edge[rank] = i;
  }
  __syncthreads();

  // Phase 4: src = edge[:r], unm = edge[r:], dst = node_idx[src] (token_compression.py:86-88).
  for (int k = threadIdx.x; k < ta; k += blockDim.x) {
    const int e = edge[k];
    if (k < r) {
      src_idx[(int64_t)n * r + k] = e;
      dst_idx[(int64_t)n * r + k] = nidx[e];
    } else {
      unm_idx[(int64_t)n * (ta - r) + (k - r)] = e;
    }
    if (node_max_out) node_max_out[(int64_t)n * ta + k] = nmax[k];
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
    int64_t os_n, int64_t os_t, float* __restrict__ size_out, int32_t* __restrict__ pos_map) {
  __shared__ int32_t s_unm[1024];
  __shared__ int32_t s_src[512];
  __shared__ int32_t s_dst[512];
  __shared__ int32_t m_prim[kMergeRows], m_cnt[kMergeRows], m_j[kMergeRows];
  __shared__ float m_sp[kMergeRows], m_S[kMergeRows];
  __shared__ int32_t m_list[kMergeRows][kMergeSeg];
  __shared__ float m_ss[kMergeRows][kMergeSeg];
  const int n = blockIdx.x;
  const int ta = (t + 1) / 2;
  const int nu = ta - r;
  const bool dis = flags & MMT_TOME_DISTILL_TOKEN;
  const bool plain = flags & MMT_TOME_PLAIN_SUM;      // merge(x, "sum") without the size weights
  const bool scatter = !(flags & MMT_TOME_NO_SCATTER);  // merge(x, mode != "sum"): dst unchanged
  for (int k = threadIdx.x; k < nu; k += blockDim.x) s_unm[k] = unm_g[(int64_t)n * nu + k];
  for (int k = threadIdx.x; k < r; k += blockDim.x) {
    s_src[k] = src_g[(int64_t)n * r + k];
    s_dst[k] = dst_g[(int64_t)n * r + k];
  }
  __syncthreads();
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
    const int32_t* __restrict__ pos_map, T* __restrict__ g_in, int64_t gi_s_n, int64_t gi_s_t) {
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
      const int q = pos_map[(int64_t)n * t + tok];
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

size_t match_smem_bytes(int t, int c) {
  const int ta = (t + 1) / 2, tb = t / 2;
  const int ta_pad = (ta + 31) & ~31, tb_pad = (tb + 31) & ~31;
  const int PJ = tb_pad / 32 > 4 ? tb_pad / 32 : 4;
  return sizeof(float) * ((size_t)(ta_pad + tb_pad) * (c + 1) + ta_pad * 3 + 2 * PJ * ta_pad);
}

bool g_match_use_mfma = true;

}  // namespace

extern "C" void mmt_tome_set_match_path(int use_mfma) { g_match_use_mfma = use_mfma != 0; }

extern "C" int mmt_tome_match(const void* metric, int dtype, int n, int t, int heads, int c,
                              int64_t s_n, int64_t s_t, int64_t s_h, int r, int flags,
                              int32_t* unm_idx, int32_t* src_idx, int32_t* dst_idx,
                              float* node_max, mmt_stream_t stream) {
  MMT_CHECK_ARG(metric && unm_idx && src_idx && dst_idx, "mmt_tome_match: null pointer");
  MMT_CHECK_ARG(n > 0 && t >= 2 && heads >= 1 && c >= 1, "mmt_tome_match: bad shape n=%d t=%d", n, t);
  const int prot = ((flags & MMT_TOME_CLASS_TOKEN) ? 1 : 0) + ((flags & MMT_TOME_DISTILL_TOKEN) ? 1 : 0);
  MMT_CHECK_ARG(r > 0 && r <= (t - prot) / 2,
                "mmt_tome_match: r=%d must be clamped to 1..(t-protected)//2=%d", r, (t - prot) / 2);
  MMT_CHECK_ARG(dtype == MMT_F32 || dtype == MMT_BF16, "mmt_tome_match: dtype %d", dtype);
  const size_t smem = match_smem_bytes(t, c);
  MMT_CHECK_ARG(smem <= 160 * 1024, "mmt_tome_match: t=%d c=%d needs %zu B of LDS (> 160 KiB)",
                t, c, smem);
  const bool mfma = g_match_use_mfma && (c % 2 == 0);
  const int vw = dtype == MMT_BF16 ? 8 : 4;  // elements per 16 B
  const int vec = (c % 8 == 0) && (s_n % vw == 0) && (s_t % vw == 0) && (s_h % vw == 0) &&
                  ((uintptr_t)metric % 16 == 0);
  hipStream_t s = as_stream(stream);
#define LAUNCH(T, M)                                                                         \
  do {                                                                                       \
    auto kfn = tome_match_kernel<T, M>;                                                      \
    static const bool attr_set_ = (hipFuncSetAttribute((const void*)kfn,                    \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024), \
                                   true);                                                    \
    (void)attr_set_;                                                                         \
    hipLaunchKernelGGL(kfn, dim3(n), dim3(MATCH_NT), smem, s, (const T*)metric, t, heads, c, s_n, \
                       s_t, s_h, r, flags, vec, unm_idx, src_idx, dst_idx, node_max);       \
  } while (0)
  if (dtype == MMT_F32) {
    if (mfma) LAUNCH(float, true); else LAUNCH(float, false);
  } else {
    if (mfma) LAUNCH(bf16_t, true); else LAUNCH(bf16_t, false);
  }
#undef LAUNCH
  MMT_CHECK_LAUNCH("mmt_tome_match");
  return MMT_OK;
}

static int check_vec(int dtype, int D, int64_t a, int64_t b, int64_t c2, int64_t d) {
  const int V = dtype == MMT_BF16 ? 8 : 4;
  return D % V == 0 && a % V == 0 && b % V == 0 && c2 % V == 0 && d % V == 0;
}

extern "C" int mmt_tome_merge_wavg_fwd(const void* x, int dtype, int n, int L, int D, int64_t x_s_n,
                                       int64_t x_s_t, int set_start, int t, int r, int flags,
                                       const float* size_in, const int32_t* unm_idx,
                                       const int32_t* src_idx, const int32_t* dst_idx, void* x_out,
                                       int64_t o_s_n, int64_t o_s_t, float* size_out,
                                       int32_t* pos_map, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && x_out && unm_idx && src_idx && dst_idx, "mmt_tome_merge_wavg_fwd: null pointer");
  MMT_CHECK_ARG(n > 0 && L > 0 && D > 0 && t >= 2 && set_start >= 0 && set_start + t <= L,
                "mmt_tome_merge_wavg_fwd: bad shape");
  MMT_CHECK_ARG(r > 0 && r <= t / 2 && (t + 1) / 2 - r <= 1024 && r <= 512,
                "mmt_tome_merge_wavg_fwd: bad r=%d for t=%d", r, t);
  MMT_CHECK_ARG(dtype == MMT_F32 || dtype == MMT_BF16, "mmt_tome_merge_wavg_fwd: dtype");
  MMT_CHECK_ARG(check_vec(dtype, D, x_s_n, x_s_t, o_s_n, o_s_t),
                "mmt_tome_merge_wavg_fwd: D and strides must be multiples of 16 bytes");
  dim3 grid(n, (L - r + kMergeRows - 1) / kMergeRows);
  hipStream_t s = as_stream(stream);
  if (dtype == MMT_F32)
    hipLaunchKernelGGL(tome_merge_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)x, L, D,
                       x_s_n, x_s_t, set_start, t, r, flags, size_in, unm_idx, src_idx, dst_idx,
                       (float*)x_out, o_s_n, o_s_t, size_out, pos_map);
  else
    hipLaunchKernelGGL(tome_merge_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, L,
                       D, x_s_n, x_s_t, set_start, t, r, flags, size_in, unm_idx, src_idx,
                       dst_idx, (bf16_t*)x_out, o_s_n, o_s_t, size_out, pos_map);
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
  if (dtype == MMT_F32)
    hipLaunchKernelGGL(tome_merge_bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)g_out, L,
                       D, go_s_n, go_s_t, set_start, t, r, size_in, size_out, pos_map,
                       (float*)g_in, gi_s_n, gi_s_t);
  else
    hipLaunchKernelGGL(tome_merge_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)g_out,
                       L, D, go_s_n, go_s_t, set_start, t, r, size_in, size_out, pos_map,
                       (bf16_t*)g_in, gi_s_n, gi_s_t);
  MMT_CHECK_LAUNCH("mmt_tome_merge_wavg_bwd");
  return MMT_OK;
}

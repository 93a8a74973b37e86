/* ORACLE — test infrastructure only. Never linked into, or called by, the product path.
 *
 * Canonical-arithmetic CPU restatement of ToMe from the reference
 *   multi_modal_transformers/tokenizers/token_compression.py
 *     bipartite_soft_matching  :54-112
 *     merge (mode "sum")       :90-109
 *     merge_wavg               :114-129
 * The reference evaluates these with XLA, whose fp32 reduction order is unspecified, so the
 * bit-exact contract is defined by the canonical order below ("ToMe canonical
 * arithmetic"), which the HIP kernels follow too:
 *   - metric row = sum over heads h = 0..H-1 (fp32, left to right, from 0.0f);
 *   - ||m|| = sqrtf(fmaf chain over k ascending, from 0.0f); m^ = m / ||m|| (IEEE division);
 *   - score(i,j) = fmaf chain over k ascending of a^[i][k] * b^[j][k], from 0.0f;
 *   - node_idx = argmax_j with NaN as the maximum and the lowest index on ties (jnp.argmax);
 *   - edge order = descending lax.sort total order, ties -> higher index first (argsort()[::-1]);
 *   - merge: dst = x_b*s_b, then for i = 0..r-1: dst[dst_idx[i]] += x_src_i*s_src_i (separate
 *     multiply and add roundings), sizes likewise, out = dst / size (IEEE division).
 * Compile with -ffp-contract=off (oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int argmax_better(float v, int j, float bv, int bj) {
  if (isnan(bv)) return isnan(v) && j < bj;
  if (isnan(v)) return 1;
  return v > bv || (v == bv && j < bj);
}

static uint32_t sort_key(float v) {
  uint32_t b;
  if (isnan(v)) return 0xffffffffu;
  memcpy(&b, &v, 4);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

/* metric: fp32 host array, element (b,i,h,k) at metric[b*s_n + i*s_t + h*s_h + k]. */
int tome_ref_match(const float* metric, int n, int t, int heads, int c, int64_t s_n, int64_t s_t,
                   int64_t s_h, int r, int flags, int32_t* unm_idx, int32_t* src_idx,
                   int32_t* dst_idx, float* node_max) {
  const int ta = (t + 1) / 2, tb = t / 2;
  const int cls = flags & 1, dis = flags & 2;
  float* m = (float*)malloc(sizeof(float) * (size_t)t * c);
  float* nmax = (float*)malloc(sizeof(float) * ta);
  int* nidx = (int*)malloc(sizeof(int) * ta);
  int* edge = (int*)malloc(sizeof(int) * ta);
  if (!m || !nmax || !nidx || !edge) return -1;
  for (int b = 0; b < n; ++b) {
    for (int i = 0; i < t; ++i) {
      float ss = 0.f;
      for (int k = 0; k < c; ++k) {
        float acc = 0.f;
        for (int h = 0; h < heads; ++h) acc = acc + metric[b * s_n + i * s_t + h * s_h + k];
        m[i * c + k] = acc;
      }
      for (int k = 0; k < c; ++k) ss = fmaf(m[i * c + k], m[i * c + k], ss);
      const float nrm = sqrtf(ss);
      for (int k = 0; k < c; ++k) m[i * c + k] = m[i * c + k] / nrm;
    }
    for (int i = 0; i < ta; ++i) {
      const float* a = m + (2 * i) * c;
      float best = 0.f;
      int bidx = -1;
      for (int j = 0; j < tb; ++j) {
        const float* bb = m + (2 * j + 1) * c;
        float acc = 0.f;
        for (int k = 0; k < c; ++k) acc = fmaf(a[k], bb[k], acc);
        if ((cls && i == 0) || (dis && j == 0)) acc = -INFINITY;
        if (bidx < 0 || argmax_better(acc, j, best, bidx)) {
          best = acc;
          bidx = j;
        }
      }
      nmax[i] = best;
      nidx[i] = bidx;
    }
    for (int i = 0; i < ta; ++i) {
      const uint32_t kv = sort_key(nmax[i]);
      int rank = 0;
      for (int j = 0; j < ta; ++j) {
        const uint32_t kw = sort_key(nmax[j]);
        rank += (kw > kv) || (kw == kv && j > i);
      }
      edge[rank] = i;
    }
    for (int k = 0; k < ta; ++k) {
      if (k < r) {
        src_idx[b * r + k] = edge[k];
        dst_idx[b * r + k] = nidx[edge[k]];
      } else {
        unm_idx[b * (ta - r) + k - r] = edge[k];
      }
      if (node_max) node_max[b * ta + k] = nmax[k];
    }
  }
  free(m);
  free(nmax);
  free(nidx);
  free(edge);
  return 0;
}

/* merge_wavg over the token set (n, t, D) (contiguous fp32). size_in may be NULL (ones).
 * x_out (n, t - r, D), size_out (n, t - r). */
int tome_ref_merge_wavg(const float* x, const float* size_in, int n, int t, int D, int r, int flags,
                        const int32_t* unm_idx, const int32_t* src_idx, const int32_t* dst_idx,
                        float* x_out, float* size_out) {
  const int ta = (t + 1) / 2, tb = t / 2, nu = ta - r;
  const int dis = flags & 2, plain = flags & 4, scatter = !(flags & 8);
  float* dst = (float*)malloc(sizeof(float) * (size_t)tb * D);
  float* dsz = (float*)malloc(sizeof(float) * tb);
  if (!dst || !dsz) return -1;
  for (int b = 0; b < n; ++b) {
    const float* xb = x + (size_t)b * t * D;
    const float* sb = size_in ? size_in + (size_t)b * t : NULL;
    float* ob = x_out + (size_t)b * (t - r) * D;
    float* osz = size_out + (size_t)b * (t - r);
    /* dst = (x*size)[1::2] ; size[1::2] */
    for (int j = 0; j < tb; ++j) {
      const float s = sb ? sb[2 * j + 1] : 1.f;
      const float w = plain ? 1.f : s;
      for (int d = 0; d < D; ++d) dst[j * D + d] = xb[(2 * j + 1) * D + d] * w;
      dsz[j] = s;
    }
    for (int i = 0; i < r && scatter; ++i) {
      const int st = 2 * src_idx[b * r + i], j = dst_idx[b * r + i];
      const float s = sb ? sb[st] : 1.f;
      const float w = plain ? 1.f : s;
      for (int d = 0; d < D; ++d) dst[j * D + d] = dst[j * D + d] + xb[st * D + d] * w;
      dsz[j] = dsz[j] + s;
    }
    /* result rows in reference order */
    for (int q = 0; q < t - r; ++q) {
      int ui = -1, dj = -1;
      if (!dis) {
        if (q < nu) ui = q; else dj = q - nu;
      } else {
        if (q == 0) ui = 0;
        else if (q == 1) dj = 0;
        else if (q < 1 + nu) ui = q - 1;
        else dj = q - nu;
      }
      if (ui >= 0) {
        const int tok = 2 * unm_idx[b * nu + ui];
        const float s = sb ? sb[tok] : 1.f;
        for (int d = 0; d < D; ++d)
          ob[q * D + d] = plain ? xb[tok * D + d] : (xb[tok * D + d] * s) / s;
        osz[q] = s;
      } else {
        for (int d = 0; d < D; ++d) ob[q * D + d] = plain ? dst[dj * D + d] : dst[dj * D + d] / dsz[dj];
        osz[q] = dsz[dj];
      }
    }
  }
  free(dst);
  free(dsz);
  return 0;
}

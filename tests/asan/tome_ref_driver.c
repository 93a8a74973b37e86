/* The canonical ToMe oracle (oracle/tome_ref.c) under AddressSanitizer + UBSan (SURVEY §5
 * "sanitizers"; built by tests/asan/build_asan.sh). Drives tome_ref_match and tome_ref_merge_wavg
 * over the edge shapes the GPU parity tests use — odd t, t = 2 and 3, the largest r, class /
 * distill protection, plain-sum and no-scatter merges, several heads, strided metrics — with
 * exactly sized heap buffers (any read or write past them is an ASan report), and checks the
 * structural invariants: unm + src partition the a half, dst indexes the b half, the merged
 * sizes add up to t. Test infrastructure only. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int tome_ref_match(const float* metric, int n, int t, int heads, int c, int64_t s_n, int64_t s_t,
                   int64_t s_h, int r, int flags, int32_t* unm_idx, int32_t* src_idx,
                   int32_t* dst_idx, float* node_max);
int tome_ref_merge_wavg(const float* x, const float* size_in, int n, int t, int D, int r, int flags,
                        const int32_t* unm_idx, const int32_t* src_idx, const int32_t* dst_idx,
                        float* x_out, float* size_out);

static int fails = 0;
static uint32_t lcg = 12345u;
static float frand(void) {
  lcg = lcg * 1664525u + 1013904223u;
  return (float)((lcg >> 8) & 0xffff) / 32768.f - 1.f;
}

static void run(int n, int t, int heads, int c, int r, int flags, int D, int pad) {
  const int ta = (t + 1) / 2, tb = t / 2, nu = ta - r;
  const int64_t s_h = c + pad, s_t = heads * s_h, s_n = t * s_t;
  float* m = malloc(sizeof(float) * (size_t)(n * s_n));
  for (int64_t i = 0; i < n * s_n; ++i) m[i] = (i % 7 == 3) ? 0.f : frand();  /* zero rows too */
  int32_t* unm = malloc(sizeof(int32_t) * (size_t)(n * nu + 1));
  int32_t* src = malloc(sizeof(int32_t) * (size_t)(n * r));
  int32_t* dst = malloc(sizeof(int32_t) * (size_t)(n * r));
  float* nmax = malloc(sizeof(float) * (size_t)(n * ta));
  if (tome_ref_match(m, n, t, heads, c, s_n, s_t, s_h, r, flags, unm, src, dst, nmax) != 0) {
    fprintf(stderr, "FAIL match rc n=%d t=%d r=%d\n", n, t, r);
    ++fails;
  }
  for (int b = 0; b < n; ++b) {
    char* seen = calloc((size_t)ta, 1);
    for (int i = 0; i < nu; ++i) {
      const int v = unm[b * nu + i];
      if (v < 0 || v >= ta || seen[v]++) { fprintf(stderr, "FAIL unm t=%d\n", t); ++fails; break; }
    }
    for (int i = 0; i < r; ++i) {
      const int v = src[b * r + i], d = dst[b * r + i];
      if (v < 0 || v >= ta || seen[v]++) { fprintf(stderr, "FAIL src t=%d\n", t); ++fails; break; }
      if (d < 0 || d >= tb) { fprintf(stderr, "FAIL dst t=%d\n", t); ++fails; break; }
    }
    free(seen);
  }
  float* x = malloc(sizeof(float) * (size_t)(n * t * D));
  float* sz = malloc(sizeof(float) * (size_t)(n * t));
  for (int i = 0; i < n * t * D; ++i) x[i] = frand();
  for (int i = 0; i < n * t; ++i) sz[i] = 1.f + (float)(i % 3);
  float* xo = malloc(sizeof(float) * (size_t)(n * (t - r) * D));
  float* so = malloc(sizeof(float) * (size_t)(n * (t - r)));
  for (int mode = 0; mode < 2; ++mode) {
    const int mflags = (flags & 3) | (mode ? 4 : 0);
    if (tome_ref_merge_wavg(x, mode ? NULL : sz, n, t, D, r, mflags, unm, src, dst, xo, so) != 0) {
      fprintf(stderr, "FAIL merge rc\n");
      ++fails;
    }
    for (int b = 0; b < n; ++b) {
      double tot = 0, want = 0;
      for (int q = 0; q < t - r; ++q) tot += so[b * (t - r) + q];
      for (int i = 0; i < t; ++i) want += mode ? 1.0 : sz[b * t + i];
      if (tot != want) { fprintf(stderr, "FAIL sizes t=%d: %g vs %g\n", t, tot, want); ++fails; }
    }
  }
  if (tome_ref_merge_wavg(x, sz, n, t, D, r, (flags & 3) | 8, unm, src, dst, xo, so) != 0) ++fails;
  free(m); free(unm); free(src); free(dst); free(nmax); free(x); free(sz); free(xo); free(so);
}

int main(void) {
  run(4, 256, 1, 64, 16, 0, 64, 0);
  run(3, 257, 6, 64, 16, 0, 32, 8);   /* odd t, strided heads */
  run(2, 64, 1, 32, 32, 0, 16, 0);    /* r = t/2: every a token merges */
  run(2, 64, 1, 32, 31, 1, 16, 0);    /* class token protected */
  run(2, 64, 1, 32, 31, 2, 16, 0);    /* distill token protected */
  run(2, 64, 1, 32, 30, 3, 16, 0);    /* both */
  run(5, 2, 1, 8, 1, 0, 8, 0);        /* t = 2 */
  run(5, 3, 1, 8, 1, 0, 8, 0);        /* t = 3 */
  run(2, 31, 1, 6, 7, 0, 12, 4);      /* odd c, padding */
  run(2, 1024, 12, 64, 32, 0, 16, 0); /* hi-res block 0 */
  run(1, 2048, 1, 64, 64, 0, 8, 0);   /* the largest t */
  printf(fails ? "FAILED %d\n" : "OK\n", fails);
  return fails != 0;
}

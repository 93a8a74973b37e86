// DDPM inference sampler for gfx950: DiffusionActionHead.predict_action
// (reference multi_modal_transformers/action_heads/diffusion.py:146-209) as ONE launch.
//
// The denoiser's first Dense acts on concatenate([noisy, time_emb, readout]) (OctoDenoise :61),
// so it splits along its input:
//   W1 [x | temb_t | r] + b1 = W1x x + (W1t temb_t + b1) + W1r r = W1x x + Q[t] + P[b]
// Q (steps, H) and P (B, H) are plain GEMMs issued by the host wrapper before this call (the
// library's MFMA GEMM); what remains per step and sample is an (H x 8) and an (8 x H)
// matrix-vector product, a ReLU and the update
//   x <- clip(c1_t (x - c2_t eps_hat) + c3_t z, -5, 5)                      (:182-188)
// This kernel runs all steps for a sample with its state in registers: one wave per sample, the
// H hidden units spread over the lanes (unit j = lane + 64 u), W1x rows and W2 columns of those
// units in registers, Q[t] read from L2 each step. eps_hat needs one wave reduction per action
// component per step; no LDS, no barriers, no global writes until the end.
//
// Reference quirks kept: z is drawn once per sample (:198-200) and, because the scan never splits
// the keys (:178, :190), reused as every step's noise; noise is added at t = 0 too; the action
// dimension is hard-coded to 8 (:200).
#include <math.h>

#include "common.h"

using namespace mmt;

namespace {

constexpr int SA = 8;     // action dimension (diffusion.py:200)
constexpr int SNT = 256;  // threads per workgroup: 4 samples

template <int NU>
__global__ __launch_bounds__(SNT) void diffusion_sample_kernel(
    const uint32_t* __restrict__ rng, int B, int steps, int64_t sample_offset,
    const float* __restrict__ P, int64_t ld_p, const float* __restrict__ Q, int64_t ld_q,
    const bf16_t* __restrict__ w1, int64_t ld_w1, const bf16_t* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ coef, const float* __restrict__ z_in,
    int H, float* __restrict__ actions, float* __restrict__ z_out) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (SNT / 64) + (threadIdx.x >> 6);
  if (b >= B) return;  // wave-uniform: the whole wave leaves

  float w1x[NU][SA], w2c[NU][SA], pb[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int j = lane + 64 * u;
    const int jj = j < H ? j : H - 1;  // clamped, zeroed below
    const float keep = j < H ? 1.f : 0.f;
    const uint4 row = *reinterpret_cast<const uint4*>(w1 + (int64_t)jj * ld_w1);  // W1[j][0:8]
    const uint32_t rw[4] = {row.x, row.y, row.z, row.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      w1x[u][2 * q] = keep * __uint_as_float(rw[q] << 16);
      w1x[u][2 * q + 1] = keep * __uint_as_float(rw[q] & 0xffff0000u);
    }
#pragma unroll
    for (int a = 0; a < SA; ++a) w2c[u][a] = keep * bf2f(w2[(int64_t)a * H + jj]);
    pb[u] = keep * P[(int64_t)b * ld_p + jj];
  }

  float z[SA], x[SA];
  if (z_in) {
#pragma unroll
    for (int a = 0; a < SA; ++a) z[a] = z_in[(int64_t)b * SA + a];
  } else {
    const uint32_t key = stream_key(rng[0], rng[1], 0xFFFEu, 3);
#pragma unroll
    for (int a = 0; a < SA; ++a) {
      const uint32_t c = (uint32_t)((sample_offset + b) * SA + a);
      const float u1 = ((draw_u32(key, 2 * c) >> 8) + 1) * (1.f / 16777216.f);  // (0, 1]
      const float u2 = (draw_u32(key, 2 * c + 1) >> 8) * (1.f / 16777216.f);
      z[a] = sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
    }
  }
#pragma unroll
  for (int a = 0; a < SA; ++a) x[a] = z[a];  // x_T = z

  float b2r[SA];
#pragma unroll
  for (int a = 0; a < SA; ++a) b2r[a] = b2[a];

#pragma unroll 1
  for (int t = steps - 1; t >= 0; --t) {
    const float* q = Q + (int64_t)t * ld_q;
    float e[SA];
#pragma unroll
    for (int a = 0; a < SA; ++a) e[a] = 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int j = lane + 64 * u;
      float h = pb[u] + (j < H ? 1.f : 0.f) * q[j < H ? j : H - 1];
#pragma unroll
      for (int a = 0; a < SA; ++a) h = fmaf(x[a], w1x[u][a], h);
      h = fmaxf(h, 0.f);
#pragma unroll
      for (int a = 0; a < SA; ++a) e[a] = fmaf(h, w2c[u][a], e[a]);
    }
    const float c1 = coef[3 * t], c2 = coef[3 * t + 1], c3 = coef[3 * t + 2];
#pragma unroll
    for (int a = 0; a < SA; ++a) {
      const float eps = wave_sum(e[a]) + b2r[a];
      x[a] = fminf(fmaxf(c1 * (x[a] - c2 * eps) + c3 * z[a], -5.f), 5.f);
    }
  }

  if (lane < SA) {
    float xv = 0.f, zv = 0.f;
#pragma unroll
    for (int a = 0; a < SA; ++a)
      if (a == lane) {
        xv = x[a];
        zv = z[a];
      }
    actions[(int64_t)b * SA + lane] = xv;
    if (z_out) z_out[(int64_t)b * SA + lane] = zv;
  }
}

}  // namespace

extern "C" int mmt_diffusion_sample(const uint32_t* rng, int B, int A, int steps,
                                    int64_t sample_offset, const float* P, int64_t ld_p,
                                    const float* Q, int64_t ld_q, const void* w1, int64_t ld_w1,
                                    const void* w2, const float* b2, const float* coef,
                                    const float* z_in, int H, float* actions, float* z_out,
                                    mmt_stream_t stream) {
  MMT_CHECK_ARG(P && Q && w1 && w2 && b2 && coef && actions && B > 0 && steps > 0 && H > 0,
                "mmt_diffusion_sample: args");
  MMT_CHECK_ARG(A == SA, "mmt_diffusion_sample: the action dimension must be %d (diffusion.py:200)",
                SA);
  MMT_CHECK_ARG(z_in || rng, "mmt_diffusion_sample: need rng or an injected initial sample");
  MMT_CHECK_ARG(ld_p >= H && ld_q >= H && ld_w1 >= SA, "mmt_diffusion_sample: leading dims");
  MMT_CHECK_ARG(ld_w1 % 8 == 0 && ((uintptr_t)w1 & 15) == 0,
                "mmt_diffusion_sample: W1 rows must start on 16-B boundaries");
  MMT_CHECK_ARG(H <= 1024, "mmt_diffusion_sample: hidden width %d > 1024", H);
  const int nu = (H + 63) / 64;
  const dim3 grid((B + SNT / 64 - 1) / (SNT / 64));
  hipStream_t s = as_stream(stream);
#define MMT_SAMPLE(NU_)                                                                        \
  hipLaunchKernelGGL(diffusion_sample_kernel<NU_>, grid, dim3(SNT), 0, s, rng, B, steps,        \
                     sample_offset, P, ld_p, Q, ld_q, (const bf16_t*)w1, ld_w1,                \
                     (const bf16_t*)w2, b2, coef, z_in, H, actions, z_out)
  if (nu <= 2) MMT_SAMPLE(2);
  else if (nu <= 4) MMT_SAMPLE(4);
  else if (nu <= 6) MMT_SAMPLE(6);
  else if (nu <= 8) MMT_SAMPLE(8);
  else if (nu <= 12) MMT_SAMPLE(12);
  else MMT_SAMPLE(16);
#undef MMT_SAMPLE
  MMT_CHECK_LAUNCH("mmt_diffusion_sample");
  return MMT_OK;
}

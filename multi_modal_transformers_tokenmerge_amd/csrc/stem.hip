// Gato-style image tokenizer (reference tokenizers/images/image_tokenizer.py) for gfx950:
//   image_to_patches (:35-71) + normalisation 2*(x/255)-1        -> fused into patch_im2col
//   encode_patch_position (:74-132)                              -> patch_positions
//   ResNetV2Block stem (:140-178, model_configs/.../gato_resnet.yaml:41-104):
//     Conv 12x12 s2 VALID (im2col here + MFMA GEMM) -> max_pool 3x3 s1 VALID (maxpool_patch)
//     -> 2 x [GroupNorm(32, eps 1e-6) -> gelu(tanh) -> Conv 3x3 SAME] (groupnorm_gelu + GEMM)
// At patch 16 the pooled map is 1 x 1, so each 3x3 SAME conv reduces to its centre tap (a
// 64 x 64 Dense) and flatten is the identity; GroupNorm statistics span all images x patches x
// (C / G) channels of a sample (flax GroupNorm reduces every non-batch axis).
#include <math.h>

#include <algorithm>

#include "common.h"

using namespace mmt;

namespace {

// image_tokenizer.py:67-68 in the reference's fp32 order: 2 * (x / 255) - 1 (division, exact
// doubling, subtraction; no fused multiply-add). normalize == 0 passes x through.
__device__ __forceinline__ float normalize_px(float x, float normalize) {
  return normalize != 0.f ? __fsub_rn(__fmul_rn(__fdiv_rn(x, 255.f), 2.f), 1.f) : x;
}

// One thread per (row, 8-element chunk) of the im2col matrix [rows][K], rows =
// ((b*I + i)*NP + p)*OH*OW + oy*OW + ox, K = KH*KW*C in (ky, kx, c) order (Flax HWIO kernels).
template <typename T>
__global__ void patch_im2col_kernel(const T* __restrict__ img, int64_t s_img, int Himg, int C,
                                    int P, int KH, int KW, int S, int OH, int OW, int64_t rows,
                                    int K, bf16_t* __restrict__ out, float in_scale, float in_bias) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int kchunks = K / 8;
  if (idx >= rows * kchunks) return;
  const int64_t row = idx / kchunks;
  const int k0 = (int)(idx - row * kchunks) * 8;
  const int ox = row % OW, oy = (row / OW) % OH;
  const int64_t pimg = row / ((int64_t)OH * OW);  // (b*I + i)*NP + p
  const int PPD = Himg / P, NP = PPD * PPD;
  const int p = pimg % NP;
  const int64_t bi = pimg / NP;
  const int py = p / PPD, px = p % PPD;  // raster order "(h p1) (w p2) -> (h w)"
  const T* base = img + bi * s_img;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = k0 + e;
    const int c = k % C, kx = (k / C) % KW, ky = k / (C * KW);
    const int yy = py * P + oy * S + ky, xx = px * P + ox * S + kx;
    const float raw = (float)base[((int64_t)yy * Himg + xx) * C + c];
    v[e] = normalize_px(raw, in_scale);
  }
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = (uint32_t)f2bf(v[2 * q]) | ((uint32_t)f2bf(v[2 * q + 1]) << 16);
  *reinterpret_cast<uint4*>(out + row * K + k0) = make_uint4(w[0], w[1], w[2], w[3]);
}

// Same im2col, one thread per (row, ky): the KW*C values of a kernel row are contiguous in the
// NHWC image, so a thread reads them in order and writes KW*C bf16 with 8-byte stores (needs
// KW*C % 4 == 0). The per-element index arithmetic of the generic kernel is gone.
template <typename T, int SEG>
__global__ void patch_im2col_rows_kernel(const T* __restrict__ img, int64_t s_img, int Himg, int C,
                                         int P, int KH, int S, int OH, int OW, int64_t rows, int K,
                                         bf16_t* __restrict__ out, float in_scale, float in_bias) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * KH) return;
  const int64_t row = idx / KH;
  const int ky = (int)(idx - row * KH);
  const int ox = row % OW, oy = (row / OW) % OH;
  const int64_t pimg = row / ((int64_t)OH * OW);
  const int PPD = Himg / P, NP = PPD * PPD;
  const int p = pimg % NP;
  const int64_t bi = pimg / NP;
  const int py = p / PPD, px = p % PPD;
  const T* src = img + bi * s_img + ((int64_t)(py * P + oy * S + ky) * Himg + px * P + ox * S) * C;
  bf16_t* dst = out + row * K + ky * SEG;
#pragma unroll
  for (int e = 0; e < SEG; e += 4) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = normalize_px((float)src[e + q], in_scale);
    *reinterpret_cast<uint2*>(dst + e) =
        make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                   (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
  }
}

// Same im2col for uint8 images, PG patches per 256-thread workgroup through LDS: the patches'
// P x P x C bytes are read as dwords (P*C % 4 == 0), normalised once into a bf16 LDS image, and
// the PG*OH*OW rows of K values are written as consecutive 16-B chunks (fully coalesced); the
// row-segment kernel's 8-B stores touched a new cache line every 72 B of a wave's store.
template <int SEG, int PG>
__global__ __launch_bounds__(256) void patch_im2col_lds_kernel(
    const uint8_t* __restrict__ img, int64_t s_img, int Himg, int C, int P, int KH, int S, int OH,
    int OW, int64_t npatch, int K, bf16_t* __restrict__ out, float in_scale) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  bf16_t* pix = reinterpret_cast<bf16_t*>(dsm);  // [PG][P][P*C]
  const int PPD = Himg / P, NP = PPD * PPD, RB = P * C;  // bytes per patch row
  const int64_t p0 = (int64_t)blockIdx.x * PG;
  const int np = (int)min<int64_t>(PG, npatch - p0);
  const int words = np * P * (RB / 4);
  for (int w = threadIdx.x; w < words; w += 256) {
    const int pl = w / (P * (RB / 4)), rem = w - pl * (P * (RB / 4));
    const int y = rem / (RB / 4), xw = rem - y * (RB / 4);
    const int64_t pimg = p0 + pl;
    const int p = (int)(pimg % NP);
    const int64_t bi = pimg / NP;
    const int py = p / PPD, px = p % PPD;
    const uint32_t u = *reinterpret_cast<const uint32_t*>(
        img + bi * s_img + ((int64_t)(py * P + y) * Himg + px * P) * C + xw * 4);
    bf16_t* d = pix + (pl * P + y) * RB + xw * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = f2bf(normalize_px((float)((u >> (8 * q)) & 0xffu), in_scale));
  }
  __syncthreads();
  const int per = OH * OW, kc = K / 8;
  const int chunks = np * per * kc;
  bf16_t* obase = out + p0 * per * K;
  for (int ch = threadIdx.x; ch < chunks; ch += 256) {
    const int r = ch / kc, k0 = (ch - r * kc) * 8;
    const int pl = r / per, o = r - pl * per;
    const int oy = o / OW, ox = o - oy * OW;
    const bf16_t* src = pix + (pl * P + oy * S) * RB + ox * S * C;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t h2[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int k = k0 + 2 * q + e, ky = k / SEG;
        h2[e] = src[ky * RB + (k - ky * SEG)];
      }
      w[q] = h2[0] | (h2[1] << 16);
    }
    *reinterpret_cast<uint4*>(obase + (int64_t)r * K + k0) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ---------------------------------------------------------------- fused stem conv + max-pool
// The 12x12 stride-2 VALID conv of the 64-channel stem on 16x16 RGB uint8 patches, then the 3x3
// max-pool over its 3x3 map, without the im2col matrix: a tile is 16 consecutive patches of one
// patch row (12 KB of the image), normalised once into LDS as bf16 (patch-local rows of 56
// elements, 48 used; patch stride 902 elements = 3 banks mod 64, so the 16 patches x 4 k-groups
// of an A-fragment read hit at most 2 lanes per bank). K = 432 = 12 ky x 36 (kx, c) is padded to
// 12 x 40 (weights zero in the pad) so an 8-element k-chunk never crosses a kernel row. Wave w
// owns channels 16w .. 16w+15 with its weight fragments in registers for the whole launch; rows of
// the 16x16x32 MFMA are the 16 patches, one accumulator per conv position, so the max-pool is a
// register max over the 9 accumulators (first maximum, as maxpool_patch_kernel).
constexpr int SCP_RB = 56, SCP_PS = 902, SCP_KS = 15;  // row / patch stride (elements), k-steps
constexpr int STEM_PXW = 12;  // pixel dwords per thread per tile (16 rows x 16 patches x 48 B / 256)
__global__ __launch_bounds__(256, 2) void stem_conv_pool_kernel(
    const uint8_t* __restrict__ img, int64_t s_img, int Himg, int64_t n_tiles,
    const bf16_t* __restrict__ w, const float* __restrict__ bias, float* __restrict__ pooled,
    uint8_t* __restrict__ arg) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  typedef float floatx4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) bf16_t pix[16 * SCP_PS];
  __shared__ bf16_t lut[256];  // bf16(2 * (x / 255) - 1) per byte value
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l15 = lane & 15, lg = lane >> 4;
  const int PPD = Himg / 16, G16 = (PPD + 15) / 16, NP = PPD * PPD;
  for (int i = threadIdx.x; i < 16 * SCP_PS; i += 256) pix[i] = 0;  // pads stay zero
  lut[threadIdx.x] = f2bf(normalize_px((float)threadIdx.x, 1.f));
  // weight fragments: column n = 16 wave + l15, k' = 32 ks + 8 lg + j -> (ky, e) = (k' / 40, k' % 40)
  bf16x8 bf[SCP_KS];
  const int n = 16 * wave + l15;
#pragma unroll
  for (int ks = 0; ks < SCP_KS; ++ks) {
    const int kc = 32 * ks + 8 * lg, ky = kc / 40, e0 = kc % 40;
    short v8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v8[j] = e0 + j < 36 ? (short)w[n * 432 + ky * 36 + e0 + j] : (short)0;
    bf[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<short __attribute__((ext_vector_type(8)))*>(v8));
  }
  const float bn = bias[n];
  // A-fragment word offsets of this lane (patch l15, k-group lg) per k-step, without the position
  int aoff[SCP_KS];
#pragma unroll
  for (int ks = 0; ks < SCP_KS; ++ks) {
    const int kc = 32 * ks + 8 * lg, ky = kc / 40, e0 = kc % 40;
    aoff[ks] = l15 * SCP_PS + ky * SCP_RB + e0;
  }
  // The tile's 16 pixel rows x np*48 bytes as dwords (12 per thread), loaded into registers one
  // tile ahead so the global latency hides under the previous tile's MFMAs.
  uint32_t px[STEM_PXW];
  auto fetch = [&](int64_t t) {
    const int64_t bi = t / (PPD * G16);
    const int rem = (int)(t - bi * PPD * G16), py = rem / G16, px0 = (rem - py * G16) * 16;
    const int wpr = min(16, PPD - px0) * 12;
    const uint8_t* src = img + bi * s_img + ((int64_t)py * 16 * Himg + px0 * 16) * 3;
#pragma unroll
    for (int j = 0; j < STEM_PXW; ++j) {
      const int i = min((int)threadIdx.x + 256 * j, 16 * wpr - 1), y = i / wpr, xw = i - y * wpr;
      px[j] = *reinterpret_cast<const uint32_t*>(src + (int64_t)y * Himg * 3 + xw * 4);
    }
  };
  if (blockIdx.x < n_tiles) fetch(blockIdx.x);
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int64_t bi = t / (PPD * G16);
    const int rem = (int)(t - bi * PPD * G16), py = rem / G16, px0 = (rem - py * G16) * 16;
    const int np = min(16, PPD - px0);
    __syncthreads();  // the previous tile's fragment reads are done
    {  // normalise (image_tokenizer.py:67-68 order) into the patch-local LDS rows
      const int wpr = np * 12;
#pragma unroll
      for (int j = 0; j < STEM_PXW; ++j) {
        const int i = threadIdx.x + 256 * j;
        if (i >= 16 * wpr) break;
        const int y = i / wpr, xw = i - y * wpr;
        const int byte0 = xw * 4, pl = byte0 / 48, off = byte0 - pl * 48;  // 48 = 16 px x 3
        bf16_t* d = pix + pl * SCP_PS + y * SCP_RB + off;
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = lut[(px[j] >> (8 * q)) & 0xffu];
      }
    }
    __syncthreads();
    if (t + gridDim.x < n_tiles) fetch(t + gridDim.x);
    floatx4 acc[9];
#pragma unroll
    for (int pos = 0; pos < 9; ++pos) acc[pos] = floatx4{0.f, 0.f, 0.f, 0.f};
    // A fragments of k-step ks + 1 (all 9 positions) are read while the MFMAs of ks run
    auto afrag = [&](int ks, int pos) {
      const int oy = pos / 3, ox = pos % 3;
      const uint32_t* q = reinterpret_cast<const uint32_t*>(pix + aoff[ks] + oy * 2 * SCP_RB + ox * 6);
      const uint32_t a4[4] = {q[0], q[1], q[2], q[3]};
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(a4));
    };
    bf16x8 acur[9], anxt[9];
#pragma unroll
    for (int pos = 0; pos < 9; ++pos) acur[pos] = afrag(0, pos);
#pragma unroll
    for (int ks = 0; ks < SCP_KS; ++ks) {
      if (ks + 1 < SCP_KS)
#pragma unroll
        for (int pos = 0; pos < 9; ++pos) anxt[pos] = afrag(ks + 1, pos);
#pragma unroll
      for (int pos = 0; pos < 9; ++pos)
        acc[pos] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[pos], bf[ks], acc[pos], 0, 0, 0);
#pragma unroll
      for (int pos = 0; pos < 9; ++pos) acur[pos] = anxt[pos];
    }
    // lane holds patches 4 lg + r, channel n: conv + bias, max over the 9 positions
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pl = 4 * lg + r;
      float best = acc[0][r] + bn;
      int bpos = 0;
#pragma unroll
      for (int pos = 1; pos < 9; ++pos) {
        const float v = acc[pos][r] + bn;
        if (v > best) {
          best = v;
          bpos = pos;
        }
      }
      if (pl < np) {
        const int64_t pimg = bi * NP + (int64_t)py * PPD + px0 + pl;
        pooled[pimg * 64 + n] = best;
        arg[pimg * 64 + n] = (uint8_t)bpos;
      }
    }
  }
}

// Weight gradient of the same conv without im2col: dW[n][k] = sum over patches p and positions
// s of G[p, s, n] A[p, s, k], G the max-pool backward (dpooled[p, n] at s = argmax[p, n], else 0,
// rounded to bf16 as maxpool_patch_bwd stores it). A tile = 16 patches of a patch row: the pixels
// normalised into LDS patch-minor ([y][x*3 + c][patch], so 8 patches of one k are one 16-B read)
// and G per position ([s][n][patch]); per position one 32x32x16 MFMA per (32 channels, 32 k)
// block with the 16 patches as the reduction. Wave w owns the k-blocks w, w + 4, ... of the
// 12 x 40 padded K; each workgroup writes its partial (64, 432) to a slab row.
constexpr int SCW_XE = 56;  // padded elements per pixel row (48 used)
__global__ __launch_bounds__(256, 2) void stem_conv_wgrad_kernel(
    const uint8_t* __restrict__ img, int64_t s_img, int Himg, int64_t n_tiles,
    const float* __restrict__ dpooled, const uint8_t* __restrict__ arg, float* __restrict__ slab) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  typedef float floatx16 __attribute__((ext_vector_type(16)));
  __shared__ __attribute__((aligned(16))) bf16_t pixT[16 * SCW_XE * 16];  // [y][xe][patch]
  __shared__ __attribute__((aligned(16))) bf16_t gt[9 * 64 * 16];         // [s][n][patch]
  __shared__ bf16_t lut[256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l31 = lane & 31, lh = lane >> 5;
  const int PPD = Himg / 16, G16 = (PPD + 15) / 16, NP = PPD * PPD;
  for (int i = threadIdx.x; i < 16 * SCW_XE * 16; i += 256) pixT[i] = 0;  // pads stay zero
  lut[threadIdx.x] = f2bf(normalize_px((float)threadIdx.x, 1.f));
  floatx16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][nb][r] = 0.f;
  // this lane's k' column of each of its k-blocks: (ky, e) of k' = 32 kb + l31
  int kyo[4], eo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kp = 32 * (wave + 4 * i) + l31;
    kyo[i] = kp / 40;
    eo[i] = kp % 40;
  }
  // pixels (12 dwords per thread) and the pooled gradient / argmax of the tile (4 (patch,
  // channel) pairs per thread) loaded into registers one tile ahead
  uint32_t px[STEM_PXW];
  float dq[4];
  int aq[4];
  auto fetch = [&](int64_t t) {
    const int64_t bi = t / (PPD * G16);
    const int rem = (int)(t - bi * PPD * G16), py = rem / G16, px0 = (rem - py * G16) * 16;
    const int np = min(16, PPD - px0), wpr = np * 12;
    const int64_t pbase = bi * NP + (int64_t)py * PPD + px0;
    const uint8_t* src = img + bi * s_img + ((int64_t)py * 16 * Himg + px0 * 16) * 3;
#pragma unroll
    for (int j = 0; j < STEM_PXW; ++j) {
      const int i = min((int)threadIdx.x + 256 * j, 16 * wpr - 1), y = i / wpr, xw = i - y * wpr;
      px[j] = *reinterpret_cast<const uint32_t*>(src + (int64_t)y * Himg * 3 + xw * 4);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = threadIdx.x + 256 * j, pl = i / 64, n = i - pl * 64;
      const int64_t e = (pbase + min(pl, np - 1)) * 64 + n;
      dq[j] = pl < np ? dpooled[e] : 0.f;
      aq[j] = pl < np ? (int)arg[e] : -1;
    }
  };
  if (blockIdx.x < n_tiles) fetch(blockIdx.x);
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int64_t bi = t / (PPD * G16);
    const int rem = (int)(t - bi * PPD * G16), py = rem / G16, px0 = (rem - py * G16) * 16;
    const int np = min(16, PPD - px0);
    __syncthreads();
    {
      const int wpr = np * 12;
#pragma unroll
      for (int j = 0; j < STEM_PXW; ++j) {
        const int i = threadIdx.x + 256 * j;
        if (i >= 16 * wpr) break;
        const int y = i / wpr, xw = i - y * wpr;
        const int byte0 = xw * 4, pl = byte0 / 48, off = byte0 - pl * 48;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          pixT[(y * SCW_XE + off + q) * 16 + pl] = lut[(px[j] >> (8 * q)) & 0xffu];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = threadIdx.x + 256 * j, pl = i / 64, n = i - pl * 64;
        const bf16_t db = f2bf(dq[j]);
#pragma unroll
        for (int s = 0; s < 9; ++s) gt[(s * 64 + n) * 16 + pl] = s == aq[j] ? db : (bf16_t)0;
      }
    }
    __syncthreads();
    if (t + gridDim.x < n_tiles) fetch(t + gridDim.x);
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const int oy = s / 3, ox = s % 3;
      bf16x8 af[2];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        af[nb] = *reinterpret_cast<const bf16x8*>(gt + (s * 64 + 32 * nb + l31) * 16 + 8 * lh);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (wave + 4 * i >= 15) continue;  // wave-uniform
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(
            pixT + ((oy * 2 + kyo[i]) * SCW_XE + ox * 6 + eo[i]) * 16 + 8 * lh);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[i][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[nb], bfr, acc[i][nb], 0, 0, 0);
      }
    }
  }
  float* out = slab + (int64_t)blockIdx.x * 64 * 432;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (wave + 4 * i >= 15 || eo[i] >= 36) continue;
    const int k = kyo[i] * 36 + eo[i];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = 32 * nb + (r & 3) + 8 * (r >> 2) + 4 * lh;
        out[n * 432 + k] = acc[i][nb][r];
      }
  }
}

// max over the `win` conv positions of each patch (3x3 window on a 3x3 map -> 1x1), per channel.
__global__ void maxpool_patch_kernel(const float* __restrict__ conv, int64_t npatch, int win,
                                     int C, float* __restrict__ pooled, uint8_t* __restrict__ arg) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= npatch * C) return;
  const int64_t p = idx / C;
  const int c = idx % C;
  const float* src = conv + p * win * C + c;
  float best = src[0];
  int bi = 0;
  for (int s = 1; s < win; ++s) {
    const float v = src[(int64_t)s * C];
    if (v > best) {  // first maximum wins (lax.reduce_window max: gradient to one input)
      best = v;
      bi = s;
    }
  }
  pooled[idx] = best;
  arg[idx] = (uint8_t)bi;
}

// G[p, s, c] = dpooled[p, c] if s == argmax(p, c) else 0 (bf16) -> dW_conv = G^T . im2col
__global__ void maxpool_patch_bwd_kernel(const float* __restrict__ dpooled,
                                         const uint8_t* __restrict__ arg, int64_t npatch, int win,
                                         int C, bf16_t* __restrict__ G) {
  // one thread per (patch, window slot, 8 channels): one 16-B store of G
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c8 = C / 8;
  if (idx >= npatch * win * c8) return;
  const int c = (int)(idx % c8) * 8;
  const int s = (int)((idx / c8) % win);
  const int64_t p = idx / ((int64_t)c8 * win);
  const uint2 a = *reinterpret_cast<const uint2*>(arg + p * C + c);
  const float4 d0 = *reinterpret_cast<const float4*>(dpooled + p * C + c);
  const float4 d1 = *reinterpret_cast<const float4*>(dpooled + p * C + c + 4);
  const float d[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t lo = ((q < 2 ? a.x : a.y) >> (16 * (q & 1))) & 0xffu;
    const uint32_t hi = ((q < 2 ? a.x : a.y) >> (16 * (q & 1) + 8)) & 0xffu;
    const uint32_t vlo = lo == (uint32_t)s ? (uint32_t)f2bf(d[2 * q]) : 0u;
    const uint32_t vhi = hi == (uint32_t)s ? (uint32_t)f2bf(d[2 * q + 1]) : 0u;
    w[q] = vlo | (vhi << 16);
  }
  *reinterpret_cast<uint4*>(G + (p * win + s) * C + c) = make_uint4(w[0], w[1], w[2], w[3]);
}

// ---- general stem maps (patch sizes whose pooled map is larger than 1 x 1, e.g. the reference's
// own patch 56: 23 x 23 conv map -> 21 x 21 pooled map, gato_resnet.yaml:45-92)
// max_pool KP x KP, stride 1, VALID over (npatch, OH, OW, C) fp32 -> (npatch, PH, PW, C), with the
// window slot of the first maximum (lax.reduce_window max routes the gradient to one input).
__global__ void maxpool2d_kernel(const float* __restrict__ x, int64_t npatch, int OH, int OW, int C,
                                 int KP, float* __restrict__ y, uint8_t* __restrict__ arg) {
  const int PH = OH - KP + 1, PW = OW - KP + 1;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= npatch * PH * PW * C) return;
  const int c = idx % C;
  const int64_t o = idx / C;
  const int px = o % PW, py = (o / PW) % PH;
  const int64_t p = o / ((int64_t)PW * PH);
  const float* src = x + ((p * OH + py) * OW + px) * C + c;
  float best = src[0];
  int bi = 0;
  for (int dy = 0; dy < KP; ++dy)
    for (int dx = 0; dx < KP; ++dx) {
      const float v = src[((int64_t)dy * OW + dx) * C];
      if (v > best) {
        best = v;
        bi = dy * KP + dx;
      }
    }
  y[idx] = best;
  arg[idx] = (uint8_t)bi;
}

// G[p, y, x, c] = sum of dpooled[p, py, px, c] over the windows (py, px) whose first maximum is
// (y, x) (gather form, windows in raster order: deterministic), bf16 — the operand of dW_conv.
__global__ void maxpool2d_bwd_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ arg,
                                     int64_t npatch, int OH, int OW, int C, int KP,
                                     bf16_t* __restrict__ G) {
  const int PH = OH - KP + 1, PW = OW - KP + 1;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= npatch * OH * OW * C) return;
  const int c = idx % C;
  const int64_t o = idx / C;
  const int x = o % OW, yy = (o / OW) % OH;
  const int64_t p = o / ((int64_t)OW * OH);
  float acc = 0.f;
  for (int py = max(0, yy - KP + 1); py <= min(yy, PH - 1); ++py)
    for (int px = max(0, x - KP + 1); px <= min(x, PW - 1); ++px) {
      const int64_t q = ((p * PH + py) * PW + px) * C + c;
      if (arg[q] == (uint8_t)((yy - py) * KP + (x - px))) acc += dy[q];
    }
  G[idx] = f2bf(acc);
}

// im2col of a KS x KS stride-1 SAME convolution (zero padding KS/2) over (npatch, H, W, C) bf16:
// cols[(p, y, x)][(ky, kx, c)] = X[p, y + ky - KS/2, x + kx - KS/2, c] (Flax HWIO order), one
// thread per 8-channel chunk (C % 8 == 0).
__global__ void im2col_same_kernel(const bf16_t* __restrict__ X, int64_t npatch, int H, int W, int C,
                                   int KS, bf16_t* __restrict__ cols) {
  const int c8 = C / 8, K = KS * KS * C;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= npatch * H * W * KS * KS * c8) return;
  const int ch = idx % c8;
  const int tap = (idx / c8) % (KS * KS);
  const int64_t row = idx / ((int64_t)c8 * KS * KS);
  const int x = row % W, y = (row / W) % H;
  const int64_t p = row / ((int64_t)W * H);
  const int yy = y + tap / KS - KS / 2, xx = x + tap % KS - KS / 2;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (yy >= 0 && yy < H && xx >= 0 && xx < W)
    v = *reinterpret_cast<const uint4*>(X + ((p * H + yy) * W + xx) * C + ch * 8);
  *reinterpret_cast<uint4*>(cols + row * K + tap * C + ch * 8) = v;
}

// col2im (gather): dX[p, y, x, c] = sum over taps of dcols[(p, y - ky + KS/2, x - kx + KS/2)]
// [(ky, kx, c)] in tap order, fp32.
__global__ void col2im_same_kernel(const float* __restrict__ dcols, int64_t npatch, int H, int W, int C,
                                   int KS, float* __restrict__ dX) {
  const int K = KS * KS * C;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= npatch * H * W * C) return;
  const int c = idx % C;
  const int64_t o = idx / C;
  const int x = o % W, y = (o / W) % H;
  const int64_t p = o / ((int64_t)W * H);
  float acc = 0.f;
  for (int ky = 0; ky < KS; ++ky) {
    const int sy = y - ky + KS / 2;
    if (sy < 0 || sy >= H) continue;
    for (int kx = 0; kx < KS; ++kx) {
      const int sx = x - kx + KS / 2;
      if (sx < 0 || sx >= W) continue;
      acc += dcols[((p * H + sy) * W + sx) * K + (ky * KS + kx) * C + c];
    }
  }
  dX[idx] = acc;
}

__device__ __forceinline__ float gelu_tanh(float z) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * z * (1.f + tanhf(k0 * (z + k1 * z * z * z)));
}
__device__ __forceinline__ float gelu_tanh_grad(float z) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (z + k1 * z * z * z);
  const float th = tanhf(u);
  return 0.5f * (1.f + th) + 0.5f * z * (1.f - th * th) * k0 * (1.f + 3.f * k1 * z * z);
}

// GroupNorm + gelu forward over x (B, R, C) bf16: one workgroup per sample; stats per group of
// C/G adjacent channels over all R rows. y = gelu((x - mu) * rstd * gamma + beta).
constexpr int GN_NT = 256;
__global__ __launch_bounds__(GN_NT) void groupnorm_gelu_fwd_kernel(
    const float* __restrict__ x, int R, int C, int G, float eps, const float* __restrict__ gamma,
    const float* __restrict__ beta, bf16_t* __restrict__ y, float* __restrict__ mean,
    float* __restrict__ rstd) {
  extern __shared__ float sh[];  // [2][GN_NT/64 waves][C] partials, then mu/rs per group
  const int b = blockIdx.x;
  const float* xb = x + (int64_t)b * R * C;
  const int c = threadIdx.x % C;             // C divides GN_NT
  const int rstep = GN_NT / C;
  float s1 = 0.f, s2 = 0.f;
  for (int r = threadIdx.x / C; r < R; r += rstep) {
    const float v = xb[(int64_t)r * C + c];
    s1 += v;
    s2 += v * v;
  }
  float* p1 = sh;
  float* p2 = sh + GN_NT;
  p1[threadIdx.x] = s1;
  p2[threadIdx.x] = s2;
  __syncthreads();
  float* gmu = sh + 2 * GN_NT;
  float* grs = gmu + G;
  if (threadIdx.x < G) {
    const int cpg = C / G;
    float a = 0.f, q = 0.f;
    for (int t = 0; t < rstep; ++t)
      for (int j = 0; j < cpg; ++j) {
        a += p1[t * C + threadIdx.x * cpg + j];
        q += p2[t * C + threadIdx.x * cpg + j];
      }
    const float n = (float)R * cpg;
    const float mu = a / n;
    const float var = fmaxf(0.f, q / n - mu * mu);
    gmu[threadIdx.x] = mu;
    grs[threadIdx.x] = rsqrtf(var + eps);
    mean[b * G + threadIdx.x] = mu;
    rstd[b * G + threadIdx.x] = grs[threadIdx.x];
  }
  __syncthreads();
  const int g = c / (C / G);
  const float mu = gmu[g], rs = grs[g], ga = gamma[c], be = beta[c];
  bf16_t* yb = y + (int64_t)b * R * C;
  for (int r = threadIdx.x / C; r < R; r += rstep) {
    const float v = xb[(int64_t)r * C + c];
    yb[(int64_t)r * C + c] = f2bf(gelu_tanh((v - mu) * rs * ga + be));
  }
}

// Backward: dz = dy * gelu'(z); dxhat = dz * gamma; dx = rstd*(dxhat - mean(dxhat) -
// xhat*mean(dxhat*xhat)) over the group; dgamma += sum dz*xhat; dbeta += sum dz. dx is ADDED
// to `dx_accum` when accumulate != 0 (the residual branch of the stem).
__global__ __launch_bounds__(GN_NT) void groupnorm_gelu_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int R, int C, int G,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* dx, int accumulate,
    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  extern __shared__ float sh[];
  const int b = blockIdx.x;
  const float* xb = x + (int64_t)b * R * C;
  const float* db = dy + (int64_t)b * R * C;
  const int c = threadIdx.x % C;
  const int rstep = GN_NT / C;
  const int g = c / (C / G);
  const float mu = mean[b * G + g], rs = rstd[b * G + g], ga = gamma[c], be = beta[c];
  float a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;  // sum dxhat, sum dxhat*xhat, sum dz*xhat, sum dz
  for (int r = threadIdx.x / C; r < R; r += rstep) {
    const float xh = (xb[(int64_t)r * C + c] - mu) * rs;
    const float dz = db[(int64_t)r * C + c] * gelu_tanh_grad(xh * ga + be);
    const float dxh = dz * ga;
    a1 += dxh;
    a2 += dxh * xh;
    a3 += dz * xh;
    a4 += dz;
  }
  float* p = sh;  // [4][GN_NT]
  p[threadIdx.x] = a1;
  p[GN_NT + threadIdx.x] = a2;
  p[2 * GN_NT + threadIdx.x] = a3;
  p[3 * GN_NT + threadIdx.x] = a4;
  __syncthreads();
  float* gm1 = sh + 4 * GN_NT;
  float* gm2 = gm1 + G;
  const int cpg = C / G;
  if (threadIdx.x < G) {
    float s1 = 0.f, s2 = 0.f;
    for (int t = 0; t < rstep; ++t)
      for (int j = 0; j < cpg; ++j) {
        s1 += p[t * C + threadIdx.x * cpg + j];
        s2 += p[GN_NT + t * C + threadIdx.x * cpg + j];
      }
    const float n = (float)R * cpg;
    gm1[threadIdx.x] = s1 / n;
    gm2[threadIdx.x] = s2 / n;
  }
  if (threadIdx.x < C) {
    float s3 = 0.f, s4 = 0.f;
    for (int t = 0; t < rstep; ++t) {
      s3 += p[2 * GN_NT + t * C + threadIdx.x];
      s4 += p[3 * GN_NT + t * C + threadIdx.x];
    }
    grad_add(dgamma + threadIdx.x, s3);
    grad_add(dbeta + threadIdx.x, s4);
  }
  __syncthreads();
  const float m1 = gm1[g], m2 = gm2[g];
  float* dxb = dx + (int64_t)b * R * C;
  for (int r = threadIdx.x / C; r < R; r += rstep) {
    const int64_t o = (int64_t)r * C + c;
    const float xh = (xb[o] - mu) * rs;
    const float dz = db[o] * gelu_tanh_grad(xh * ga + be);
    float v = rs * (dz * ga - m1 - xh * m2);
    if (accumulate) v += dxb[o];
    dxb[o] = v;
  }
}

// Register-resident variants (R*C == NV * GN_NT * 4, C a power of two <= 256): every thread
// keeps its NV float4 of the sample in registers, so x (and dy) are read once with all loads in
// flight, and each thread owns one fixed channel quad c0..c0+3 ((4 t) % C): the per-channel sums
// reduce across the lanes sharing it with xor shuffles, then across the 4 waves in LDS.
template <int NV>
__global__ __launch_bounds__(GN_NT) void groupnorm_gelu_fwd_reg_kernel(
    const float* __restrict__ x, int R, int C, int G, float eps, const float* __restrict__ gamma,
    const float* __restrict__ beta, bf16_t* __restrict__ y, float* __restrict__ mean,
    float* __restrict__ rstd) {
  __shared__ float red[2][GN_NT / 64][256];
  __shared__ float gst[2][256];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const float4* xb = reinterpret_cast<const float4*>(x + (int64_t)b * R * C);
  float4 v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = xb[t + k * GN_NT];
  const int c0 = (4 * t) % C, cpg = C / G;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const float e4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s1[e] += e4[e];
      s2[e] = fmaf(e4[e], e4[e], s2[e]);
    }
  }
  for (int o = C / 4; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s1[e] += __shfl_xor(s1[e], o, 64);
      s2[e] += __shfl_xor(s2[e], o, 64);
    }
  if (lane < C / 4)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[0][wave][c0 + e] = s1[e];
      red[1][wave][c0 + e] = s2[e];
    }
  __syncthreads();
  if (t < G) {
    float a = 0.f, q = 0.f;
    for (int w = 0; w < GN_NT / 64; ++w)
      for (int j = 0; j < cpg; ++j) {
        a += red[0][w][t * cpg + j];
        q += red[1][w][t * cpg + j];
      }
    const float n = (float)R * cpg;
    const float mu = a / n;
    const float rs = rsqrtf(fmaxf(0.f, q / n - mu * mu) + eps);
    gst[0][t] = mu;
    gst[1][t] = rs;
    mean[b * G + t] = mu;
    rstd[b * G + t] = rs;
  }
  __syncthreads();
  float mu[4], rs[4], ga[4], be[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int g = (c0 + e) / cpg;
    mu[e] = gst[0][g];
    rs[e] = gst[1][g];
    ga[e] = gamma[c0 + e];
    be[e] = beta[c0 + e];
  }
  uint2* yb = reinterpret_cast<uint2*>(y + (int64_t)b * R * C);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const float e4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = gelu_tanh((e4[e] - mu[e]) * rs[e] * ga[e] + be[e]);
    yb[t + k * GN_NT] = make_uint2((uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16),
                                   (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16));
  }
}

template <int NV>
__global__ __launch_bounds__(GN_NT) void groupnorm_gelu_bwd_reg_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int R, int C, int G,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* dx, int accumulate,
    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[4][GN_NT / 64][256];
  __shared__ float gm[2][256];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const float4* xb = reinterpret_cast<const float4*>(x + (int64_t)b * R * C);
  const float4* db = reinterpret_cast<const float4*>(dy + (int64_t)b * R * C);
  float4 xv[NV], dv[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    xv[k] = xb[t + k * GN_NT];
    dv[k] = db[t + k * GN_NT];
  }
  const int c0 = (4 * t) % C, cpg = C / G;
  float mu[4], rs[4], ga[4], be[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int g = (c0 + e) / cpg;
    mu[e] = mean[b * G + g];
    rs[e] = rstd[b * G + g];
    ga[e] = gamma[c0 + e];
    be[e] = beta[c0 + e];
  }
  float a[4][4] = {};  // [sum dxhat, sum dxhat*xhat, sum dz*xhat, sum dz][channel]
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float* xe = reinterpret_cast<float*>(&xv[k]);
    float* de = reinterpret_cast<float*>(&dv[k]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (xe[e] - mu[e]) * rs[e];
      const float dz = de[e] * gelu_tanh_grad(xh * ga[e] + be[e]);
      xe[e] = xh;  // keep xhat and dz for the final pass
      de[e] = dz;
      a[0][e] += dz * ga[e];
      a[1][e] = fmaf(dz * ga[e], xh, a[1][e]);
      a[2][e] = fmaf(dz, xh, a[2][e]);
      a[3][e] += dz;
    }
  }
  for (int o = C / 4; o < 64; o <<= 1)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) a[i][e] += __shfl_xor(a[i][e], o, 64);
  if (lane < C / 4)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[i][wave][c0 + e] = a[i][e];
  __syncthreads();
  if (t < G) {
    float s1 = 0.f, s2 = 0.f;
    for (int w = 0; w < GN_NT / 64; ++w)
      for (int j = 0; j < cpg; ++j) {
        s1 += red[0][w][t * cpg + j];
        s2 += red[1][w][t * cpg + j];
      }
    const float n = (float)R * cpg;
    gm[0][t] = s1 / n;
    gm[1][t] = s2 / n;
  }
  if (t < C) {
    float s3 = 0.f, s4 = 0.f;
    for (int w = 0; w < GN_NT / 64; ++w) {
      s3 += red[2][w][t];
      s4 += red[3][w][t];
    }
    grad_add(dgamma + t, s3);
    grad_add(dbeta + t, s4);
  }
  __syncthreads();
  float m1[4], m2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int g = (c0 + e) / cpg;
    m1[e] = gm[0][g];
    m2[e] = gm[1][g];
  }
  float4* dxb = reinterpret_cast<float4*>(dx + (int64_t)b * R * C);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const float* xe = reinterpret_cast<const float*>(&xv[k]);
    const float* de = reinterpret_cast<const float*>(&dv[k]);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = rs[e] * (de[e] * ga[e] - m1[e] - xe[e] * m2[e]);
    float4 r = make_float4(o[0], o[1], o[2], o[3]);
    if (accumulate) {
      const float4 p = dxb[t + k * GN_NT];
      r.x += p.x; r.y += p.y; r.z += p.z; r.w += p.w;
    }
    dxb[t + k * GN_NT] = r;
  }
}

// NV of the register-resident kernels for this (R, C), or 0 (general kernel).
inline int gn_reg_nv(int R, int C) {
  if (C < 4 || C > 256 || (C & (C - 1)) || (int64_t)R * C % (GN_NT * 4)) return 0;
  const int64_t nv = (int64_t)R * C / (GN_NT * 4);
  return (nv == 4 || nv == 8 || nv == 16 || nv == 32) ? (int)nv : 0;
}

// encode_patch_position (image_tokenizer.py:74-132) for every (b, i, p):
// interval [k*P, (k+1)*P) -> floor(idx / Himg * (Q - 1)) in fp32; "row" token from interval
// p % PPD, "col" from p // PPD (the reference's transposed convention, :91-92, pinned by
// tests/test_image_tokenizer.py:53). train: uniform integer in [start, stop) (randint; stop <=
// start -> start), eval: (start + stop) // 2.
__global__ void patch_positions_kernel(const uint32_t* __restrict__ rng, uint32_t site, int B,
                                       int I, int Himg, int P, int Q, int train,
                                       int64_t sample_offset, int32_t* __restrict__ row_tok,
                                       int32_t* __restrict__ col_tok) {
  const int PPD = Himg / P, NP = PPD * PPD;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * I * NP) return;
  const int p = idx % NP;
  const int64_t bi = idx / NP;
  auto q = [&](int v) { return (int)floorf(((float)v / (float)Himg) * (float)(Q - 1)); };
  const int ri = p % PPD, ci = p / PPD;
  const int rs = q(ri * P), re = q((ri + 1) * P), cs = q(ci * P), ce = q((ci + 1) * P);
  int rt, ct;
  if (train) {
    const uint32_t key = stream_key(rng[0], rng[1], 0xFFFFu, site);
    const uint64_t g = (uint64_t)(sample_offset * I) * NP + idx;  // global (sample, image, patch)
    const uint32_t u1 = draw_u32(key, (uint32_t)(2 * g)), u2 = draw_u32(key, (uint32_t)(2 * g + 1));
    rt = re > rs ? rs + (int)(((uint64_t)u1 * (uint32_t)(re - rs)) >> 32) : rs;
    ct = ce > cs ? cs + (int)(((uint64_t)u2 * (uint32_t)(ce - cs)) >> 32) : cs;
  } else {
    rt = (rs + re) / 2;
    ct = (cs + ce) / 2;
  }
  row_tok[idx] = rt;
  col_tok[idx] = ct;
}

}  // namespace

extern "C" int mmt_patch_im2col(const void* img, int in_dtype, int B, int I, int Himg, int C,
                                int P, int KH, int KW, int S, int normalize, void* out,
                                mmt_stream_t stream) {
  MMT_CHECK_ARG(img && out && B > 0 && I > 0 && Himg > 0 && C > 0 && P > 0, "mmt_patch_im2col: args");
  MMT_CHECK_ARG(Himg % P == 0, "mmt_patch_im2col: image %d not divisible by patch %d (the "
                "reference's resize branch image_tokenizer.py:54-59 is broken; rejected)", Himg, P);
  MMT_CHECK_ARG(KH <= P && KW <= P && S > 0, "mmt_patch_im2col: kernel larger than patch");
  const int OH = (P - KH) / S + 1, OW = (P - KW) / S + 1;
  const int K = KH * KW * C;
  MMT_CHECK_ARG(K % 8 == 0, "mmt_patch_im2col: KH*KW*C must be a multiple of 8");
  const int NP = (Himg / P) * (Himg / P);
  const int64_t rows = (int64_t)B * I * NP * OH * OW;
  const int64_t n = rows * (K / 8);
  const float sc = normalize ? 1.f : 0.f, bi = 0.f;  // sc: the normalize flag of normalize_px
  const int64_t s_img = (int64_t)Himg * Himg * C;
  MMT_CHECK_ARG(in_dtype == 2 || in_dtype == MMT_F32, "mmt_patch_im2col: dtype must be fp32 (0) or uint8 (2)");
  if (KW * C == 36 && in_dtype == 2 && (P * C) % 4 == 0 && P * P * C * 2 * 8 <= 65536) {
    // the 12x12 RGB stem conv (gato_resnet.yaml:45-60) on uint8 images: LDS-staged kernel
    const int64_t npatch = (int64_t)B * I * NP;
    constexpr int PG = 8;
    hipLaunchKernelGGL((patch_im2col_lds_kernel<36, PG>), dim3((npatch + PG - 1) / PG), dim3(256),
                       (size_t)PG * P * P * C * 2, as_stream(stream), (const uint8_t*)img, s_img,
                       Himg, C, P, KH, S, OH, OW, npatch, K, (bf16_t*)out, sc);
  } else if (KW * C == 36) {  // row-segment kernel (fp32 images)
    const int64_t nr = rows * KH;
    if (in_dtype == 2)
      hipLaunchKernelGGL((patch_im2col_rows_kernel<uint8_t, 36>), dim3((nr + 255) / 256), dim3(256),
                         0, as_stream(stream), (const uint8_t*)img, s_img, Himg, C, P, KH, S, OH,
                         OW, rows, K, (bf16_t*)out, sc, bi);
    else
      hipLaunchKernelGGL((patch_im2col_rows_kernel<float, 36>), dim3((nr + 255) / 256), dim3(256),
                         0, as_stream(stream), (const float*)img, s_img, Himg, C, P, KH, S, OH, OW,
                         rows, K, (bf16_t*)out, sc, bi);
  } else if (in_dtype == 2)  // uint8
    hipLaunchKernelGGL(patch_im2col_kernel<uint8_t>, dim3((n + 255) / 256), dim3(256), 0,
                       as_stream(stream), (const uint8_t*)img, s_img, Himg, C, P, KH, KW, S, OH,
                       OW, rows, K, (bf16_t*)out, sc, bi);
  else if (in_dtype == MMT_F32)
    hipLaunchKernelGGL(patch_im2col_kernel<float>, dim3((n + 255) / 256), dim3(256), 0,
                       as_stream(stream), (const float*)img, s_img, Himg, C, P, KH, KW, S, OH, OW,
                       rows, K, (bf16_t*)out, sc, bi);
  else
    MMT_CHECK_ARG(false, "mmt_patch_im2col: dtype must be fp32 (0) or uint8 (2)");
  MMT_CHECK_LAUNCH("mmt_patch_im2col");
  return MMT_OK;
}

extern "C" int mmt_stem_conv_pool(const void* img, int B, int I, int Himg, const void* w,
                                  const float* bias, float* pooled, uint8_t* argmax,
                                  mmt_stream_t stream) {
  MMT_CHECK_ARG(img && w && bias && pooled && argmax && B > 0 && I > 0 && Himg >= 16 &&
                    Himg % 16 == 0, "mmt_stem_conv_pool: args");
  const int PPD = Himg / 16;
  const int64_t n_tiles = (int64_t)B * I * PPD * ((PPD + 15) / 16);
  const int grid = (int)std::min<int64_t>(n_tiles, 2 * 256);
  hipLaunchKernelGGL(stem_conv_pool_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                     (const uint8_t*)img, (int64_t)Himg * Himg * 3, Himg, n_tiles,
                     (const bf16_t*)w, bias, pooled, argmax);
  MMT_CHECK_LAUNCH("mmt_stem_conv_pool");
  return MMT_OK;
}

extern "C" int mmt_stem_conv_wgrad_slabs(int B, int I, int Himg) {
  if (B <= 0 || I <= 0 || Himg < 16 || Himg % 16) return 0;
  const int PPD = Himg / 16;
  // two workgroups per CU (the kernel's launch bound): one per CU left the tile loop's
  // fetch / LDS staging / MFMA phases unoverlapped (one wave per SIMD)
  return (int)std::min<int64_t>((int64_t)B * I * PPD * ((PPD + 15) / 16), 2 * 256);
}

extern "C" int mmt_stem_conv_wgrad(const void* img, int B, int I, int Himg, const float* dpooled,
                                   const uint8_t* argmax, float* slab, int64_t slab_elems,
                                   mmt_stream_t stream) {
  const int grid = mmt_stem_conv_wgrad_slabs(B, I, Himg);
  MMT_CHECK_ARG(img && dpooled && argmax && slab && grid > 0 && slab_elems >= (int64_t)grid * 64 * 432,
                "mmt_stem_conv_wgrad: args (slab of mmt_stem_conv_wgrad_slabs x 64 x 432 floats)");
  const int PPD = Himg / 16;
  const int64_t n_tiles = (int64_t)B * I * PPD * ((PPD + 15) / 16);
  hipLaunchKernelGGL(stem_conv_wgrad_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                     (const uint8_t*)img, (int64_t)Himg * Himg * 3, Himg, n_tiles, dpooled, argmax,
                     slab);
  MMT_CHECK_LAUNCH("mmt_stem_conv_wgrad");
  return MMT_OK;
}

extern "C" int mmt_maxpool_patch(const void* conv, int64_t npatch, int win, int C, void* pooled,
                                 uint8_t* argmax, mmt_stream_t stream) {
  MMT_CHECK_ARG(conv && pooled && argmax && npatch > 0 && win > 0 && win <= 255 && C > 0,
                "mmt_maxpool_patch: args");
  const int64_t n = npatch * C;
  hipLaunchKernelGGL(maxpool_patch_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     (const float*)conv, npatch, win, C, (float*)pooled, argmax);
  MMT_CHECK_LAUNCH("mmt_maxpool_patch");
  return MMT_OK;
}

extern "C" int mmt_maxpool_patch_bwd(const void* dpooled, const uint8_t* argmax, int64_t npatch,
                                     int win, int C, void* G, mmt_stream_t stream) {
  MMT_CHECK_ARG(dpooled && argmax && G && npatch > 0 && win > 0 && C > 0 && C % 8 == 0,
                "mmt_maxpool_patch_bwd: args (C %% 8 == 0)");
  const int64_t n = npatch * win * (C / 8);
  hipLaunchKernelGGL(maxpool_patch_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     as_stream(stream), (const float*)dpooled, argmax, npatch, win, C, (bf16_t*)G);
  MMT_CHECK_LAUNCH("mmt_maxpool_patch_bwd");
  return MMT_OK;
}

extern "C" int mmt_groupnorm_gelu_fwd(const void* x, int B, int R, int C, int G, float eps,
                                      const float* gamma, const float* beta, void* y, float* mean,
                                      float* rstd, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && y && gamma && beta && mean && rstd && B > 0 && R > 0,
                "mmt_groupnorm_gelu_fwd: args");
  MMT_CHECK_ARG(C > 0 && GN_NT % C == 0 && G > 0 && C % G == 0, "mmt_groupnorm_gelu_fwd: C=%d G=%d", C, G);
  const int nv = gn_reg_nv(R, C);
#define GN_FWD_REG(NV_)                                                                          \
  hipLaunchKernelGGL(groupnorm_gelu_fwd_reg_kernel<NV_>, dim3(B), dim3(GN_NT), 0, as_stream(stream), \
                     (const float*)x, R, C, G, eps, gamma, beta, (bf16_t*)y, mean, rstd)
  if (nv == 4) GN_FWD_REG(4);
  else if (nv == 8) GN_FWD_REG(8);
  else if (nv == 16) GN_FWD_REG(16);
  else if (nv == 32) GN_FWD_REG(32);
  else {
    const size_t sh = sizeof(float) * (2 * GN_NT + 2 * G);
    hipLaunchKernelGGL(groupnorm_gelu_fwd_kernel, dim3(B), dim3(GN_NT), sh, as_stream(stream),
                       (const float*)x, R, C, G, eps, gamma, beta, (bf16_t*)y, mean, rstd);
  }
#undef GN_FWD_REG
  MMT_CHECK_LAUNCH("mmt_groupnorm_gelu_fwd");
  return MMT_OK;
}

extern "C" int mmt_groupnorm_gelu_bwd(const void* dy, const void* x, int B, int R, int C, int G,
                                      const float* gamma, const float* beta, const float* mean,
                                      const float* rstd, void* dx, int accumulate, float* dgamma,
                                      float* dbeta, mmt_stream_t stream) {
  MMT_CHECK_ARG(dy && x && dx && gamma && beta && mean && rstd && dgamma && dbeta && B > 0,
                "mmt_groupnorm_gelu_bwd: args");
  MMT_CHECK_ARG(C > 0 && GN_NT % C == 0 && G > 0 && C % G == 0, "mmt_groupnorm_gelu_bwd: C/G");
  const int nv = gn_reg_nv(R, C);
#define GN_BWD_REG(NV_)                                                                          \
  hipLaunchKernelGGL(groupnorm_gelu_bwd_reg_kernel<NV_>, dim3(B), dim3(GN_NT), 0, as_stream(stream), \
                     (const float*)dy, (const float*)x, R, C, G, gamma, beta, mean, rstd,          \
                     (float*)dx, accumulate, dgamma, dbeta)
  if (nv == 4) GN_BWD_REG(4);
  else if (nv == 8) GN_BWD_REG(8);
  else if (nv == 16) GN_BWD_REG(16);
  else if (nv == 32) GN_BWD_REG(32);
  else {
    const size_t sh = sizeof(float) * (4 * GN_NT + 2 * G);
    hipLaunchKernelGGL(groupnorm_gelu_bwd_kernel, dim3(B), dim3(GN_NT), sh, as_stream(stream),
                       (const float*)dy, (const float*)x, R, C, G, gamma, beta, mean, rstd,
                       (float*)dx, accumulate, dgamma, dbeta);
  }
#undef GN_BWD_REG
  MMT_CHECK_LAUNCH("mmt_groupnorm_gelu_bwd");
  return MMT_OK;
}

extern "C" int mmt_patch_positions(const uint32_t* rng, uint32_t site, int B, int I, int Himg,
                                   int P, int Q, int train, int64_t sample_offset, int32_t* row_tok,
                                   int32_t* col_tok, mmt_stream_t stream) {
  MMT_CHECK_ARG(row_tok && col_tok && B > 0 && I > 0 && P > 0 && Himg % P == 0 && Q > 1,
                "mmt_patch_positions: args");
  MMT_CHECK_ARG(!train || rng, "mmt_patch_positions: train mode needs the rng state");
  const int NP = (Himg / P) * (Himg / P);
  const int64_t n = (int64_t)B * I * NP;
  hipLaunchKernelGGL(patch_positions_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     as_stream(stream), rng, site, B, I, Himg, P, Q, train, sample_offset, row_tok,
                     col_tok);
  MMT_CHECK_LAUNCH("mmt_patch_positions");
  return MMT_OK;
}

extern "C" int mmt_maxpool2d(const void* x, int64_t npatch, int OH, int OW, int C, int KP, void* y,
                             uint8_t* argmax, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && y && argmax && npatch > 0 && C > 0 && KP > 0 && KP * KP <= 255 && OH >= KP &&
                    OW >= KP, "mmt_maxpool2d: args");
  const int64_t n = npatch * (OH - KP + 1) * (OW - KP + 1) * C;
  hipLaunchKernelGGL(maxpool2d_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     (const float*)x, npatch, OH, OW, C, KP, (float*)y, argmax);
  MMT_CHECK_LAUNCH("mmt_maxpool2d");
  return MMT_OK;
}

extern "C" int mmt_maxpool2d_bwd(const void* dy, const uint8_t* argmax, int64_t npatch, int OH,
                                 int OW, int C, int KP, void* G, mmt_stream_t stream) {
  MMT_CHECK_ARG(dy && argmax && G && npatch > 0 && C > 0 && KP > 0 && OH >= KP && OW >= KP,
                "mmt_maxpool2d_bwd: args");
  const int64_t n = npatch * OH * OW * C;
  hipLaunchKernelGGL(maxpool2d_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     (const float*)dy, argmax, npatch, OH, OW, C, KP, (bf16_t*)G);
  MMT_CHECK_LAUNCH("mmt_maxpool2d_bwd");
  return MMT_OK;
}

extern "C" int mmt_im2col_same(const void* x, int64_t npatch, int H, int W, int C, int KS,
                               void* cols, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && cols && npatch > 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0 && KS > 0 &&
                    KS % 2 == 1, "mmt_im2col_same: args (C %% 8 == 0, odd KS)");
  const int64_t n = npatch * H * W * KS * KS * (C / 8);
  hipLaunchKernelGGL(im2col_same_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)x, npatch, H, W, C, KS, (bf16_t*)cols);
  MMT_CHECK_LAUNCH("mmt_im2col_same");
  return MMT_OK;
}

extern "C" int mmt_col2im_same(const float* dcols, int64_t npatch, int H, int W, int C, int KS,
                               float* dx, mmt_stream_t stream) {
  MMT_CHECK_ARG(dcols && dx && npatch > 0 && H > 0 && W > 0 && C > 0 && KS > 0 && KS % 2 == 1,
                "mmt_col2im_same: args");
  const int64_t n = npatch * H * W * C;
  hipLaunchKernelGGL(col2im_same_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     dcols, npatch, H, W, C, KS, dx);
  MMT_CHECK_LAUNCH("mmt_col2im_same");
  return MMT_OK;
}

namespace mmt {
int det_set_stem(const DetState& st) { return det_set_unit(st); }
}  // namespace mmt

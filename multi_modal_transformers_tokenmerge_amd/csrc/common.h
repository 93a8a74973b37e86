// Shared device/host helpers for libmmt_hip (gfx950 / CDNA4 only).
//
// Conventions of the C ABI (include/mmt_api.h):
//   * every tensor is a caller-owned device pointer; the library never allocates on the hot path;
//   * every entry point is stream-ordered and returns 0 (MMT_OK) or a negative code, never aborts;
//   * mmt_last_error() returns a thread-local message for the last failing call.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/mmt_api.h"

namespace mmt {

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);

// workspace sizes (bytes) behind mmt_workspace_size
int64_t tome_match_workspace(int64_t n, int64_t t, int64_t c);

#define MMT_CHECK_ARG(cond, ...)              \
  do {                                        \
    if (!(cond)) {                            \
      ::mmt::set_error(__VA_ARGS__);          \
      return MMT_ERR_INVALID;                 \
    }                                         \
  } while (0)

#define MMT_CHECK_LAUNCH(name)                                             \
  do {                                                                     \
    hipError_t e_ = hipGetLastError();                                     \
    if (e_ != hipSuccess) {                                                \
      ::mmt::set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
      return MMT_ERR_HIP;                                                  \
    }                                                                      \
  } while (0)

// ---------------------------------------------------------------- bf16
typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even; NaN stays NaN (the compiler emits v_cvt_pk_bf16_f32 for the cast).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T> __device__ __forceinline__ float ld_f32(const T* p);
template <> __device__ __forceinline__ float ld_f32<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld_f32<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> __device__ __forceinline__ void st_f32(T* p, float v);
template <> __device__ __forceinline__ void st_f32<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st_f32<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// ---------------------------------------------------------------- counter-based RNG
// lowbias32 (a bijective 32-bit mixer). The oracle (oracle/rng.py) restates it in numpy uint32
// arithmetic, so dropout masks / sampled tokens are bit-identical on both sides.
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// Key of one random stream: (seed, step, layer, site). Element draw = mix32(key ^ mix32(ctr)).
__host__ __device__ __forceinline__ uint32_t stream_key(uint32_t seed, uint32_t step, uint32_t layer,
                                                        uint32_t site) {
  uint32_t k = mix32(seed ^ 0x9e3779b9u);
  k = mix32(k ^ (step * 0x85ebca6bu));
  k = mix32(k ^ (layer * 0xc2b2ae35u) ^ (site << 24));
  return k;
}
__host__ __device__ __forceinline__ uint32_t draw_u32(uint32_t key, uint32_t ctr) {
  return mix32(key ^ mix32(ctr));
}
// keep-probability threshold: keep iff draw < thresh, thresh = floor(keep_prob * 2^32)
__host__ __device__ __forceinline__ bool keep_draw(uint32_t key, uint32_t ctr, uint32_t thresh) {
  return draw_u32(key, ctr) < thresh;
}

// thresh = min(2^32 - 1, floor(keep_prob * 2^32)), computed in double on the host
inline uint32_t keep_threshold(float keep_prob) {
  double t = (double)keep_prob * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
}

// Dropout keep decisions (every flax.linen.Dropout site of the path): element idx of a stream
// keeps iff the 16-bit half (idx & 1) of mix32(key ^ (idx >> 1)) is < thresh16 =
// floor(keep_prob * 65536). One mixer evaluation serves two elements (half the multiplies of
// draw_u32); keep probability is exact to 2^-16.
inline uint32_t keep_threshold16(float keep_prob) {
  double t = (double)keep_prob * 65536.0;
  return t >= 65536.0 ? 65536u : (uint32_t)t;
}
__host__ __device__ __forceinline__ uint32_t pair_draw(uint32_t key, uint32_t pair) {
  return mix32(key ^ pair);
}
__host__ __device__ __forceinline__ bool keep_elem(uint32_t key, uint32_t idx, uint32_t thresh16) {
  return ((pair_draw(key, idx >> 1) >> ((idx & 1u) << 4)) & 0xffffu) < thresh16;
}

// ---------------------------------------------------------------- sequence-LN launch grids
// The (sample, 64-column block) workgroups of the sequence-axis LayerNorm family: column blocks
// fastest (MMT_LN_COLFIRST = 1: the D / 64 workgroups of one sample run together and read its
// whole rows, one DRAM page run per token row) or samples fastest (0: a sample's column blocks run
// B workgroups apart, each reading a 256-B piece of every row).
#ifndef MMT_LN_COLFIRST
#define MMT_LN_COLFIRST 1
#endif
__device__ __forceinline__ int ln_sample() { return MMT_LN_COLFIRST ? blockIdx.y : blockIdx.x; }
__device__ __forceinline__ int ln_colblk() { return MMT_LN_COLFIRST ? blockIdx.x : blockIdx.y; }
inline dim3 ln_grid(int n, int cblocks) { return MMT_LN_COLFIRST ? dim3(cblocks, n) : dim3(n, cblocks); }

// ---------------------------------------------------------------- wave helpers (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// One 16-B-per-lane LDS-DMA piece (buffer_load_dwordx4 ... lds, 1 KB per wave-instruction) as
// inline asm: issued through the builtin, the compiler cannot tell LDS reads from the region
// being filled and puts a vmcnt(0) behind every DMA. Invisible to the compiler's vmcnt
// bookkeeping, so the caller waits for it explicitly (s_waitcnt vmcnt). Raw buffer resource:
// stride 0, num_records = bytes (reads past it return 0); lds = this lane group's destination
// base (lane-linear, 16 B per lane), voffset = the lane's source byte offset.
__device__ __forceinline__ void dma16_asm(const void* base, int64_t bytes, void* lds, int voffset) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const uint64_t b = (uint64_t)(uintptr_t)base;
  i32x4 r;
  // every operand but voffset is wave-uniform by contract: readfirstlane keeps it in SGPRs where
  // the compiler cannot prove the uniformity (free when it already can)
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(b >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)min(bytes, (int64_t)0x7ffffff0));
  r[3] = 0x00020000;
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)lds));
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voffset), "s"(r), "s"(l) : "m0", "memory");
}

// ---------------------------------------------------------------- deterministic mode
// mmt_set_deterministic (SURVEY §5 "deterministic-mode reruns"): every gradient accumulation that
// is otherwise an fp32 atomicAdd into the flat gradient buffer (bias / LayerNorm / GroupNorm /
// embedding / Fourier gradients: the per-workgroup partials of a column sum) becomes an integer
// add of round(v * 2^36) into a signed 64-bit fixed-point shadow of that buffer. Integer adds
// commute, so the sum no longer depends on the order in which workgroups arrive: the gradients
// of a step are bitwise reproducible. mmt_det_flush adds the shadow (x 2^-36) into the fp32
// buffer and clears it. Resolution 2^-36 (1.5e-11) per contribution, range |sum| < 2^27.
// Each translation unit holds its own copy of the state (static __constant__), set by its
// det_set_<unit> (core.hip's mmt_set_deterministic calls them all).
struct DetState {
  float* base;     // the fp32 gradient buffer whose additions go to fx (NULL: mode off)
  long long* fx;   // fixed-point shadow, same offsets as base
  int64_t n;       // elements
};
// Range: the shadow holds |sum| < 2^27 per element (int64 at 2^-36 resolution). A contribution
// enters it only if |v| < 2^15 (det_fits), so up to 2^12 = 4096 contributions per element and
// flush can never wrap the int64 (the step's busiest site, a column sum over B*L rows in
// 256-row partials, gives about 550 at B = 512). A contribution that is not finite or larger
// goes to the fp32 buffer as a plain fp32 atomic instead, so a NaN / Inf / huge gradient still
// reaches flat_grad (and survives the flush: NaN + x = NaN): the mode trades bitwise reruns
// for visibility there, never a silently wrapped sum.
constexpr double DET_SCALE = 68719476736.0;  // 2^36
constexpr float DET_VMAX = 32768.f;          // 2^15
static __constant__ DetState g_det;
static DetState g_det_host{};  // this unit's host copy (kernel-variant choices)

// false for NaN / Inf and for contributions too large for the shadow's range
__device__ __forceinline__ bool det_fits(float v) { return fabsf(v) < DET_VMAX; }
__device__ __forceinline__ long long det_fixed(float v) {  // callers check det_fits(v) first
  return __double2ll_rn((double)v * DET_SCALE);
}
// dst += v: an fp32 atomic, or in deterministic mode (dst inside the registered gradient buffer,
// v within det_fits) a 64-bit integer atomic on the fixed-point shadow
__device__ __forceinline__ void grad_add(float* dst, float v) {
  if (g_det.fx != nullptr) {
    const int64_t i = dst - g_det.base;
    if (i >= 0 && i < g_det.n && det_fits(v)) {
      atomicAdd(reinterpret_cast<unsigned long long*>(g_det.fx + i), (unsigned long long)det_fixed(v));
      return;
    }
  }
  atomicAdd(dst, v);
}
inline int det_set_unit(const DetState& st) {
  g_det_host = st;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_det), &st, sizeof st) == hipSuccess ? 0 : -1;
}
int det_set_attention(const DetState&);
int det_set_glue(const DetState&);
int det_set_norm(const DetState&);
int det_set_stem(const DetState&);

// XCD-aware bijective remap: workgroups b and b+8 share an XCD (round-robin dispatch), so give
// each XCD a contiguous range of work ids: items that share operands (a GEMM's A row panel, the
// key/query blocks of one attention (sample, head)) then meet in one L2. Speed only.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

inline hipStream_t as_stream(mmt_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- device-side index checks
// Kernels that address memory through caller-supplied index arrays (the ToMe merge maps, pos_map,
// the pruning row lists) range-check every index they use: an out-of-range value is replaced by 0
// (a valid row, so no access leaves its tensor) and its fault bit is OR-ed into the library's
// device status word, which mmt_device_status() reports as MMT_ERR_INVALID (include/mmt_api.h).
// The word lives in core.hip's code object; fault_word() is its device address (NULL before HIP
// is usable), passed to the kernels as an argument.
unsigned int* fault_word();
__device__ __forceinline__ int checked_index(int v, int hi, unsigned int* fault, unsigned int bit) {
  if ((unsigned)v < (unsigned)hi) return v;
  if (fault) atomicOr(fault, bit);
  return 0;
}
__device__ __forceinline__ void record_fault(unsigned int* fault, unsigned int bit) {
  if (fault) atomicOr(fault, bit);
}

}  // namespace mmt

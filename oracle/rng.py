"""ORACLE — test infrastructure only.

numpy uint32 restatement of the counter-based RNG of csrc/common.h (mix32 = lowbias32,
stream_key, draw_u32). The reference draws with JAX Threefry, which cannot be matched (SURVEY §7
"Hard parts"); parity runs therefore share THIS stream between the HIP path and the oracle, so
dropout keep-masks, sampled position tokens and diffusion (t, eps) are identical on both sides.
"""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def mix32(x):
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def stream_key(seed: int, step: int, layer: int, site: int) -> int:
    k = mix32(np.uint64(seed) ^ np.uint64(0x9E3779B9))
    k = mix32(k ^ ((np.uint64(step) * np.uint64(0x85EBCA6B)) & M32))
    k = mix32(k ^ ((np.uint64(layer) * np.uint64(0xC2B2AE35)) & M32) ^ ((np.uint64(site) << np.uint64(24)) & M32))
    return int(k)


def draw_u32(key: int, ctr):
    return mix32(np.uint64(key) ^ mix32(np.asarray(ctr, dtype=np.uint64) & M32))


def keep_thresh(keep_prob: float) -> int:
    t = float(np.float32(keep_prob)) * 4294967296.0
    return 0xFFFFFFFF if t >= 4294967295.0 else int(t)


def keep_thresh16(keep_prob: float) -> int:
    t = float(np.float32(keep_prob)) * 65536.0
    return 65536 if t >= 65536.0 else int(t)


def keep_mask(key: int, idx, keep_prob: float) -> np.ndarray:
    """csrc/common.h keep_elem: 16-bit half (idx & 1) of mix32(key ^ (idx >> 1)) < thresh16."""
    idx = np.asarray(idx, dtype=np.uint64) & M32
    d = mix32(np.uint64(key) ^ (idx >> np.uint64(1)))
    half = (d >> ((idx & np.uint64(1)) << np.uint64(4))) & np.uint64(0xFFFF)
    return half < np.uint64(keep_thresh16(keep_prob))


def dropout_mask_2d(seed, step, layer, site, rows: int, cols: int, row_offset: int, keep_prob: float):
    """Keep-mask of the GEMM-epilogue dropout: ctr = (row_offset + m) * cols + n."""
    m = np.arange(rows, dtype=np.uint64)[:, None] + np.uint64(row_offset)
    ctr = (m * np.uint64(cols) + np.arange(cols, dtype=np.uint64)[None, :]) & M32
    return keep_mask(stream_key(seed, step, layer, site), ctr, keep_prob)


def uniform01(key: int, ctr) -> np.ndarray:
    """float32 in [0, 1): top 24 bits of the draw."""
    return (draw_u32(key, ctr) >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def patch_positions(seed: int, step: int, site: int, B: int, I: int, himg: int, patch: int, Q: int,
                    sample_offset: int = 0, train: bool = True):
    """csrc/stem.hip patch_positions_kernel (reference image_tokenizer.py:74-132
    encode_patch_position): interval [i p, (i + 1) p) quantised as floor(v / H * (Q - 1)) in
    fp32 (:100), the "row" token from interval p % P and the "col" token from p // P (:91-92,
    the reference's transpose quirk), train: randint[start, stop) by the counter stream (seed,
    step, layer 0xFFFF, site) at counters 2 g, 2 g + 1 of the global (sample, image, patch) index
    g, as (u32 * (stop - start)) >> 32; eval: (start + stop) // 2. Returns (rt, ct) int32 (B, I NP)."""
    ppd = himg // patch
    NP = ppd * ppd
    idx = np.arange(B * I * NP, dtype=np.uint64)
    p = (idx % np.uint64(NP)).astype(np.int64)
    ri, ci = p % ppd, p // ppd

    def q(v):
        return np.floor((np.asarray(v, np.float32) / np.float32(himg)) * np.float32(Q - 1)).astype(np.int64)
    rs, re_, cs, ce = q(ri * patch), q((ri + 1) * patch), q(ci * patch), q((ci + 1) * patch)
    if train:
        key = stream_key(seed, step, 0xFFFF, site)
        g = np.uint64(sample_offset * I * NP) + idx
        u1 = draw_u32(key, (np.uint64(2) * g) & M32).astype(np.uint64)
        u2 = draw_u32(key, (np.uint64(2) * g + np.uint64(1)) & M32).astype(np.uint64)
        rt = np.where(re_ > rs, rs + ((u1 * (re_ - rs).astype(np.uint64)) >> np.uint64(32)).astype(np.int64), rs)
        ct = np.where(ce > cs, cs + ((u2 * (ce - cs).astype(np.uint64)) >> np.uint64(32)).astype(np.int64), cs)
    else:
        rt, ct = (rs + re_) // 2, (cs + ce) // 2
    return rt.astype(np.int32).reshape(B, I * NP), ct.astype(np.int32).reshape(B, I * NP)


def diffusion_t_eps(seed: int, step: int, B: int, A: int, steps: int, sample_offset: int = 0):
    """csrc/glue.hip diffusion_prep_kernel (reference diffusion.py:124-127): t ~ randint[0, steps)
    as (u32 * steps) >> 32 of the stream (seed, step, 0xFFFE, 1) at the global sample index;
    eps ~ N(0, 1) by Box-Muller, sqrt(-2 ln u1) cos(2 pi u2) in fp32, u1 = ((u >> 8) + 1) / 2^24
    in (0, 1], u2 = (u >> 8) / 2^24 from counters 2 c, 2 c + 1 of c = sample * A + j on the stream
    (seed, step, 0xFFFE, 2). eps agrees with the device's logf / cosf to a few ulp, not bitwise."""
    b = np.arange(B, dtype=np.uint64) + np.uint64(sample_offset)
    kt = stream_key(seed, step, 0xFFFE, 1)
    t = ((draw_u32(kt, b).astype(np.uint64) * np.uint64(steps)) >> np.uint64(32)).astype(np.int32)
    ke = stream_key(seed, step, 0xFFFE, 2)
    c = (b[:, None] * np.uint64(A) + np.arange(A, dtype=np.uint64)[None, :]) & M32
    d1 = draw_u32(ke, (np.uint64(2) * c) & M32)
    d2 = draw_u32(ke, (np.uint64(2) * c + np.uint64(1)) & M32)
    u1 = ((d1 >> np.uint64(8)) + np.uint64(1)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    u2 = (d2 >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    eps = np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.283185307179586) * u2)
    return t, eps.astype(np.float32)

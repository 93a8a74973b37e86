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

"""ORACLE — test infrastructure only (imported by tests/ and never by the package).

CPU restatement of the DDPM inference sampler, the reference's
``DiffusionActionHead.predict_action`` (multi_modal_transformers/action_heads/diffusion.py:146-209)
and the denoiser it scans (``OctoDenoise`` :53-65, ``FourierFeatures`` :30-51,
``predict_denoise_term`` :88-107):

  x_T = z ~ N(0, I)                                         (:198-200, one key per sample)
  for t = steps-1 .. 0:                                     (:203-207)
      eps_hat = denoiser(x_t, t, mean(readouts))            (:169-175)
      x_{t-1} = clip(1/sqrt(a_t) (x_t - (1-a_t)/sqrt(1-abar_t) eps_hat) + sqrt(b_t) z, -5, 5)
                                                            (:182-188)

Reference quirks kept on purpose: the per-sample keys are never split inside the scan (:178
reuses ``keys`` from the carry), so every step's noise equals the initial sample z; noise is
added at t = 0 as well.

Rounding model = the MI355X path's: the Fourier features, the time-MLP hidden layer, the time
embedding and the readout mean are bf16 (GEMM operands); the denoiser weights are the bf16
shadow. Everything else is float64 here (fp32 on the GPU).
"""
from __future__ import annotations

import numpy as np


def bf16(x) -> np.ndarray:
    """Round-to-nearest-even to bfloat16, returned as float64."""
    f = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    u = f.view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) << np.uint64(16)
    return r.astype(np.uint32).view(np.float32).astype(np.float64)


def sampler_coefficients(betas: np.ndarray, alpha_hats: np.ndarray) -> np.ndarray:
    """(steps, 3) rows [1/sqrt(a_t), (1-a_t)/sqrt(1-abar_t), sqrt(b_t)] (:182-184), float64."""
    b = np.asarray(betas, dtype=np.float64)
    a = 1.0 - b
    ah = np.asarray(alpha_hats, dtype=np.float64)
    return np.stack([1.0 / np.sqrt(a), (1.0 - a) / np.sqrt(1.0 - ah), np.sqrt(b)], axis=1)


def time_embedding(steps: int, fourier_w, w_t1, b_t1, w_t2, b_t2) -> np.ndarray:
    """FourierFeatures (:41-51) + its MLPBlock for t = 0..steps-1 -> (steps, T), bf16 values.
    fourier_w (F,); w_t1 / w_t2 (T, T) stored [out][in]."""
    t = np.arange(steps, dtype=np.float64)[:, None]
    h = 2.0 * np.pi * t * np.asarray(fourier_w, dtype=np.float64).reshape(1, -1)
    feats = bf16(np.concatenate([np.cos(h), np.sin(h)], axis=1))
    ht = bf16(np.maximum(feats @ bf16(w_t1).T + np.asarray(b_t1, np.float64), 0.0))
    return bf16(ht @ bf16(w_t2).T + np.asarray(b_t2, np.float64))


def predict_action(readout_mean, z, temb, w1, b1, w2, b2, coef, clip: float = 5.0,
                   stored_bf16: bool = False) -> np.ndarray:
    """readout_mean (B, D); z (B, A) initial sample; temb (steps, T); w1 (H, A+T+D) [out][in];
    b1 (H,); w2 (A, H); b2 (A,); coef (steps, 3). Returns the (B, A) actions (float64).
    stored_bf16: the noisy sample and the hidden layer rounded to bf16 where the per-step launch
    form (DiffusionActionHead._predict_action_loop: predict_denoise_term_mean per step) stores
    them; the fused one-launch sampler keeps both fp32 (False)."""
    z = np.asarray(z, dtype=np.float64)
    A = z.shape[1]
    temb = np.asarray(temb, dtype=np.float64)
    T = temb.shape[1]
    w1 = bf16(w1)
    w2 = bf16(w2)
    # concatenate([noisy, time_emb, readout]) . W1^T as three products (:61)
    P = bf16(readout_mean) @ w1[:, A + T:].T                          # (B, H)
    Q = temb @ w1[:, A:A + T].T + np.asarray(b1, np.float64)          # (steps, H)
    x = z.copy()
    for t in range(coef.shape[0] - 1, -1, -1):
        xin = bf16(x) if stored_bf16 else x
        h = np.maximum(xin @ w1[:, :A].T + Q[t][None, :] + P, 0.0)
        if stored_bf16:
            h = bf16(h)
        eps = h @ w2.T + np.asarray(b2, np.float64)
        c1, c2, c3 = (float(v) for v in coef[t])
        x = np.clip(c1 * (x - c2 * eps) + c3 * z, -clip, clip)
    return x

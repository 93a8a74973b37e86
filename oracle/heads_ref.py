"""ORACLE — test infrastructure only (imported by tests/, never by the package).

float64 restatement of the continuous and categorical action heads and their losses:
reference action_heads/continuous.py:19-26, action_heads/categorical.py:12-40 and
models/octo/octo.py:167-198 (compute_l2_loss / compute_ce_loss) with the train steps' means
(:262, :302). Returns the loss and its gradient w.r.t. the head's pre-activation z."""
from __future__ import annotations

import numpy as np


def continuous(z, actions, max_action):
    """z (B, A) Dense output. Returns (pred (B, 1, A), loss, dloss/dz)."""
    z = np.asarray(z, np.float64)
    t = np.tanh(z / max_action)
    p = t * max_action
    d = p - np.asarray(actions, np.float64)
    B = z.shape[0]
    loss = np.mean(np.sum(d * d, axis=-1))
    dz = 2.0 * d * (1.0 - t * t) / B
    return p[:, None, :], loss, dz


def digitize_bins(actions, max_action, num_bins):
    """assign_bins (categorical.py:12-22): jnp.digitize against float32 linspace edges."""
    edges = np.linspace(-max_action, max_action, num_bins + 1, dtype=np.float32)
    return np.digitize(np.asarray(actions, np.float32), edges)


def categorical(z, actions, max_action, num_bins):
    """z (B, A, num_bins) logits. Returns (loss, dloss/dz) with one_hot(bin, num_bins) labels
    (zero past the last class) and optax.softmax_cross_entropy, mean over (b, a)."""
    z = np.asarray(z, np.float64)
    bins = digitize_bins(actions, max_action, num_bins)
    lab = np.zeros_like(z)
    b_idx, a_idx = np.nonzero(bins < num_bins)
    lab[b_idx, a_idx, bins[b_idx, a_idx]] = 1.0
    m = z.max(axis=-1, keepdims=True)
    lse = m + np.log(np.exp(z - m).sum(axis=-1, keepdims=True))
    ce = -(lab * (z - lse)).sum(-1)
    n = ce.size
    sm = np.exp(z - lse)
    dz = (lab.sum(-1, keepdims=True) * sm - lab) / n
    return ce.mean(), dz

"""DDPM action head, mirroring the reference's ``multi_modal_transformers/action_heads/diffusion.py``:
``cosine_beta_schedule`` (:17-27), ``FourierFeatures`` (:30-51), ``OctoDenoise`` (:53-65) and
``DiffusionActionHead`` (:68-209: ``denoise_loss`` :110-143, ``predict_denoise_term`` :88-107,
``predict_action`` :146-209).

Training path on MI355X: one fused kernel draws (t, eps), noises the actions and emits the Fourier
features straight into the denoiser's concatenated input buffer; the time-encoder MLP writes its
output into that same buffer (GEMM with a column-offset output), the readout mean is written into
its last columns, so ``concatenate([noisy, time_emb, readout])`` (:61) never materialises
separately. MLPBlocks here run with dropout disabled, as in the reference (they are called without
``train``, attention.py:29 default False).
"""
from __future__ import annotations


import numpy as np
import torch

from .. import _C, _kernels as K
from ..layers import Dense
from ..params import ParamStore, he_normal


def cosine_beta_schedule(timesteps: int, s: float = 0.008) -> np.ndarray:
    """Reference :17-27 (float32 like jnp)."""
    steps = timesteps + 1
    t = (np.linspace(0, timesteps, steps, dtype=np.float32) / np.float32(timesteps)).astype(np.float32)
    ac = np.cos((t + np.float32(s)) / np.float32(1 + s) * np.float32(np.pi) * np.float32(0.5)) ** 2
    ac = (ac / ac[0]).astype(np.float32)
    betas = (1 - (ac[1:] / ac[:-1])).astype(np.float32)
    return np.clip(betas, 0, 0.999).astype(np.float32)


def alpha_hats_of(betas: np.ndarray) -> np.ndarray:
    """Reference :84-86: prod(alphas[:i+1]) for each i (float32)."""
    alphas = (1 - betas).astype(np.float32)
    return np.array([np.prod(alphas[: i + 1], dtype=np.float32) for i in range(len(betas))],
                    dtype=np.float32)


class DiffusionActionHead:
    def __init__(self, store: ParamStore, name: str, embedding_dim: int, action_dim: int = 8,
                 diffusion_steps: int = 32, time_dim: int | None = None, hidden: int | None = None):
        D = embedding_dim
        self.D, self.A, self.steps = D, action_dim, diffusion_steps
        self.F = (time_dim or D) // 2
        T = 2 * self.F
        self.time_dim = T
        self.hidden = hidden or D
        p = f"{name}/OctoDenoise_0"
        self.fourier = store.add(f"{p}/FourierFeatures_0/fourier_kernel", (self.F, 1),
                                 he_normal((self.F, 1)))
        self.t1 = Dense(store, f"{p}/FourierFeatures_0/MLPBlock_0/Dense_0", T, T)
        self.t2 = Dense(store, f"{p}/FourierFeatures_0/MLPBlock_0/Dense_1", T, T)
        self.cat_dim = action_dim + T + D
        self.d1 = Dense(store, f"{p}/MLPBlock_0/Dense_0", self.cat_dim, self.hidden)
        self.d2 = Dense(store, f"{p}/MLPBlock_0/Dense_1", self.hidden, action_dim)
        betas = cosine_beta_schedule(diffusion_steps)
        self.betas_np = betas
        self.alpha_hats_np = alpha_hats_of(betas)
        self._dev_consts = {}
        if self.cat_dim % 8:
            raise ValueError("action_dim + time_dim + D must be a multiple of 8 (16-B rows)")

    def consts(self, device):
        if device not in self._dev_consts:
            self._dev_consts[device] = torch.from_numpy(self.alpha_hats_np).to(device)
        return self._dev_consts[device]

    def new_cat(self, B, device):
        return torch.empty((B, self.cat_dim), dtype=torch.bfloat16, device=device)

    def readout_slot(self, cat: torch.Tensor) -> torch.Tensor:
        return cat[:, self.A + self.time_dim:]

    # ------------------------------------------------------------------------- denoise_loss
    def loss_forward(self, cat: torch.Tensor, actions: torch.Tensor, rng, sample_offset: int = 0,
                     t_in=None, eps_in=None):
        """cat: (B, A+T+D) bf16 whose readout slot is already filled. Returns (loss (1,) fp32,
        saved). Mirrors denoise_loss (:110-143)."""
        B = cat.shape[0]
        dev = cat.device
        t = torch.empty(B, dtype=torch.int32, device=dev)
        eps = torch.empty((B, self.A), dtype=torch.float32, device=dev)
        feats = torch.empty((B, self.time_dim), dtype=torch.bfloat16, device=dev)
        _C.call("mmt_diffusion_prep", _C.ptr(rng), B, self.A, self.steps, sample_offset,
                _C.ptr(actions), _C.ptr(self.consts(dev)), _C.ptr(self.fourier.data), self.F,
                _C.ptr(t_in), _C.ptr(eps_in), _C.ptr(t), _C.ptr(eps), _C.ptr(cat), cat.stride(0),
                _C.ptr(feats), _C.stream_ptr())
        ht = self.t1.fwd(feats, act=K.ACT_RELU)
        self.t2.fwd(ht, out=cat[:, self.A:self.A + self.time_dim])
        hd = self.d1.fwd(cat, act=K.ACT_RELU)
        pred = self.d2.fwd(hd, out_mode=K.OUT_F32)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        dpred = torch.empty((B, self.A), dtype=torch.bfloat16, device=dev)
        _C.call("mmt_diffusion_loss", _C.ptr(pred), pred.stride(0), _C.ptr(eps), B, self.A, 1.0,
                _C.ptr(loss), _C.ptr(dpred), _C.stream_ptr())
        return loss, dict(cat=cat, feats=feats, ht=ht, hd=hd, dpred=dpred, t=t, eps=eps, pred=pred)

    def loss_backward(self, sv: dict) -> torch.Tensor:
        """Returns d(readout mean) (B, D) bf16 view."""
        B = sv["cat"].shape[0]
        dzd = self.d2.bwd(sv["dpred"], sv["hd"], gate=sv["hd"], gate_scale=1.0)
        dcat = self.d1.bwd(dzd, sv["cat"])
        dtemb = dcat[:, self.A:self.A + self.time_dim]
        dzt = self.t2.bwd(dtemb, sv["ht"], gate=sv["ht"], gate_scale=1.0)
        dfeats = self.t1.bwd(dzt, sv["feats"])
        _C.call("mmt_fourier_bwd", _C.ptr(dfeats), B, self.F, _C.ptr(sv["t"]),
                _C.ptr(self.fourier.data), _C.ptr(self.fourier.grad), _C.stream_ptr())
        return dcat[:, self.A + self.time_dim:]

    # ------------------------------------------------------------------ predict_denoise_term
    def predict_denoise_term(self, readout_mean: torch.Tensor, time: torch.Tensor,
                             noisy_actions: torch.Tensor) -> torch.Tensor:
        """Reference :88-107 (``OctoDenoise(noisy, time, mean(readouts))``) for given integer
        times (B,) or (B, 1) and noisy actions (B, A) fp32. Returns eps_hat (B, A) fp32."""
        B = readout_mean.shape[0]
        dev = readout_mean.device
        t = time.reshape(-1).to(torch.int32).contiguous()
        if t.numel() != B or tuple(noisy_actions.shape) != (B, self.A):
            raise ValueError("time must hold one step per sample and noisy_actions be (B, A)")
        if readout_mean.shape[1] != self.D or readout_mean.dtype != torch.bfloat16:
            raise ValueError(f"readout_mean must be bf16 (B, {self.D})")
        cat = self.new_cat(B, dev)
        zeros = torch.zeros((B, self.A), dtype=torch.float32, device=dev)
        feats = torch.empty((B, self.time_dim), dtype=torch.bfloat16, device=dev)
        t_out = torch.empty(B, dtype=torch.int32, device=dev)
        eps_out = torch.empty((B, self.A), dtype=torch.float32, device=dev)
        _C.call("mmt_diffusion_prep", None, B, self.A, self.steps, 0, _C.ptr(zeros),
                _C.ptr(self.consts(dev)), _C.ptr(self.fourier.data), self.F, _C.ptr(t),
                _C.ptr(zeros), _C.ptr(t_out), _C.ptr(eps_out), _C.ptr(cat), cat.stride(0),
                _C.ptr(feats), _C.stream_ptr())
        cat[:, :self.A].copy_(noisy_actions)           # the given noisy sample (bf16 operand)
        self.readout_slot(cat).copy_(readout_mean)
        ht = self.t1.fwd(feats, act=K.ACT_RELU)
        self.t2.fwd(ht, out=cat[:, self.A:self.A + self.time_dim])
        hd = self.d1.fwd(cat, act=K.ACT_RELU)
        return self.d2.fwd(hd, out_mode=K.OUT_F32)

    # ------------------------------------------------------------------------- predict_action
    def sampler_coef(self, device) -> torch.Tensor:
        """(steps, 3) fp32 [1/sqrt(a_t), (1-a_t)/sqrt(1-abar_t), sqrt(b_t)] (:182-184)."""
        key = ("coef", device)
        if key not in self._dev_consts:
            b = self.betas_np.astype(np.float32)
            a = (np.float32(1) - b).astype(np.float32)
            c = np.stack([np.float32(1) / np.sqrt(a),
                          (np.float32(1) - a) / np.sqrt(np.float32(1) - self.alpha_hats_np),
                          np.sqrt(b)], axis=1).astype(np.float32)
            self._dev_consts[key] = torch.from_numpy(np.ascontiguousarray(c)).to(device)
        return self._dev_consts[key]

    def time_embeddings(self, device) -> torch.Tensor:
        """FourierFeatures (:41-51) + its MLPBlock for every t = 0..steps-1 -> (steps, T) bf16,
        through the training path's kernels (prep kernel with injected t, two GEMMs)."""
        S, A = self.steps, self.A
        t_in = torch.arange(S, dtype=torch.int32, device=device)
        zeros = torch.zeros((S, A), dtype=torch.float32, device=device)
        scratch = self.new_cat(S, device)
        feats = torch.empty((S, self.time_dim), dtype=torch.bfloat16, device=device)
        t_out = torch.empty(S, dtype=torch.int32, device=device)
        eps_out = torch.empty((S, A), dtype=torch.float32, device=device)
        _C.call("mmt_diffusion_prep", None, S, A, S, 0, _C.ptr(zeros), _C.ptr(self.consts(device)),
                _C.ptr(self.fourier.data), self.F, _C.ptr(t_in), _C.ptr(zeros), _C.ptr(t_out),
                _C.ptr(eps_out), _C.ptr(scratch), scratch.stride(0), _C.ptr(feats),
                _C.stream_ptr())
        ht = self.t1.fwd(feats, act=K.ACT_RELU)
        return self.t2.fwd(ht)

    def predict_action(self, readout_mean: torch.Tensor, rng=None, sample_offset: int = 0,
                       z: torch.Tensor | None = None, return_noise: bool = False):
        """Reference :146-209 (the 32-step DDPM loop of jax.lax.scan) on the device.
        readout_mean: (B, D) bf16 = mean of the readout tokens (:102). The initial sample z is
        drawn from the counter stream (rng = the (seed, step) device tensor, keyed by the global
        sample index sample_offset + b) unless injected. Returns actions (B, A) fp32 (and z)."""
        if readout_mean.dim() != 2 or readout_mean.shape[1] != self.D \
                or readout_mean.dtype != torch.bfloat16 or readout_mean.stride(1) != 1:
            raise ValueError(f"readout_mean must be bf16 (B, {self.D}) with unit inner stride")
        if self.A != 8:
            raise ValueError("the reference sampler hard-codes an 8-dim action (diffusion.py:200)")
        B = readout_mean.shape[0]
        dev = readout_mean.device
        if z is not None and (tuple(z.shape) != (B, self.A) or z.dtype != torch.float32
                              or not z.is_contiguous()):
            raise ValueError(f"z must be contiguous fp32 ({B}, {self.A})")
        if z is None and rng is None:
            raise ValueError("need rng (or an injected initial sample z)")
        A, T = self.A, self.time_dim
        temb = self.time_embeddings(dev)
        w1 = self.d1.w.bf16
        # concatenate([noisy, time_emb, readout]) . W1^T (OctoDenoise :61) split along the input
        Q = K.gemm(temb, w1[:, A:A + T], trans_b=True, bias=self.d1.b.data, out_mode=K.OUT_F32)
        P = K.gemm(readout_mean, w1[:, A + T:], trans_b=True, out_mode=K.OUT_F32)
        actions = torch.empty((B, A), dtype=torch.float32, device=dev)
        z_out = torch.empty((B, A), dtype=torch.float32, device=dev) if return_noise else None
        _C.call("mmt_diffusion_sample", _C.ptr(rng), B, A, self.steps, sample_offset, _C.ptr(P),
                P.stride(0), _C.ptr(Q), Q.stride(0), _C.ptr(w1), w1.stride(0),
                _C.ptr(self.d2.w.bf16), _C.ptr(self.d2.b.data), _C.ptr(self.sampler_coef(dev)),
                _C.ptr(z), self.hidden, _C.ptr(actions), _C.ptr(z_out), _C.stream_ptr())
        return (actions, z_out) if return_noise else actions

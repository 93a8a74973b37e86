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
from ..module_api import Bindable, init_from_spec, sget, spec
from ..params import ParamStore

_REF = "multi_modal_transformers."
_REF_MLP = _REF + "attention_blocks.attention.MLPBlock"
_REF_DENOISE = _REF + "action_heads.diffusion.OctoDenoise"
_REF_FOURIER = _REF + "action_heads.diffusion.FourierFeatures"


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


class DiffusionActionHead(Bindable):
    """Reference :68-209: ``DiffusionActionHead(diffusion_steps, attention_pooling,
    denoising_model, rng_collection="diffusion")`` with the model_configs/action_heads/diffusion.yaml
    nodes: ``denoising_model`` = OctoDenoise(time_encoder = FourierFeatures(output_dim, kernel_init,
    mlp_block), num_blocks, mlp_block) (:30-65). ``attention_pooling`` is accepted and unused, as in
    the reference (the pooling call is commented out, :99-102: the readouts are averaged).
    ``denoise_loss(readouts, actions)``, ``predict_denoise_term(readouts, time, noisy_actions)`` and
    ``predict_action(readouts)`` take the readout tokens (B, n, D) like the reference; the Octo
    training path feeds the readout MEAN straight from the backbone's fused rows-mean kernel
    (``loss_forward`` / ``*_mean``)."""

    def __init__(self, diffusion_steps: int = 32, attention_pooling=None, denoising_model=None,
                 rng_collection: str = "diffusion"):
        self.steps = int(diffusion_steps)
        self.rng_collection = rng_collection
        self.attention_pooling = attention_pooling
        dm = spec(denoising_model)
        te = spec(sget(dm, "time_encoder"))
        self.num_blocks = int(sget(dm, "num_blocks", 1))
        if self.num_blocks < 1:
            raise ValueError("OctoDenoise num_blocks must be >= 1")
        mlp = spec(sget(dm, "mlp_block"))
        self.time_dim_cfg = sget(te, "output_dim")
        self.fourier_init = sget(te, "kernel_init")
        tm = spec(sget(te, "mlp_block"))
        self.time_mlp_cfg = (sget(getattr(tm, "dense_spec", None), "features"),
                             sget(getattr(tm, "dense_out_spec", None), "features"))
        self.hidden_cfg = sget(getattr(mlp, "dense_spec", None), "features")
        self.A = int(sget(getattr(mlp, "dense_out_spec", None), "features", 8))
        betas = cosine_beta_schedule(self.steps)
        self.betas_np = betas
        self.alpha_hats_np = alpha_hats_of(betas)
        self._dev_consts = {}

    @classmethod
    def create(cls, store: ParamStore, name: str, embedding_dim: int, action_dim: int = 8,
               diffusion_steps: int = 32, time_dim: int | None = None,
               hidden: int | None = None, num_blocks: int = 1) -> "DiffusionActionHead":
        """The head from its dimensions, declared in ``store`` (the Octo model's path)."""
        D = embedding_dim
        T = time_dim or D

        def mlp(h, o):
            return {"_target_": _REF_MLP, "dense": {"_target_": "flax.linen.Dense", "features": h},
                    "dense_out": {"_target_": "flax.linen.Dense", "features": o}}
        dm = {"_target_": _REF_DENOISE, "num_blocks": num_blocks,
              "time_encoder": {"_target_": _REF_FOURIER, "output_dim": T, "mlp_block": mlp(T, T)},
              "mlp_block": mlp(hidden or D, action_dim)}
        return cls(diffusion_steps, None, dm).bind(store, name, D)

    def _declare(self, store: ParamStore, name: str, embedding_dim: int):
        D = embedding_dim
        self.D = D
        T0 = int(self.time_dim_cfg or D)
        self.F = T0 // 2
        T = 2 * self.F
        t_h, t_o = self.time_mlp_cfg
        if (t_h is not None and int(t_h) != T) or (t_o is not None and int(t_o) != T):
            raise NotImplementedError("FourierFeatures' MLPBlock must keep the output_dim width")
        self.time_dim = T
        self.hidden = int(self.hidden_cfg or D)
        p = f"{name}/OctoDenoise_0"
        self.fourier = store.add(f"{p}/FourierFeatures_0/fourier_kernel", (self.F, 1),
                                 init_from_spec(self.fourier_init, (self.F, 1)))
        self.t1 = Dense(store, f"{p}/FourierFeatures_0/MLPBlock_0/Dense_0", T, T)
        self.t2 = Dense(store, f"{p}/FourierFeatures_0/MLPBlock_0/Dense_1", T, T)
        self.cat_dim = self.A + T + D
        self.d1 = Dense(store, f"{p}/MLPBlock_0/Dense_0", self.cat_dim, self.hidden)
        self.d2 = Dense(store, f"{p}/MLPBlock_0/Dense_1", self.hidden, self.A)
        if self.cat_dim % 8:
            raise ValueError("action_dim + time_dim + D must be a multiple of 8 (16-B rows)")
        # OctoDenoise blocks 1.. (diffusion.py:62-63: a fresh MLPBlock per iteration, Flax names
        # MLPBlock_{i}) on the previous block's (B, A) output
        self.extra = [(Dense(store, f"{p}/MLPBlock_{i}/Dense_0", self.A, self.hidden),
                       Dense(store, f"{p}/MLPBlock_{i}/Dense_1", self.hidden, self.A))
                      for i in range(1, self.num_blocks)]
        if self.extra and self.A % 8:
            raise ValueError("OctoDenoise num_blocks > 1 needs action_dim % 8 == 0 (16-B rows)")

    # ------------------------------------------------------------- reference-signature methods
    def _mean_into(self, readouts: torch.Tensor, out: torch.Tensor):
        """mean over the readout axis (:102) of (B, n, D) readouts into a (B, D) bf16 view."""
        if readouts.dim() != 3 or readouts.stride(2) != 1:
            raise ValueError(f"readouts must be (batch, tokens, {self.D}) with unit inner stride")
        B, n, D = readouts.shape
        x = readouts if readouts.dtype == torch.float32 else readouts.float()
        rows = torch.arange(n, dtype=torch.int32, device=readouts.device)
        _C.call("mmt_rows_mean_fwd", _C.ptr(x), x.stride(0), x.stride(1), B, D, _C.ptr(rows), n,
                _C.ptr(out), out.stride(0), _C.stream_ptr())
        return out

    def denoise_loss(self, readouts: torch.Tensor, actions: torch.Tensor, train: bool = True, *,
                     rng=None, sample_offset: int = 0) -> torch.Tensor:
        """Reference :110-143: t ~ U{0..steps-1}, eps ~ N(0, 1) from the 'diffusion' counter
        stream (rng, keyed by the global sample index), noisy = sqrt(abar) a + sqrt(1 - abar) eps,
        loss = mean_b sum_a 0.5 (pred - eps)^2. Returns the loss (1,) fp32 on the device."""
        self._ensure(readouts.device, int(readouts.shape[-1]))
        if rng is None:
            raise ValueError("denoise_loss needs the diffusion rng (rng=)")
        B = readouts.shape[0]
        if tuple(actions.shape) != (B, self.A):
            raise ValueError(f"actions must be ({B}, {self.A})")
        cat = self.new_cat(B, readouts.device)
        self._mean_into(readouts, self.readout_slot(cat))
        loss, _ = self.loss_forward(cat, actions.float().contiguous(), rng, sample_offset)
        return loss

    def predict_denoise_term(self, readouts: torch.Tensor, time: torch.Tensor,
                             noisy_actions: torch.Tensor, train: bool = True) -> torch.Tensor:
        """Reference :88-107: OctoDenoise(noisy, time, mean(readouts)) -> (B, A) fp32."""
        self._ensure(readouts.device, int(readouts.shape[-1]))
        e = torch.empty((readouts.shape[0], self.D), dtype=torch.bfloat16, device=readouts.device)
        return self.predict_denoise_term_mean(self._mean_into(readouts, e), time,
                                              noisy_actions.float().contiguous())

    def predict_action(self, readouts: torch.Tensor, train: bool = True, *, rng=None,
                       sample_offset: int = 0, z: torch.Tensor | None = None,
                       return_noise: bool = False):
        """Reference :146-209: the 32-step DDPM sampler from the readouts (B, n, D)."""
        self._ensure(readouts.device, int(readouts.shape[-1]))
        e = torch.empty((readouts.shape[0], self.D), dtype=torch.bfloat16, device=readouts.device)
        return self.predict_action_mean(self._mean_into(readouts, e), rng, sample_offset, z,
                                        return_noise)

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
        pred, chain = self._extra_fwd(pred)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        dpred = torch.empty((B, self.A), dtype=torch.bfloat16, device=dev)
        _C.call("mmt_diffusion_loss", _C.ptr(pred), pred.stride(0), _C.ptr(eps), B, self.A, 1.0,
                _C.ptr(loss), _C.ptr(dpred), _C.stream_ptr())
        return loss, dict(cat=cat, feats=feats, ht=ht, hd=hd, dpred=dpred, t=t, eps=eps, pred=pred,
                          chain=chain)

    def _extra_fwd(self, pred):
        """OctoDenoise blocks 1.. on the block-0 output pred (B, A) fp32: each input cast to bf16
        (the GEMM operand), Dense -> relu -> Dense. Returns (final pred, [(x, h) per block])."""
        chain = []
        for d1, d2 in self.extra:
            x = K.cast_f32_bf16(pred, torch.empty(pred.shape, dtype=torch.bfloat16, device=pred.device))
            h = d1.fwd(x, act=K.ACT_RELU)
            pred = d2.fwd(h, out_mode=K.OUT_F32)
            chain.append((x, h))
        return pred, chain

    def loss_backward(self, sv: dict) -> torch.Tensor:
        """Returns d(readout mean) (B, D) bf16 view."""
        B = sv["cat"].shape[0]
        dpred = sv["dpred"]
        for (d1, d2), (x, h) in reversed(list(zip(self.extra, sv.get("chain") or []))):
            dz = d2.bwd(dpred, h, gate=h, gate_scale=1.0)     # relu backward in the dX epilogue
            dpred = d1.bwd(dz, x)                              # bf16 (B, A): the previous output's
        dzd = self.d2.bwd(dpred, sv["hd"], gate=sv["hd"], gate_scale=1.0)
        dcat = self.d1.bwd(dzd, sv["cat"])
        dtemb = dcat[:, self.A:self.A + self.time_dim]
        dzt = self.t2.bwd(dtemb, sv["ht"], gate=sv["ht"], gate_scale=1.0)
        dfeats = self.t1.bwd(dzt, sv["feats"])
        _C.call("mmt_fourier_bwd", _C.ptr(dfeats), B, self.F, _C.ptr(sv["t"]),
                _C.ptr(self.fourier.data), _C.ptr(self.fourier.grad), _C.stream_ptr())
        return dcat[:, self.A + self.time_dim:]

    # ------------------------------------------------------------------ predict_denoise_term
    def predict_denoise_term_mean(self, readout_mean: torch.Tensor, time: torch.Tensor,
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
        return self._extra_fwd(self.d2.fwd(hd, out_mode=K.OUT_F32))[0]

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

    def predict_action_mean(self, readout_mean: torch.Tensor, rng=None, sample_offset: int = 0,
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
        if self.extra:
            return self._predict_action_loop(readout_mean, rng, sample_offset, z, return_noise)
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

    def _predict_action_loop(self, readout_mean, rng, sample_offset, z, return_noise):
        """predict_action for OctoDenoise num_blocks > 1 (the fused one-launch sampler holds one
        MLPBlock in registers): the reference's 32-step scan (:146-209) as a loop of
        predict_denoise_term_mean launches and the clipped update on the device; the initial
        sample z comes from the fused sampler's own counter-stream draw (a one-step launch), so
        both paths start from the same z. The noisy sample enters the denoiser as its bf16 GEMM
        operand (the fused kernel keeps it fp32)."""
        B, A, dev = readout_mean.shape[0], self.A, readout_mean.device
        if z is None:
            z = torch.empty((B, A), dtype=torch.float32, device=dev)
            T = self.time_dim
            temb = self.time_embeddings(dev)
            w1 = self.d1.w.bf16
            Q = K.gemm(temb, w1[:, A:A + T], trans_b=True, bias=self.d1.b.data, out_mode=K.OUT_F32)
            P = K.gemm(readout_mean, w1[:, A + T:], trans_b=True, out_mode=K.OUT_F32)
            scratch = torch.empty((B, A), dtype=torch.float32, device=dev)
            _C.call("mmt_diffusion_sample", _C.ptr(rng), B, A, 1, sample_offset, _C.ptr(P),
                    P.stride(0), _C.ptr(Q), Q.stride(0), _C.ptr(w1), w1.stride(0),
                    _C.ptr(self.d2.w.bf16), _C.ptr(self.d2.b.data), _C.ptr(self.sampler_coef(dev)),
                    None, self.hidden, _C.ptr(scratch), _C.ptr(z), _C.stream_ptr())
        coef = self.sampler_coef(dev)
        x = z.clone()
        for t in range(self.steps - 1, -1, -1):
            tt = torch.full((B,), t, dtype=torch.int32, device=dev)
            eps = self.predict_denoise_term_mean(readout_mean, tt, x)
            x = torch.clamp(coef[t, 0] * (x - coef[t, 1] * eps) + coef[t, 2] * z, -5.0, 5.0)
        return (x, z) if return_noise else x

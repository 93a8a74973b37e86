"""Gato-style image tokenizer, mirroring the reference's
``multi_modal_transformers/tokenizers/images/image_tokenizer.py``:
``image_to_patches`` (:35-71), ``encode_patch_position`` (:74-132), ``ResNetV2Block`` (:140-178)
and ``ImageTokenizer`` (:216-309), configured by ``model_configs/tokenizers/images/gato_resnet.yaml``.

On MI355X the whole stem is five kernels + four MFMA GEMMs per step (csrc/stem.hip): fused
patchify/normalise/im2col, conv-as-GEMM, per-patch max-pool, GroupNorm+gelu (x2) with the 3x3 SAME
convolutions reduced to their centre tap (the pooled map is 1x1 at patch 16), residual add fused
into a GEMM epilogue, and the output Dense. Position tokens are drawn on the device.

Geometry: the pooled map is 1x1 at patch 16 (every BASELINE config; the centre-tap form above).
Larger maps — the reference's own patch 56 (23x23 conv map, 21x21 pooled) — take the general
form: max_pool 3x3 s1 over the map, the 3x3 SAME convs as im2col + GEMM (+ col2im backward),
GroupNorm over all patches x positions of a sample, flatten (h, w, c) and the output Dense over
PH*PW*C features (image_tokenizer.py:156-176). Its Conv_{1,2} kernels are the full (3, 3, C, C)
(stored (9C, C)); the 1x1 form stores only the centre tap (C, C).
"""
from __future__ import annotations

import numpy as np
import torch

from ... import _kernels as K
from ...layers import Dense
from ...params import ParamStore, const, he_normal, normal, variance_scaling_normal


# ------------------------------------------------------------------ reference helper API (host)
def image_to_patches(image: torch.Tensor, patch_size: int, normalize: bool) -> torch.Tensor:
    """Reference :35-71 for one (H, W, C) image (torch; reference-API helper)."""
    h, w, c = image.shape
    if h != w:
        raise ValueError("image must be square (image_tokenizer.py:49-50)")
    if h % patch_size:
        raise ValueError("image size must be divisible by the patch size (the reference's resize "
                         "branch, :54-59, is broken; rejected here)")
    n = h // patch_size
    p = image.reshape(n, patch_size, n, patch_size, c).permute(0, 2, 1, 3, 4).reshape(
        n * n, patch_size, patch_size, c)
    if normalize:
        p = 2 * (p / 255.0) - 1.0
    return p


def encode_patch_position(image_hw: int, patch_size: int, num_tokens: int, train: bool = False,
                          rng=None, sample_offset: int = 0, device="cuda"):
    """Reference :74-132 for one square image side ``image_hw``; returns (row, col) int32 tokens
    computed by the device kernel (train: counter-stream randint; eval: interval centre)."""
    rt, ct = K.patch_positions(1, 1, image_hw, patch_size, num_tokens, train, rng=rng,
                               sample_offset=sample_offset, device=device)
    return rt[0], ct[0]


class ResNetV2Block:
    """Reference :140-178 / gato_resnet.yaml:41-104 parameters."""

    def __init__(self, store: ParamStore, name: str, in_channels: int, features: int = 64,
                 conv_kernel=(12, 12), conv_stride=2, pool=(3, 3), num_blocks: int = 2,
                 num_groups: int = 32, gn_eps: float = 1e-6, embedding_dim: int = 384,
                 patch_size: int = 16):
        kh, kw = conv_kernel
        self.kh, self.kw, self.stride = kh, kw, conv_stride
        self.oh = (patch_size - kh) // conv_stride + 1
        self.ow = (patch_size - kw) // conv_stride + 1
        if pool[0] != pool[1] or self.oh < pool[0] or self.ow < pool[1]:
            raise ValueError(f"pool {pool} on a {self.oh}x{self.ow} conv map")
        self.kp = pool[0]
        self.ph, self.pw = self.oh - pool[0] + 1, self.ow - pool[1] + 1
        self.general = (self.ph, self.pw) != (1, 1)   # else the 1x1 centre-tap form
        self.ks = 3                                   # resnet_conv 3x3 SAME (gato_resnet.yaml:88-92)
        self.win = self.oh * self.ow
        self.C, self.G, self.eps = features, num_groups, gn_eps
        self.num_blocks = num_blocks
        K_in = kh * kw * in_channels
        # input_conv (Conv 12x12 s2 VALID, he_normal over (kh, kw, cin, cout) -> fan_in = K_in)
        self.conv = Dense(store, f"{name}/Conv_0", K_in, features,
                          kernel_init=he_normal((K_in, features)), bias_init=normal(0.01))
        self.gn, self.convs = [], []
        for i in range(num_blocks):
            self.gn.append((store.add(f"{name}/GroupNorm_{i}/scale", (features,), const(1.0)),
                            store.add(f"{name}/GroupNorm_{i}/bias", (features,), const(0.0))))
            # 3x3 SAME conv: the full (9C, C) kernel on a larger map; on a 1x1 map only the centre
            # tap acts (fan_in of the full kernel either way)
            cin = 9 * features if self.general else features
            self.convs.append(Dense(store, f"{name}/Conv_{i + 1}", cin, features,
                                    kernel_init=he_normal((9 * features, features))))
        flat = self.ph * self.pw * features                 # flatten (h, w, c) (:174-175)
        self.out = Dense(store, f"{name}/Dense_0", flat, embedding_dim,
                         kernel_init=he_normal((flat, embedding_dim)))

    def fused_ok(self, images: torch.Tensor, patch_size: int, normalize: bool) -> bool:
        """The 64-channel 12x12 s2 conv + 3x3 pool on 16x16 uint8 RGB patches runs as one kernel
        (csrc/stem.hip stem_conv_pool_kernel) without an im2col matrix."""
        return (images.dtype == torch.uint8 and images.shape[-1] == 3 and patch_size == 16 and
                normalize and (self.kh, self.kw, self.stride, self.kp, self.C) == (12, 12, 2, 3, 64))

    def forward(self, A, B: int, R: int, images=None):
        """A: im2col rows (B*R*win, K_in), or None with `images` (B, I, H, W, 3) uint8 for the
        fused conv + pool (fused_ok). Returns tokens (B*R, D) bf16 and the saved state."""
        if self.general:
            return self._forward_general(A, B, R)
        # pre-normalisation tensors are fp32 (GroupNorm spans all patches of a sample: same
        # conditioning argument as the sequence LayerNorm, csrc/norm.hip)
        if A is None:
            pooled, arg = K.stem_conv_pool(images, self.conv.w.bf16, self.conv.b.data)
        else:
            conv = self.conv.fwd(A, out_mode=K.OUT_F32)           # (B*R*win, C)
            pooled, arg = K.maxpool_patch(conv, self.win)         # (B*R, C) fp32
        hs, zs, stats = [], [], []
        z = pooled
        for i in range(self.num_blocks):
            g, b = self.gn[i]
            h, mu, rs = K.groupnorm_gelu_fwd(z.view(B, R, self.C), self.G, g.data, b.data, self.eps)
            residual = pooled if i == self.num_blocks - 1 else None
            zn = self.convs[i].fwd(h.view(B * R, self.C), residual=residual, out_mode=K.OUT_F32)
            hs.append(h)
            zs.append(z)
            stats.append((mu, rs))
            z = zn
        r16 = K.cast_f32_bf16(z, torch.empty(z.shape, dtype=torch.bfloat16, device=z.device))
        tok = self.out.fwd(r16)                                   # (B*R, D)
        return tok, dict(A=A, images=images, arg=arg, pooled=pooled, hs=hs, zs=zs, stats=stats,
                         r=r16, B=B, R=R)

    def backward(self, dtok: torch.Tensor, sv: dict):
        if self.general:
            return self._backward_general(dtok, sv)
        B, R = sv["B"], sv["R"]
        dz = self.out.bwd(dtok, sv["r"], out_mode=K.OUT_F32)     # d(residual sum) (B*R, C) fp32
        dpooled = dz.clone()                                     # residual branch
        for i in reversed(range(self.num_blocks)):
            g, b = self.gn[i]
            dz16 = K.cast_f32_bf16(dz, torch.empty(dz.shape, dtype=torch.bfloat16, device=dz.device))
            dh = self.convs[i].bwd(dz16, sv["hs"][i].view(B * R, self.C), out_mode=K.OUT_F32)
            mu, rs = sv["stats"][i]
            zin = sv["zs"][i].view(B, R, self.C)
            if i == 0:   # input of GN_0 is pooled: accumulate into the residual gradient
                K.groupnorm_gelu_bwd(dh.view(B, R, self.C), zin, self.G, g.data, b.data, mu, rs,
                                     g.grad, b.grad, dx=dpooled.view(B, R, self.C), accumulate=True)
            else:
                dz = K.groupnorm_gelu_bwd(dh.view(B, R, self.C), zin, self.G, g.data, b.data, mu,
                                          rs, g.grad, b.grad).view(B * R, self.C)
        K.colsum(dpooled, self.conv.b.grad)                      # bias added before the max
        if sv["A"] is None:  # fused forward: the weight gradient straight from the images
            K.stem_conv_wgrad(sv["images"], dpooled, sv["arg"], self.conv.w.grad)
            return
        G = K.maxpool_patch_bwd(dpooled, sv["arg"], self.win)    # (B*R*win, C)
        self.conv.bwd(G, sv["A"], need_dx=False, bias_grad_done=True)


    # ---------------------------------------------------------------- general maps (patch 56)
    def _forward_general(self, A: torch.Tensor, B: int, R: int):
        n, C, PH, PW, ks = B * R, self.C, self.ph, self.pw, self.ks
        conv = self.conv.fwd(A, out_mode=K.OUT_F32)               # (n*OH*OW, C)
        pooled, arg = K.maxpool2d(conv, n, self.oh, self.ow, self.kp)   # (n*PH*PW, C) fp32
        hs, cols, zs, stats = [], [], [], []
        z = pooled
        for i in range(self.num_blocks):
            g, b = self.gn[i]
            # GroupNorm over every non-batch axis: the R patches x PH x PW positions of a sample
            h, mu, rs = K.groupnorm_gelu_fwd(z.view(B, R * PH * PW, C), self.G, g.data, b.data, self.eps)
            col = K.im2col_same(h.view(n * PH * PW, C), n, PH, PW, ks)
            residual = pooled if i == self.num_blocks - 1 else None
            zn = self.convs[i].fwd(col, residual=residual, out_mode=K.OUT_F32)
            cols.append(col)
            zs.append(z)
            stats.append((mu, rs))
            z = zn
        r16 = K.cast_f32_bf16(z, torch.empty(z.shape, dtype=torch.bfloat16, device=z.device))
        tok = self.out.fwd(r16.view(n, PH * PW * C))               # flatten (h, w, c)
        return tok, dict(A=A, arg=arg, cols=cols, zs=zs, stats=stats, r=r16, B=B, R=R)

    def _backward_general(self, dtok: torch.Tensor, sv: dict):
        B, R = sv["B"], sv["R"]
        n, C, PH, PW, ks = B * R, self.C, self.ph, self.pw, self.ks
        dz = self.out.bwd(dtok, sv["r"].view(n, PH * PW * C), out_mode=K.OUT_F32)
        dz = dz.view(n * PH * PW, C)
        dpooled = dz.clone()                                       # residual branch
        for i in reversed(range(self.num_blocks)):
            g, b = self.gn[i]
            dz16 = K.cast_f32_bf16(dz, torch.empty(dz.shape, dtype=torch.bfloat16, device=dz.device))
            dcol = self.convs[i].bwd(dz16, sv["cols"][i], out_mode=K.OUT_F32)   # (rows, 9C)
            dh = K.col2im_same(dcol, n, PH, PW, C, ks)
            mu, rs = sv["stats"][i]
            zin = sv["zs"][i].view(B, R * PH * PW, C)
            if i == 0:
                K.groupnorm_gelu_bwd(dh.view(B, R * PH * PW, C), zin, self.G, g.data, b.data, mu, rs,
                                     g.grad, b.grad, dx=dpooled.view(B, R * PH * PW, C),
                                     accumulate=True)
            else:
                dz = K.groupnorm_gelu_bwd(dh.view(B, R * PH * PW, C), zin, self.G, g.data, b.data,
                                          mu, rs, g.grad, b.grad).view(n * PH * PW, C)
        G = K.maxpool2d_bwd(dpooled, sv["arg"], n, self.oh, self.ow, self.kp)
        K.colsum(dpooled, self.conv.b.grad)                        # bias added before the max
        self.conv.bwd(G, sv["A"], need_dx=False, bias_grad_done=True)


class ImageTokenizer:
    """Reference :216-309: patches -> ResNetV2 stem -> Dense, + row/col position embeddings."""

    def __init__(self, store: ParamStore, name: str, image_size, patch_size: int, normalize: bool,
                 position_interval: int, embedding_dim: int, rng_collection: str = "patch_encoding",
                 resnet: dict | None = None):
        self.image_size = tuple(image_size)
        self.patch_size = patch_size
        self.normalize = normalize
        self.Q = position_interval
        self.D = embedding_dim
        self.rng_collection = rng_collection
        H, W, C = self.image_size
        if H != W:
            raise ValueError("square images only (image_tokenizer.py:49-50)")
        self.num_patches = (H // patch_size) ** 2
        emb_init = variance_scaling_normal(1.0, (position_interval, embedding_dim))
        self.row_emb = store.add(f"{name}/image_row_position_embedding/embedding",
                                 (position_interval, embedding_dim), emb_init)
        self.col_emb = store.add(f"{name}/image_col_position_embedding/embedding",
                                 (position_interval, embedding_dim), emb_init)
        self.resnet = ResNetV2Block(store, f"{name}/ResNetV2Block_0", C,
                                    embedding_dim=embedding_dim, patch_size=patch_size,
                                    **(resnet or {}))

    def check(self, images: torch.Tensor):
        if tuple(images.shape[-3:]) != self.image_size:
            # the reference calls sys.exit here (:246-249)
            raise ValueError(f"input image size {tuple(images.shape[-3:])} != {self.image_size}")

    def forward(self, images: torch.Tensor, train: bool, rng=None, sample_offset: int = 0,
                positions=None):
        """images (B, I, H, W, C) fp32 [0, 255] or uint8. Returns patch tokens (B, I*NP, D)
        WITHOUT the position embeddings (added by the fused sequence assembly), the (row, col)
        tokens and the saved state."""
        self.check(images)
        B, I = images.shape[:2]
        rs = self.resnet
        images = images.contiguous()
        if not rs.general and rs.fused_ok(images, self.patch_size, self.normalize):
            tok, sv = rs.forward(None, B, I * self.num_patches, images=images)
        else:
            A = K.patch_im2col(images, self.patch_size, rs.kh, rs.kw, rs.stride, self.normalize)
            tok, sv = rs.forward(A, B, I * self.num_patches)
        if positions is None:
            positions = K.patch_positions(B, I, self.image_size[0], self.patch_size, self.Q, train,
                                          rng=rng, site=0, sample_offset=sample_offset,
                                          device=images.device)
        return tok.view(B, I * self.num_patches, self.D), positions, sv

    def backward(self, dtok: torch.Tensor, sv: dict):
        self.resnet.backward(dtok.reshape(-1, self.D), sv)

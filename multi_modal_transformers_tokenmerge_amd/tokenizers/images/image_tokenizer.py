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

from ... import _C, _kernels as K
from ...config_loader import LayerSpec
from ...layers import Dense
from ...module_api import Bindable, init_from_spec, sget, spec
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


class ResNetV2Block(Bindable):
    """Reference :140-178: ``ResNetV2Block(num_blocks, input_conv, input_pool, resnet_norm,
    resnet_activation, resnet_conv, output_dense)(x)`` with the gato_resnet.yaml:41-104 nodes
    (Conv 12x12 s2 VALID, max_pool 3x3 s1 VALID, GroupNorm, gelu, Conv 3x3 SAME, Dense); x are
    the normalised patches (B, I, NP, p, p, C) -> (B, I, NP, D). The input channels / patch size
    come from the first call or ``bind(store, name, in_channels, patch_size, embedding_dim)``."""

    def __init__(self, num_blocks: int = 2, input_conv=None, input_pool=None, resnet_norm=None,
                 resnet_activation=None, resnet_conv=None, output_dense=None):
        conv, pool, norm = spec(input_conv), spec(input_pool), spec(resnet_norm)
        rconv, act, dense = spec(resnet_conv), spec(resnet_activation), spec(output_dense)
        self.num_blocks = int(num_blocks)
        self.features = int(sget(conv, "features", 64))
        kh, kw = (int(v) for v in sget(conv, "kernel_size", (12, 12)))
        strides = tuple(int(v) for v in sget(conv, "strides", (2, 2)))
        if strides[0] != strides[1] or str(sget(conv, "padding", "VALID")).upper() != "VALID":
            raise NotImplementedError("input_conv: equal strides, VALID padding (gato_resnet.yaml:44-50)")
        self.kh, self.kw, self.stride = kh, kw, strides[0]
        pw = tuple(int(v) for v in sget(pool, "window_shape", (3, 3)))
        if tuple(int(v) for v in sget(pool, "strides", (1, 1))) != (1, 1) or pw[0] != pw[1]:
            raise NotImplementedError("input_pool: square window, stride 1 (gato_resnet.yaml:60-65)")
        self.kp = pw[0]
        self.G = int(sget(norm, "num_groups", 32))
        self.eps = float(sget(norm, "epsilon", 1e-6))
        if act is not None and not getattr(act, "target", "gelu").endswith("gelu"):
            raise NotImplementedError("resnet_activation: the fused GroupNorm kernels apply gelu")
        if rconv is not None and (int(sget(rconv, "features", self.features)) != self.features or
                                  tuple(int(v) for v in sget(rconv, "kernel_size", (3, 3))) != (3, 3)):
            raise NotImplementedError("resnet_conv: 3x3 SAME with the input_conv's features")
        self.out_features = sget(dense, "features")
        self.specs = dict(conv=conv, rconv=rconv, dense=dense)
        self.ks = 3
        self.C = self.features

    @classmethod
    def from_hparams(cls, features: int = 64, conv_kernel=(12, 12), conv_stride: int = 2,
                     pool=(3, 3), num_blocks: int = 2, num_groups: int = 32, gn_eps: float = 1e-6,
                     embedding_dim: int | None = None) -> "ResNetV2Block":
        """The block from OctoConfig.stem's hyper-parameters (config_loader.octo_config_from_yaml)."""
        return cls(num_blocks,
                   LayerSpec("flax.linen.Conv", {"features": features, "kernel_size": list(conv_kernel),
                                                 "strides": [conv_stride, conv_stride], "padding": "VALID"}),
                   LayerSpec("flax.linen.max_pool", {"window_shape": list(pool), "strides": [1, 1],
                                                     "padding": "VALID"}, partial=True),
                   LayerSpec("flax.linen.GroupNorm", {"num_groups": num_groups, "epsilon": gn_eps}),
                   LayerSpec("flax.linen.gelu", partial=True),
                   LayerSpec("flax.linen.Conv", {"features": features, "kernel_size": [3, 3],
                                                 "strides": [1, 1], "padding": "SAME"}),
                   LayerSpec("flax.linen.Dense", {"features": embedding_dim}))

    def _declare(self, store: ParamStore, name: str, in_channels: int, patch_size: int,
                 embedding_dim: int | None = None):
        D = int(self.out_features or embedding_dim or 0)
        if embedding_dim is not None and self.out_features is not None and int(self.out_features) != embedding_dim:
            raise ValueError(f"output_dense features {self.out_features} != embedding_dim {embedding_dim}")
        if D <= 0:
            raise ValueError("ResNetV2Block needs output_dense.features (or the tokenizer's embedding_dim)")
        kh, kw, features = self.kh, self.kw, self.features
        self.patch_size, self.D = patch_size, D
        self.oh = (patch_size - kh) // self.stride + 1
        self.ow = (patch_size - kw) // self.stride + 1
        if self.oh < self.kp or self.ow < self.kp:
            raise ValueError(f"pool {self.kp} on a {self.oh}x{self.ow} conv map")
        self.ph, self.pw = self.oh - self.kp + 1, self.ow - self.kp + 1
        self.general = (self.ph, self.pw) != (1, 1)   # else the 1x1 centre-tap form
        self.win = self.oh * self.ow
        K_in = kh * kw * in_channels
        sc, sr, sd = self.specs["conv"], self.specs["rconv"], self.specs["dense"]
        # input_conv (Conv 12x12 s2 VALID, he_normal over (kh, kw, cin, cout) -> fan_in = K_in)
        self.conv = Dense(store, f"{name}/Conv_0", K_in, features,
                          kernel_init=init_from_spec(sget(sc, "kernel_init"), (K_in, features)),
                          bias_init=init_from_spec(sget(sc, "bias_init"), (features,), normal(0.01)))
        self.gn, self.convs = [], []
        for i in range(self.num_blocks):
            self.gn.append((store.add(f"{name}/GroupNorm_{i}/scale", (features,), const(1.0)),
                            store.add(f"{name}/GroupNorm_{i}/bias", (features,), const(0.0))))
            # 3x3 SAME conv: the full (9C, C) kernel on a larger map; on a 1x1 map only the centre
            # tap acts (fan_in of the full kernel either way)
            cin = 9 * features if self.general else features
            self.convs.append(Dense(store, f"{name}/Conv_{i + 1}", cin, features,
                                    kernel_init=init_from_spec(sget(sr, "kernel_init"), (9 * features, features)),
                                    bias_init=init_from_spec(sget(sr, "bias_init"), (features,), normal(0.01))))
        flat = self.ph * self.pw * features                 # flatten (h, w, c) (:174-175)
        self.out = Dense(store, f"{name}/Dense_0", flat, D,
                         kernel_init=init_from_spec(sget(sd, "kernel_init"), (flat, D)),
                         bias_init=init_from_spec(sget(sd, "bias_init"), (D,), normal(0.01)))

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """x (B, I, NP, p, p, C) normalised patch pixels (fp32) -> tokens (B, I, NP, D) fp32."""
        if x.dim() != 6 or x.shape[3] != x.shape[4]:
            raise ValueError(f"patches must be (B, I, NP, p, p, C), got {tuple(x.shape)}")
        B, I, NP, p, _, C = x.shape
        self._ensure(x.device, C, p)
        if (p, C) != (self.patch_size, self.conv.in_f // (self.kh * self.kw)):
            raise ValueError(f"patches {p}x{p}x{C} do not match the bound block")
        pix = x.float().contiguous().view(B * I * NP, 1, p, p, C)  # one patch per "image"
        A = K.patch_im2col(pix, p, self.kh, self.kw, self.stride, normalize=False)
        tok, _ = self.forward(A, B, I * NP)
        return tok.float().view(B, I, NP, -1)

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


class ImageTokenizer(Bindable):
    """Reference :216-309: ``ImageTokenizer(image_size, patch_size, normalize, position_interval,
    rng_collection, embedding_dim, row_position_embedding, col_position_embedding, resnet)
    (image, train=True) -> (B, I, NP, D)`` = ResNetV2 patch embeddings + row / column position
    embeddings (flax.linen.Embed nodes, position_interval x embedding_dim). ``resnet`` is the
    ResNetV2Block node (or module, or OctoConfig.stem's hyper-parameter dict)."""

    def __init__(self, image_size, patch_size: int, normalize: bool = True,
                 position_interval: int = 128, rng_collection: str = "patch_encoding",
                 embedding_dim: int = 768, row_position_embedding=None, col_position_embedding=None,
                 resnet=None):
        self.image_size = tuple(int(v) for v in image_size)
        self.patch_size = int(patch_size)
        self.normalize = bool(normalize)
        self.Q = int(position_interval)
        self.D = int(embedding_dim)
        self.rng_collection = rng_collection
        H, W, C = self.image_size
        if H != W:
            raise ValueError("square images only (image_tokenizer.py:49-50)")
        self.num_patches = (H // self.patch_size) ** 2
        self.emb_specs = []
        for e in (spec(row_position_embedding), spec(col_position_embedding)):
            if e is not None and (int(sget(e, "num_embeddings", self.Q)) != self.Q or
                                  int(sget(e, "features", self.D)) != self.D):
                raise ValueError("position embeddings must be (position_interval, embedding_dim)")
            self.emb_specs.append(e)
        rs = spec(resnet)
        if rs is None:
            rs = ResNetV2Block.from_hparams(embedding_dim=self.D)
        elif isinstance(rs, dict):
            rs = ResNetV2Block.from_hparams(**rs, embedding_dim=self.D)
        if not isinstance(rs, ResNetV2Block):
            raise TypeError(f"resnet must be a ResNetV2Block node, got {type(rs).__name__}")
        self.resnet = rs
        self.row_emb = self.col_emb = None
        self._zero_pe = {}

    def _declare(self, store: ParamStore, name: str):
        H, W, C = self.image_size
        Q, D = self.Q, self.D

        def emb_init(e):
            return init_from_spec(sget(e, "embedding_init"), (Q, D), variance_scaling_normal(1.0, (Q, D)))
        self.row_emb = store.add(f"{name}/image_row_position_embedding/embedding", (Q, D),
                                 emb_init(self.emb_specs[0]))
        self.col_emb = store.add(f"{name}/image_col_position_embedding/embedding", (Q, D),
                                 emb_init(self.emb_specs[1]))
        self.resnet.bind(store, f"{name}/ResNetV2Block_0", C, self.patch_size, D)

    def __call__(self, image: torch.Tensor, train: bool = True, *, rng=None,
                 sample_offset: int = 0, positions=None) -> torch.Tensor:
        """image (B, I, H, W, C) uint8 / fp32 [0, 255] -> (B, I, NP, D) fp32 = patch embeddings +
        row + column position embeddings (:300-307). train draws the patch positions from the
        counter RNG ``rng`` (the 'patch_encoding' collection), keyed by the global sample index
        sample_offset + b; eval uses the interval midpoints."""
        self._ensure(image.device)
        if train and rng is None and positions is None:
            raise ValueError("ImageTokenizer(train=True) needs the patch_encoding rng (rng=)")
        tok, (rt, ct), _ = self.forward(image, train, rng, sample_offset, positions)
        B, NI, D = tok.shape
        key = (NI, image.device)
        if key not in self._zero_pe:
            self._zero_pe[key] = (torch.zeros((NI, D), dtype=torch.float32, device=image.device),
                                  torch.tensor([(1 << 24) | j for j in range(NI)], dtype=torch.int32,
                                               device=image.device))
        zpe, rows = self._zero_pe[key]
        out = torch.empty((B, NI, D), dtype=torch.float32, device=image.device)
        # tok + (row_emb[rt] + col_emb[ct]) in the arithmetic of the fused sequence assembly
        _C.call("mmt_seq_assemble_fwd", B, NI, D, _C.ptr(rows), None, 1, _C.ptr(tok), NI,
                _C.ptr(rt), _C.ptr(ct), _C.ptr(self.row_emb.data), _C.ptr(self.col_emb.data), None,
                _C.ptr(zpe), _C.ptr(out), _C.stream_ptr())
        return out.view(B, image.shape[1], self.num_patches, D)

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

"""GroupNorm+gelu forward: device bf16 output vs a float64 reference, in bf16 ulps; parity
cos_all over seeds (diagnostic)."""
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from multi_modal_transformers_tokenmerge_amd import _kernels as K  # noqa: E402

dev = torch.device("cuda")
for (B, R, C, G) in [(4, 256, 64, 32), (4, 100, 64, 32)]:
    g = torch.Generator().manual_seed(0)
    x = torch.randn((B, R, C), generator=g) * 2 + 0.5
    gamma = 1 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    y, mu, rs = K.groupnorm_gelu_fwd(x.to(dev), G, gamma.to(dev), beta.to(dev), 1e-6)
    xd = x.double().view(B, R, G, C // G)
    m = xd.mean(dim=(1, 3), keepdim=True)
    v = xd.var(dim=(1, 3), unbiased=False, keepdim=True)
    z = ((xd - m) / torch.sqrt(v + 1e-6)).view(B, R, C) * gamma.double() + beta.double()
    ref = 0.5 * z * (1 + torch.tanh(math.sqrt(2 / math.pi) * (z + 0.044715 * z ** 3)))
    yd = y.double().cpu()
    ulp = torch.clamp(ref.abs(), min=2 ** -20) * 2 ** -8
    err = ((yd - ref).abs() / ulp)
    print(B, R, C, G, "max err in bf16 ulps", float(err.max()), "frac > 1 ulp", float((err > 1).double().mean()),
          "mu err", float((mu.cpu().double() - m.view(B, G)).abs().max()))

from oracle.parity import run_parity  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config  # noqa: E402
for seed in range(4):
    res = run_parity(get_config("octo-small-tome16", num_blocks=3, t5=T5Config(num_layers=2)), 2, seed=seed)
    print("seed", seed, "loss", res["loss"], res["ref_loss"], "cos_all", res["cos_all"],
          "min cos", min(res["cos"].values()))

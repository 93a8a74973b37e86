"""Scale bias of the attention backward (VERDICT r04 item 1 diagnosis): HIP dq / dk / dv against
the fp32 autograd reference and the bf16-emulating restatement (oracle/octo_ref.FlashAttnBF16 in
float64) on the same bf16 inputs, per component: norm ratio |hip| / |ref|, projection coefficient
<hip, ref> / |ref|^2 and relative L2, also for the column sums (the fused QKV bias gradient).

    python tools/attn_bias.py      (GPU)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from oracle.octo_ref import FlashAttnBF16
from tests.test_attn_norm_gpu import bits_to_keep, dense_mask, octo_small_table


def stats(h, r):
    h, r = h.double().flatten(), r.double().flatten()
    nr = r.norm()
    return float(h.norm() / nr), float(h @ r / nr ** 2), float((h - r).norm() / nr)


def run(B, L, H, Dh, drop, qscale, seed=0):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((B, L, 3 * H * Dh), generator=g)
    x[..., :H * Dh] *= qscale
    qkv = x.bfloat16().to(dev)
    scale = Dh ** -0.5
    starts, lens, vis = octo_small_table(32, L - 36, 4)
    table = K.SetTable(starts, lens, vis)
    mask = dense_mask(starts, lens, vis, L, dev)
    kp = 0.9 if drop else 1.0
    rng = torch.tensor([77, 5], dtype=torch.int32, device=dev)
    bits = K.dropout_bits(rng, 3, 7, L, L, kp) if drop else None
    keep = bits_to_keep(bits, L).to(dev) if drop else None
    o, lse = K.attn_fwd(qkv, H, scale, table, bits, kp)
    dout = torch.randn((B, L, H * Dh), generator=g).bfloat16().to(dev)
    dqkv = K.attn_bwd(qkv, o, dout, lse, H, scale, table, bits, kp)
    torch.cuda.synchronize()
    # the bf16-emulating restatement in float64 (the oracle's storage points)
    q, k, v = qkv.double().cpu().view(B, L, 3, H, Dh).unbind(2)
    q, k, v = (t.clone().requires_grad_() for t in (q, k, v))
    ke = keep.cpu() if keep is not None else None
    oe = FlashAttnBF16.apply(q, k, v, mask.cpu(), ke, kp, scale, None)
    oe.backward(dout.double().cpu().view(B, L, H, Dh))
    out = []
    ho = o.double().cpu().view(B, L, H, Dh)
    out.append(("O", stats(ho, oe.detach())))
    hg = dqkv.double().cpu().view(B, L, 3, H, Dh)
    for i, (nm, t) in enumerate(zip("qkv", (q, k, v))):
        out.append((f"d{nm}", stats(hg[:, :, i], t.grad)))
        out.append((f"d{nm} colsum", stats(hg[:, :, i].sum((0, 1)), t.grad.sum((0, 1)))))
    return out


def main():
    for cfg in [(2, 292, 6, 64, True, 1.0), (2, 292, 6, 64, False, 1.0), (2, 292, 6, 64, True, 4.0),
                (2, 292, 6, 64, False, 4.0), (2, 276, 6, 64, True, 2.0), (1, 1064, 2, 64, True, 2.0)]:
        res = run(*cfg)
        print(f"B={cfg[0]} L={cfg[1]} H={cfg[2]} drop={cfg[4]} qscale={cfg[5]}: " +
              "  ".join(f"{nm} ratio {r:.4f} a {a:.4f} rel {e:.2e}" for nm, (r, a, e) in res), flush=True)


if __name__ == "__main__":
    main()

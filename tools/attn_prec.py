"""Forward / backward error of the resident and the tiled attention kernels against float64
torch on the same bf16 inputs (octo-small block-0 shape, token-set mask, dropout)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tests.test_attn_norm_gpu import bits_to_keep, dense_mask, octo_small_table


def ref(qkv, H, scale, mask, keep, kp, dout):
    B, L, three = qkv.shape
    Dh = three // (3 * H)
    x = qkv.double().requires_grad_()
    q, k, v = x.view(B, L, 3, H, Dh).unbind(2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    s = torch.where(mask[None, None], s, -1e300)
    p = torch.softmax(s, -1)
    if keep is not None:
        p = torch.where(keep[None, None], p / kp, torch.zeros_like(p))
    o = torch.einsum("bhqk,bkhd->bqhd", p, v).reshape(B, L, H * Dh)
    o.backward(dout.double())
    return o, x.grad


def main():
    dev = torch.device("cuda")
    for L, drop in ((292, True), (292, False), (276, True), (116, True)):
        B, H, Dh = 4, 6, 64
        g = torch.Generator().manual_seed(L)
        qkv = (torch.randn((B, L, 3 * H * Dh), generator=g) * 1.5).bfloat16().to(dev)
        dout = torch.randn((B, L, H * Dh), generator=g).bfloat16().to(dev)
        st, ln, vi = octo_small_table(32, L - 36, 4)
        table, mask = K.SetTable(st, ln, vi), dense_mask(st, ln, vi, L, dev)
        kp = 0.9 if drop else 1.0
        rng = torch.tensor([3, 4], dtype=torch.int32, device=dev)
        bits = K.dropout_bits(rng, 0, 0, L, L, kp) if drop else None
        keep = bits_to_keep(bits, L).to(dev) if drop else None
        o_r, g_r = ref(qkv, H, Dh ** -0.5, mask, keep, kp, dout)
        for res in ("1", "0"):
            os.environ["MMT_ATTN_RES"] = res
            os.environ["MMT_ATTN_RES_BWD"] = res
            o, lse = K.attn_fwd(qkv, H, Dh ** -0.5, table, bits, kp)
            d = K.attn_bwd(qkv, o, dout, lse, H, Dh ** -0.5, table, bits, kp)
            eo = ((o.double() - o_r).norm() / o_r.norm()).item()
            eg = [((d.double().view(B, L, 3, -1)[:, :, i] - g_r.view(B, L, 3, -1)[:, :, i]).norm()
                   / g_r.view(B, L, 3, -1)[:, :, i].norm()).item() for i in range(3)]
            print(f"L={L} drop={drop} res={res}: o {eo:.3e}  dq {eg[0]:.3e} dk {eg[1]:.3e} dv {eg[2]:.3e}",
                  flush=True)


if __name__ == "__main__":
    main()

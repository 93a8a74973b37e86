"""Attention forward outputs (O, lse) at the step's shapes, saved for a bitwise comparison of two
builds: run once per build (MMT_LIB_AB selects the second), then --compare A.pt B.pt.
Usage: attn_fwd_bits.py OUT.pt | attn_fwd_bits.py --compare A.pt B.pt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    if sys.argv[1] == "--compare":
        a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        for k in a:
            print(k, "bit-identical" if torch.equal(a[k], b[k]) else f"DIFFERENT max {(a[k].float() - b[k].float()).abs().max().item()}")
        return
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    from tests.test_attn_norm_gpu import octo_small_table
    dev = torch.device("cuda")
    out = {}
    for L, drop in ((292, True), (228, True), (164, False), (101, True)):
        g = torch.Generator().manual_seed(L)
        B, H = 64, 6
        qkv = torch.randn((B, L, 3 * H * 64), generator=g).bfloat16().to(dev)
        starts, lens, vis = octo_small_table(min(32, L // 4), L - min(32, L // 4) - 4, 4)
        table = K.SetTable(starts, lens, vis)
        rng = torch.tensor([11, 3], dtype=torch.int32, device=dev)
        bits = K.dropout_bits(rng, 1, 0, L, L, 0.9) if drop else None
        o, lse = K.attn_fwd(qkv, H, 0.125, table, bits, 0.9 if drop else 1.0)
        torch.cuda.synchronize()
        out[f"o{L}"], out[f"lse{L}"] = o.cpu(), lse.cpu()
    torch.save(out, sys.argv[1])


if __name__ == "__main__":
    main()

"""Resident-forward debug: the K/V-resident attention forward against the streaming kernel on the
same inputs (one process, MMT_ATTN_RES toggled per call); error by 32-row query block, by head and
by 8-column group of the head dim."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K


def run(qkv, H, table, bits, kp, res):
    os.environ["MMT_ATTN_RES"] = "1" if res else "0"
    o, lse = K.attn_fwd(qkv, H, 0.125, table, bits, kp)
    torch.cuda.synchronize()
    return o.float(), lse


def main():
    dev = torch.device("cuda")
    rng = torch.tensor([77, 5], dtype=torch.int32, device=dev)
    for (B, L, masked, drop) in [(2, 292, False, False), (2, 292, True, False), (2, 292, True, True),
                                 (2, 130, False, False), (2, 64, False, False)]:
        H = 6
        g = torch.Generator().manual_seed(L)
        qkv = torch.randn((B, L, 3 * H * 64), generator=g).bfloat16().to(dev)
        table = K.SetTable([0, 32, L - 4], [32, L - 36, 4], [1, 3, 7]) if masked else None
        bits = K.dropout_bits(rng, 3, 7, L, L, 0.9) if drop else None
        kp = 0.9 if drop else 1.0
        a, la = run(qkv, H, table, bits, kp, False)
        b, lb = run(qkv, H, table, bits, kp, True)
        tot = ((a - b).norm() / a.norm()).item()
        print(f"B={B} L={L} masked={masked} drop={drop}: rel {tot:.3e}, lse max diff "
              f"{(la - lb).abs().max().item():.3e}", flush=True)
        if tot > 1e-2:
            e = (a - b).view(B, L, H, 64)
            for blk in range(0, L, 32):
                sl = e[:, blk:blk + 32]
                print(f"  rows {blk:4d}: {sl.norm().item() / a.view(B, L, H, 64)[:, blk:blk + 32].norm().item():.3e}"
                      f"  lse {(la[:, :, blk:blk + 32] - lb[:, :, blk:blk + 32]).abs().max().item():.3e}")
            print("  by head:", [round(e[:, :, h].norm().item(), 3) for h in range(H)])
            print("  by d8:", [round(e[..., 8 * c:8 * c + 8].norm().item(), 3) for c in range(8)])
            print("  by row%32:", [round(e[:, r::32].norm().item(), 2) for r in range(32)])


if __name__ == "__main__":
    main()

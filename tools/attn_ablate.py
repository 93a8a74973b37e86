"""Resident attention forward timing by feature (dropout masks, token-set mask) at B=512, L=292:
which part of the per-tile work costs the time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    B, H = 512, 6
    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    for L in (292, 116):
        g = torch.Generator().manual_seed(L)
        qkv = torch.randn((B, L, 3 * H * 64), generator=g).bfloat16().to(dev)
        masked = K.SetTable([0, 32, L - 4], [32, L - 36, 4], [1, 3, 7])
        bits = K.dropout_bits(rng, 0, 0, L, L, 0.9)
        fl = 4.0 * L * L * 64 * H * B
        for name, table, bb, kp in (("plain", None, None, 1.0), ("mask", masked, None, 1.0),
                                    ("drop", None, bits, 0.9), ("mask+drop", masked, bits, 0.9)):
            for res in ("1", "0"):
                os.environ["MMT_ATTN_RES"] = res
                us = timeit(lambda: K.attn_fwd(qkv, H, 0.125, table, bb, kp))
                print(f"L={L} {name:10s} res={res}: {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()

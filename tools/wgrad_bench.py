"""Time the OCTO-small block's four weight-gradient products (B = 512 token counts: QKV and
out-projection at L = 292, MLP Dense_0 / Dense_1 at L = 276) as the step launches them (TN
split-K kernel + combine into the fp32 gradient), at a split sized for 128 and for 256
workgroups. Run under `rocprofv3 --kernel-trace --stats` to split the GEMM from the combine.
    python tools/wgrad_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from multi_modal_transformers_tokenmerge_amd.layers import split_k_for
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    shapes = [("qkv", 1152, 384, 512 * 292), ("outproj", 384, 384, 512 * 292),
              ("dense0", 1536, 384, 512 * 276), ("dense1", 384, 1536, 512 * 276)]
    for name, M, N, Kd in shapes:
        dy = torch.randn((Kd, M), generator=g).bfloat16().to(dev)
        x = torch.randn((Kd, N), generator=g).bfloat16().to(dev)
        dw = torch.zeros((M, N), device=dev)
        for wgs in (128, 256):
            sk = split_k_for(M, N, Kd, wgs=wgs)
            us = min(timeit(lambda: K.gemm(dy, x, trans_a=True, out=dw, out_mode=K.OUT_F32_ACCUM,
                                           split_k=sk)) for _ in range(3))
            print(f"{name:8s} {M}x{N}x{Kd} split {sk:3d} ({wgs} wgs): {us:7.1f} us "
                  f"{2 * M * N * Kd / us / 1e6 / 2500:.3f} of bf16 peak", flush=True)
        del dy, x, dw


if __name__ == "__main__":
    main()

"""Time the two-stage TN weight-gradient kernel (variant 9) at the MLP Dense_0 dW shape of block 0
(B = 512: 1536 x 384 x 141,312, split-K + combine), for A/B of ablation builds via MMT_LIB_AB."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K, _C
from multi_modal_transformers_tokenmerge_amd.layers import split_k_for
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    M, N, Kd = 1536, 384, 512 * 276
    g = torch.Generator().manual_seed(0)
    dy = torch.randn((Kd, M), generator=g).bfloat16().to(dev)
    x = torch.randn((Kd, N), generator=g).bfloat16().to(dev)
    dw = torch.zeros((M, N), device=dev)
    _C.call("mmt_gemm_set_variant", 9)
    us = min(timeit(lambda: K.gemm(dy, x, trans_a=True, out=dw, out_mode=K.OUT_F32_ACCUM,
                                   split_k=split_k_for(M, N, Kd))) for _ in range(3))
    print(f"{os.environ.get('MMT_LIB_AB', 'base')}: {us:.1f} us  {2 * M * N * Kd / us / 1e6 / 2500:.3f}")


if __name__ == "__main__":
    main()

"""Micro-benchmark of libmmt_hip's attention kernels at the OCTO-small training-step shapes
(B = 256 per GPU): graph-timed fwd and bwd, TFLOP/s on dense (masked tiles counted) FLOPs:
fwd 4*L^2*Dh*H*B, bwd 10*L^2*Dh*H*B (dQ, dK, dV, dP and the recomputed S)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    B = 256
    Ls = (292, 212, 132)
    t5 = True
    H = 6
    drop = "--nodrop" not in sys.argv  # the OCTO cases without attention dropout
    for a in sys.argv[1:]:
        if a.startswith("--h="):
            H = int(a.split("=")[1])
        if a.startswith("--b="):
            B = int(a.split("=")[1])
        if a.startswith("--L="):
            Ls = tuple(int(v) for v in a.split("=")[1].split(","))
            t5 = False
    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    cases = []
    for L in Ls:  # default: layers 0, 5, 10 of the ToMe r=16 schedule
        n_img = L - 36
        cases.append((f"octo L={L}", L, H, 64,
                      K.SetTable([0, 32, 32 + n_img], [32, n_img, 4], [0b001, 0b011, 0b111]), drop, False))
    if t5:
        cases.append(("t5 L=32 (bias)", 32, 12, 64, None, False, True))
    for name, L, H, Dh, table, drop, bias in cases:
        g = torch.Generator().manual_seed(L)
        qkv = torch.randn((B, L, 3 * H * Dh), generator=g).bfloat16().to(dev)
        bits = K.dropout_bits(rng, 0, 0, L, L, 0.9) if drop else None
        bt = torch.randn((H, L, L), generator=g).to(dev) if bias else None
        o, lse = K.attn_fwd(qkv, H, Dh ** -0.5, table, bits, 0.9 if drop else 1.0, bias=bt)
        dout = torch.randn_like(o)
        dqkv = torch.empty_like(qkv)
        fl = 4.0 * L * L * Dh * H * B
        us_f = timeit(lambda: K.attn_fwd(qkv, H, Dh ** -0.5, table, bits, 0.9 if drop else 1.0,
                                         bias=bt, out=o))
        msg = f"{name:22s} B={B} H={H}: fwd {us_f:8.1f} us {fl / us_f / 1e6:7.1f} TF/s"
        if not bias:
            us_b = timeit(lambda: K.attn_bwd(qkv, o, dout, lse, H, Dh ** -0.5, table, bits,
                                             0.9 if drop else 1.0, dqkv=dqkv))
            msg += f" | bwd {us_b:8.1f} us {2.5 * fl / us_b / 1e6:7.1f} TF/s"
        print(msg, flush=True)


if __name__ == "__main__":
    main()

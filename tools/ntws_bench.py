"""A/B of the warp-specialised wide NT kernel (gemm_ntws_kernel, automatic choice) against
gemm_nt256_kernel (forced by variant 5 / 6) at the B = 512 step shapes, interleaved rounds in one
process, graph-replayed launches (tools/gemm_bench.timeit)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

os.environ.setdefault("MMT_NTWS", "2")  # the warp-specialised kernel at every shape (the A arm)
from multi_modal_transformers_tokenmerge_amd import _kernels as K, _C
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    B = int(os.environ.get("B", "512"))
    g = torch.Generator().manual_seed(0)
    rnd = lambda *s: torch.randn(s, generator=g).bfloat16().to(dev)  # noqa: E731
    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    M1, M0 = B * 276, B * 292
    y, w1, w1t = rnd(M1, 384), rnd(1536, 384), rnd(1536, 384)
    h = torch.empty((M1, 1536), dtype=torch.bfloat16, device=dev)
    bias = torch.randn(1536, generator=g).to(dev)
    bits = torch.empty((-(-M1 // 256) * 256, 1536 // 32), dtype=torch.int32, device=dev)
    dz2 = rnd(M1, 384)
    cs = torch.empty((-(-M1 // 256), 1536), dtype=torch.float32, device=dev)
    x0, wq = rnd(M0, 384), rnd(1152, 384)
    bq = torch.randn(1152, generator=g).to(dev)
    q = torch.empty((M0, 1152), dtype=torch.bfloat16, device=dev)
    cases = {
        "mlp_up (bias relu drop bits)": (2 * M1 * 1536 * 384, 5, lambda: K.gemm(
            y, w1, False, True, out=h, bias=bias, act=K.ACT_RELU, rng=rng, drop_layer=0,
            drop_site=2, keep_prob=0.9, relu_bits=bits, split_k=1)),
        "mlp_up plain": (2 * M1 * 1536 * 384, 5, lambda: K.gemm(y, w1, False, True, out=h, split_k=1)),
        "gated dX (bits colsum)": (2 * M1 * 1536 * 384, 5, lambda: K.gemm(
            dz2, w1t, False, True, out=h, gate_bits=bits, gate_scale=1 / 0.9, colsum=cs, split_k=1)),
        "qkv (bias)": (2 * M0 * 1152 * 384, 6, lambda: K.gemm(x0, wq, False, True, out=q, bias=bq,
                                                               split_k=1)),
    }
    # the frozen T5's products (B * 32 = 16,384 rows): QKV 2304 x 768 and the relu FF input
    # 3072 x 768 (arm "nt256" = variant 6 / 8: the 192-wide nt256 tiles / the narrow kernel)
    Mt = B * 32
    xt, wqt = rnd(Mt, 768), rnd(2304, 768)
    qt = torch.empty((Mt, 2304), dtype=torch.bfloat16, device=dev)
    wf = rnd(3072, 768)
    ft = torch.empty((Mt, 3072), dtype=torch.bfloat16, device=dev)
    cases["t5 qkv"] = (2 * Mt * 2304 * 768, 6, lambda: K.gemm(xt, wqt, False, True, out=qt, split_k=1))
    cases["t5 ff_in relu"] = (2 * Mt * 3072 * 768, 8, lambda: K.gemm(xt, wf, False, True, out=ft,
                                                                       act=K.ACT_RELU, split_k=1))
    res = {k: {"ws": [], "nt256": []} for k in cases}
    for rnd_i in range(3):
        for name, (fl, var, fn) in cases.items():
            for arm, v in (("ws", -1), ("nt256", var)):
                _C.call("mmt_gemm_set_variant", v)
                try:
                    res[name][arm].append(timeit(fn))
                finally:
                    _C.call("mmt_gemm_set_variant", -1)
    for name, (fl, _, _) in cases.items():
        a, b = min(res[name]["ws"]), min(res[name]["nt256"])
        print(f"{name:30s} ws {a:7.1f} us ({fl / a / 1e6 / 2500:.3f})   nt256 {b:7.1f} us "
              f"({fl / b / 1e6 / 2500:.3f})   {b / a:.2f}x", flush=True)


if __name__ == "__main__":
    main()

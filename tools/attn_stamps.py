"""Per-wave phase timeline of the resident attention backward (attn_bwd_res8_kernel) from the
stamp build (tools/build_abl.sh 9 -> libmmt_hip_abl9.so, s_memtime at: kernel start, DMA landed,
row constants written, end of the wave's phase loop, end of the bias reduction). B = 512,
L = 292, H = 6, Dh = 64, dropout 0.1 and the OCTO-small token-set mask (the step's block 0).

    MMT_LIB_AB=multi_modal_transformers_tokenmerge_amd/libmmt_hip_abl9.so python tools/attn_stamps.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from multi_modal_transformers_tokenmerge_amd import _C, _kernels as K
from tests.test_attn_norm_gpu import octo_small_table


def main():
    dev = torch.device("cuda")
    B, H, Dh = 512, 6, 64
    for L in (292, 228):
        g = torch.Generator().manual_seed(L)
        qkv = torch.randn((B, L, 3 * H * Dh), generator=g).bfloat16().to(dev)
        starts, lens, vis = octo_small_table(32, L - 36, 4)
        table = K.SetTable(starts, lens, vis)
        rng = torch.tensor([77, 5], dtype=torch.int32, device=dev)
        bits = K.dropout_bits(rng, 3, 7, L, L, 0.9)
        o, lse = K.attn_fwd(qkv, H, 0.125, table, bits, 0.9)
        dout = torch.randn((B, L, H * Dh), generator=g).bfloat16().to(dev)
        for _ in range(3):
            K.attn_bwd(qkv, o, dout, lse, H, 0.125, table, bits, 0.9)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        K.attn_bwd(qkv, o, dout, lse, H, 0.125, table, bits, 0.9)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3
        nwg = B * H
        buf = np.zeros(8192 * 8 * 6, np.uint64)
        rc = _C.lib().mmt_res8_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(buf.nbytes))
        assert rc == 0
        st = buf.reshape(8192, 8, 6)[:nwg].astype(np.int64)
        # s_memtime counters are per XCD (no common base): durations within a workgroup only,
        # converted with each XCD's own clock (its span over the kernel / the event time);
        # workgroup b ran on XCD b % 8 (round-robin dispatch)
        xcd = np.arange(nwg) % 8
        clk_x = np.zeros(8)
        for x in range(8):
            sx = st[xcd == x]
            clk_x[x] = (sx[:, :, 4].max() - sx[:, :, 0].min()) / (us * 1e3)  # cycles per ns
        clk = clk_x[xcd][:, None]
        def dur(a, b, waves=slice(None)):
            return ((st[:, waves, b] - st[:, waves, a]) / clk) / 1e3  # us
        def q(x):
            x = np.asarray(x).ravel()
            return f"median {np.median(x):7.2f} us  p10 {np.percentile(x, 10):7.2f}  p90 {np.percentile(x, 90):7.2f}"
        life = ((st[:, :, 4].max(1) - st[:, :, 0].min(1)) / clk[:, 0]) / 1e3
        print(f"L={L}: kernel {us:.1f} us (event), {nwg} workgroups, XCD clocks "
              f"{clk_x.min():.2f}-{clk_x.max():.2f} GHz (span / event time)", flush=True)
        print(f"  workgroup lifetime      {q(life)}")
        print(f"  DMA (start->landed)     {q(dur(0, 1, slice(0, 1)))}")
        print(f"  row constants           {q(dur(1, 2, slice(0, 1)))}")
        print(f"  phase A wave loop       {q(dur(2, 3, slice(0, 3)))}")
        print(f"  phase B wave loop       {q(dur(2, 3, slice(3, 8)))}")
        last = st[:, :, 3].max(1)
        print(f"  slowest wave - median   {q(((last - np.median(st[:, :, 3], 1)) / clk[:, 0]) / 1e3)}")
        print(f"  bias reduction tail     {q(((st[:, :, 4].max(1) - last) / clk[:, 0]) / 1e3)}")
        print(f"  workgroups resident per CU on average: {life.sum() / us / 256:.2f}", flush=True)


if __name__ == "__main__":
    main()

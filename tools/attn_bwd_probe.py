#!/usr/bin/env python
"""Attention backward (kinet_mha_backward) at the config-4 decoder self-attention shape: batch 2,
8 heads x 36, Lq = Lk = 540, f32.  Times the tiled kernels (default) and the wave-per-row ones
(gemm flag 512).   python tools/attn_bwd_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from kinet_amd import _native as N
    from kinet_amd import kernels as K
    B, L, H, D = 2, 540, 8, 36
    g = torch.Generator(device='cuda').manual_seed(0)
    q, k, v, do = (torch.randn(B, L, H * D, device='cuda', generator=g) for _ in range(4))
    for flags in (0, 512):
        N.lib().kinet_gemm_set_flags(flags)
        K.mha_backward(q, k, v, do, H, D ** -0.5)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            K.mha_backward(q, k, v, do, H, D ** -0.5)
        e.record()
        torch.cuda.synchronize()
        print(f'flags {flags:4d}: {s.elapsed_time(e) / 10 * 1e3:8.1f} us per backward', flush=True)
    N.lib().kinet_gemm_set_flags(0)


if __name__ == '__main__':
    main()

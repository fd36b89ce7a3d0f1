#!/usr/bin/env python
"""GEMM / implicit-conv main-loop comparison across kernel variants (diagnostic for
csrc/gemm.hip): the default selection, the 4-wave register-staged 128x128 tile, the 8-wave
LDS-DMA tiles wherever eligible (flag 2) and each 8-wave tile forced, on a
square GEMM and the ResNet conv shapes at batch B (bf16).  Every variant's output is
checked against the heuristic's.   python tools/gemm_probe.py [B]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import timeit  # noqa: E402

NO_RW = 4


def main():
    from kinet_amd import kernels as K, _native
    L = _native.lib()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    dt = torch.bfloat16
    variants = [('default', NO_RW, (0, 0)), ('nosplit', NO_RW | 64, (0, 0)), ('reg128', NO_RW, (128, 128)),
                ('8wave', NO_RW | 2, (0, 0)),
                ('dma256x128', NO_RW, (256, 128)), ('dma128x256', NO_RW, (128, 256)), ('dma256x256', NO_RW, (256, 256))]
    cases = []
    for M, N, Kd in [(4096, 4096, 4096), (B * 22223, 256, 1024), (B * 22223, 1024, 256)]:
        x = torch.randn(M, Kd, device='cuda', dtype=dt)
        w = (torch.randn(N, Kd, device='cuda') * 0.02).to(dt)
        cases.append((f'gemm {M}x{N}x{Kd}', 2 * M * N * Kd, lambda x=x, w=w: K.linear(x, w)))
    for H, W, Cin, Cout, k, s in [(100, 167, 128, 128, 3, 1), (50, 84, 256, 256, 3, 1), (25, 42, 512, 512, 3, 1),
                                  (50, 84, 1024, 512, 1, 1), (25, 42, 512, 2048, 1, 1)]:
        x = torch.randn(B, H, W, Cin, device='cuda', dtype=dt)
        wp = K.pack_conv_weight(torch.randn(Cout, Cin, k, k, device='cuda') * 0.02, dt)
        p = k // 2
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        cases.append((f'conv {H}x{W} {Cin}->{Cout} k{k}s{s}', 2 * B * Ho * Wo * Cout * k * k * Cin,
                      lambda x=x, wp=wp, s=s, p=p: K.conv2d_nhwc(x, wp, s, p)))
    for name, fl, fn in cases:
        L.kinet_gemm_set_flags(NO_RW)
        L.kinet_gemm_force_tile(0, 0)
        y0 = fn().float()
        row = []
        for vname, flags, tile in variants:
            L.kinet_gemm_set_flags(flags)
            L.kinet_gemm_force_tile(*tile)
            err = (fn().float() - y0).abs().max().item() / max(y0.abs().max().item(), 1e-6)
            t = timeit(fn, iters=10)
            row.append(f'{vname} {t * 1e3:7.1f}us {fl / t / 1e9:5.0f}TF/s{" ERR %.1e" % err if err > 0.02 else ""}')
        L.kinet_gemm_set_flags(0)
        L.kinet_gemm_force_tile(0, 0)
        print(f'{name:34s} | ' + ' | '.join(row), flush=True)


if __name__ == '__main__':
    main()

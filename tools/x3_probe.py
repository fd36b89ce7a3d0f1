#!/usr/bin/env python
"""Exact-f32 MFMA vs bf16x3 (KINET_F32_X3) on the training path's GEMM shapes: timing per call
of K.linear / K.conv2d_nhwc / K.gemm_tn at 'highest' vs 'high' float32 matmul precision.
python tools/x3_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    from kinet_amd import kernels as K
    dev = 'cuda'
    cases = []
    # FFN / projections at d=288, 2 frames of 800x1333 (S = 22223 tokens each)
    for M, N, Kd in [(44446, 1024, 288), (44446, 288, 1024), (44446, 288, 288), (1040, 288, 288)]:
        x = torch.randn(M, Kd, device=dev)
        w = torch.randn(N, Kd, device=dev) / Kd ** 0.5
        cases.append((f'linear M={M} N={N} K={Kd}', lambda x=x, w=w: K.linear(x, w), 2.0 * M * N * Kd))
    # backbone 3x3 convs (layer2 / layer3 / layer4 at 800x1333, batch 2)
    for H, W, C in [(100, 167, 128), (50, 84, 256), (25, 42, 512)]:
        x = torch.randn(2, H, W, C, device=dev)
        w = torch.randn(C, 3, 3, C, device=dev) / (9 * C) ** 0.5
        cases.append((f'conv3x3 {H}x{W}x{C}', lambda x=x, w=w: K.conv2d_nhwc(x, w, 1, 1), 2.0 * 2 * H * W * C * C * 9))
    # weight gradients: (K rows, M) x (K rows, N)
    for Kd, M, N in [(44446, 288, 1024), (44446, 288, 288), (2 * 100 * 167, 1152, 128)]:
        a = torch.randn(Kd, M, device=dev)
        b = torch.randn(Kd, N, device=dev)
        cases.append((f'gemm_tn K={Kd} M={M} N={N}', lambda a=a, b=b: K.gemm_tn(a, b), 2.0 * M * N * Kd))
    flags = int(os.environ.get('X3_FLAGS', '0'))
    tile = [int(v) for v in os.environ.get('X3_TILE', '0,0').split(',')]   # kinet_gemm_force_tile for the x3 runs
    from kinet_amd import _native as N
    for name, fn, flops in cases:
        r = {}
        for prec in ('highest', 'high'):
            torch.set_float32_matmul_precision(prec)
            N.lib().kinet_gemm_set_flags(flags)
            if prec == 'high':
                N.lib().kinet_gemm_force_tile(*tile)
            r[prec] = timeit(fn)
            N.lib().kinet_gemm_force_tile(0, 0)
            N.lib().kinet_gemm_set_flags(0)
        torch.set_float32_matmul_precision('highest')
        print(f'{name:34s} exact {r["highest"]*1e3:8.1f} us ({flops/r["highest"]/1e9:6.1f} TF/s)   '
              f'x3 {r["high"]*1e3:8.1f} us ({flops/r["high"]/1e9:6.1f} TF/s)   {r["highest"]/r["high"]:.2f}x', flush=True)


if __name__ == '__main__':
    main()

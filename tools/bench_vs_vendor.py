#!/usr/bin/env python
"""Side-by-side timing of kinet_amd's GEMM / implicit-conv kernels and the vendor libraries
(torch.matmul -> hipBLASLt, torch conv2d channels_last -> MIOpen) on the detector's shapes
at batch 8 (bf16).  Diagnostic only: the vendor numbers say what a tuned library reaches
on the same shape, nothing in the product calls them.
    python tools/bench_vs_vendor.py
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import timeit  # noqa: E402


def main():
    from kinet_amd import kernels as K
    dt = torch.bfloat16
    B = int(os.environ.get('KINET_BENCH_BATCH', '8'))
    S = B * 22223
    print(f'--- GEMM bf16 (ours | hipBLASLt), batch {B} ---')
    for M, N, Kd in [(4096, 4096, 4096), (8192, 8192, 8192), (S, 256, 1024), (S, 1024, 256), (S, 256, 256),
                     (S, 384, 256), (B * 300, 256, 256)]:
        x = torch.randn(M, Kd, device='cuda', dtype=dt)
        w = (torch.randn(N, Kd, device='cuda') * 0.02).to(dt)
        b = torch.randn(N, device='cuda')
        ours = timeit(lambda: K.linear(x, w, b))
        ref = timeit(lambda: F.linear(x, w, b.to(dt)))
        fl = 2 * M * N * Kd
        print(f'M={M:7d} N={N:5d} K={Kd:5d}: ours {ours * 1e3:8.1f} us {fl / ours / 1e9:6.0f} TF/s | '
              f'vendor {ref * 1e3:8.1f} us {fl / ref / 1e9:6.0f} TF/s')
    print(f'--- conv bf16 NHWC (ours | MIOpen channels_last), batch {B} ---')
    for H, W, Cin, Cout, k, s in [(800, 1333, 8, 64, 7, 2), (200, 334, 64, 64, 3, 1), (100, 167, 128, 128, 3, 1),
                                  (50, 84, 256, 256, 3, 1), (25, 42, 512, 512, 3, 1), (200, 334, 128, 128, 3, 2),
                                  (50, 84, 1024, 256, 1, 1), (25, 42, 2048, 512, 1, 1)]:
        x = torch.randn(B, H, W, Cin, device='cuda', dtype=dt)
        wt = torch.randn(Cout, Cin, k, k, device='cuda') * 0.02
        wp = K.pack_conv_weight(wt, dt)
        p = k // 2
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        ours = timeit(lambda: K.conv2d_nhwc(x, wp, s, p))
        xc = x.permute(0, 3, 1, 2)            # NCHW view of NHWC memory = channels_last
        wc = wt.to(dt).contiguous(memory_format=torch.channels_last)
        try:
            ref = timeit(lambda: F.conv2d(xc, wc, None, s, p))
        except RuntimeError as e:             # noqa: BLE001
            ref = float('nan')
            print('  vendor conv failed:', str(e)[:80])
        fl = 2 * B * Ho * Wo * Cout * k * k * Cin
        print(f'{H}x{W} {Cin:4d}->{Cout:4d} k{k}s{s}: ours {ours * 1e3:8.1f} us {fl / ours / 1e9:6.0f} TF/s | '
              f'vendor {ref * 1e3:8.1f} us {fl / ref / 1e9:6.0f} TF/s')


if __name__ == '__main__':
    main()

"""A/B of the implicit-GEMM conv variants on the detector's 3x3 shapes at batch 16: the launch
heuristic vs forced tiles (kinet_gemm_force_tile) and the LDS-DMA staging of the 4-wave tiles
(kinet_gemm_set_flags 16).  HIP-event timing over --iters launches; outputs checked against the
heuristic's.  python tools/conv_ab.py [--iters 20]"""
import argparse
import time
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd import _native  # noqa: E402
from kinet_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--shapes', default='', help='B,H,W,Cin,Cout,k,s;... (default: the batch-16 3x3 convs)')
    a = ap.parse_args()
    L = _native.lib()
    shapes = [(16, 200, 334, 64, 64, 3, 1), (16, 100, 167, 128, 128, 3, 1), (16, 50, 84, 256, 256, 3, 1),
              (16, 25, 42, 512, 512, 3, 1)]
    if a.shapes:
        shapes = [tuple(int(v) for v in t.split(',')) for t in a.shapes.split(';')]
    variants = [('heuristic', 0, (0, 0)), ('dma4', 16, (0, 0)), ('t128x64', 0, (128, 64)), ('t64x128', 0, (64, 128)),
                ('t128x128', 0, (128, 128)), ('t64x64', 0, (64, 64)), ('t256x128', 0, (256, 128)),
                ('dma4_128x64', 16, (128, 64)), ('dma4_128x128', 16, (128, 128)), ('t256x256', 0, (256, 256)),
                ('t128x256', 0, (128, 256)), ('tiled_only', 4, (0, 0))]
    for B, H, W, Cin, Cout, k, s in shapes:
        g = torch.Generator(device='cuda').manual_seed(0)
        x = torch.randn(B, H, W, Cin, device='cuda', dtype=torch.bfloat16, generator=g)
        wp = K.pack_conv_weight(torch.randn(Cout, Cin, k, k, device='cuda', generator=g) * 0.02, torch.bfloat16)
        p = k // 2
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        fl = 2.0 * B * Ho * Wo * Cout * k * k * Cin
        ref = None
        # warm the clocks before the first (heuristic) variant is timed: 10 launches left the first
        # variant of the first shape ~15 % slow (profiles/r06ak_conv128_tiles.txt); ~0.3 s of work
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            K.conv2d_nhwc(x, wp, s, p)
            torch.cuda.synchronize()
        for name, flags, tile in variants:
            L.kinet_gemm_set_flags(flags)
            L.kinet_gemm_force_tile(*tile)
            try:
                for _ in range(3):
                    y = K.conv2d_nhwc(x, wp, s, p)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.iters):
                    y = K.conv2d_nhwc(x, wp, s, p)
                en.record()
                torch.cuda.synchronize()
                us = st.elapsed_time(en) * 1e3 / a.iters
                yf = y.float()
                if ref is None:
                    ref = yf
                err = (yf - ref).abs().max().item() / (ref.abs().max().item() + 1e-9)
                print(f'{(B, H, W, Cin, Cout, k, s)} {name:14s} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s rel.err {err:.1e}',
                      flush=True)
            except RuntimeError as e:
                print(f'{(B, H, W, Cin, Cout, k, s)} {name:14s} n/a ({str(e)[:60]})', flush=True)
        L.kinet_gemm_set_flags(0)
        L.kinet_gemm_force_tile(0, 0)


if __name__ == '__main__':
    main()

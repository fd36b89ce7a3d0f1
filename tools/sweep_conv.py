"""Tile / split-K sweep of the implicit-GEMM conv kernel on the ResNet-50 shapes at batch B
(diagnostic for the launch heuristic in csrc/gemm.hip).  python tools/sweep_conv.py [B]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import timeit  # noqa: E402


def main():
    from kinet_amd import kernels as K, _native
    L = _native.lib()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dt = torch.bfloat16
    shapes = [(800, 1333, 8, 64, 7, 2), (200, 334, 64, 64, 3, 1), (200, 334, 128, 128, 3, 2), (100, 167, 128, 128, 3, 1),
              (100, 167, 256, 256, 3, 2), (50, 84, 256, 256, 3, 1), (50, 84, 512, 512, 3, 2), (25, 42, 512, 512, 3, 1),
              (25, 42, 2048, 256, 3, 2), (50, 84, 1024, 256, 1, 1), (100, 167, 512, 128, 1, 1), (25, 42, 512, 2048, 1, 1),
              (25, 42, 2048, 512, 1, 1), (100, 167, 512, 256, 1, 1), (50, 84, 1024, 512, 1, 1)]
    tiles = [(0, 0), (256, 128), (128, 256), (128, 128), (64, 128), (128, 64), (64, 64)]
    for H, W, Cin, Cout, k, s in shapes:
        x = torch.randn(B, H, W, Cin, device='cuda', dtype=dt)
        wp = K.pack_conv_weight(torch.randn(Cout, Cin, k, k, device='cuda') * 0.02, dt)
        p = k // 2 if k > 1 else 0
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        fl = 2 * B * Ho * Wo * Cout * k * k * Cin
        res = []
        for bm, bn in tiles:
            L.kinet_gemm_force_tile(bm, bn)
            for ks in ([None] if bm == 0 else [1] if bm == 256 or bn == 256 else [1, 2, 3, 4]):
                if ks and ks > 1 and k * k * Cin < 512:
                    continue
                try:
                    if ks == 1:   # every tile must agree with the heuristic's output
                        L.kinet_gemm_force_tile(0, 0)
                        y0 = K.conv2d_nhwc(x, wp, s, p).float()
                        L.kinet_gemm_force_tile(bm, bn)
                        err = (K.conv2d_nhwc(x, wp, s, p).float() - y0).abs().max().item()
                        assert err <= 0.02 * y0.abs().max().item(), (bm, bn, err)
                    t = timeit(lambda: K.conv2d_nhwc(x, wp, s, p, ksplit=ks), iters=10)
                except RuntimeError as e:   # noqa: BLE001
                    continue
                res.append((t, bm, bn, ks))
        L.kinet_gemm_force_tile(0, 0)
        res.sort()
        heur = [r for r in res if r[1] == 0][0]
        best = res[0]
        print(f'{H}x{W} {Cin}->{Cout} k{k}s{s}: heuristic {heur[0] * 1e3:7.1f} us ({fl / heur[0] / 1e9:4.0f} TF/s) | best '
              f'{best[1]}x{best[2]} ks={best[3]} {best[0] * 1e3:7.1f} us ({fl / best[0] / 1e9:4.0f} TF/s) | '
              + ' '.join(f'{b}x{n}/{q}:{t * 1e3:.0f}' for t, b, n, q in res[1:6]))


if __name__ == '__main__':
    main()

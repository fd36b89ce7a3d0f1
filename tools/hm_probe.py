#!/usr/bin/env python
"""The decoder's batched value projections (config 3: 2 x 177784 rows, K = 288, 6 layers x 288 =
1728 head-major columns of head_dim 36) under GEMM flag / forced-tile variants, interleaved.
python tools/hm_probe.py [--rows 177784] [--batch 2]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rows', type=int, default=177784)
    ap.add_argument('--batch', type=int, default=2)
    ap.add_argument('--iters', type=int, default=10)
    a = ap.parse_args()
    from kinet_amd import kernels as K
    from kinet_amd import _native as N
    L = N.lib()
    x = torch.randn(a.batch, a.rows, 288, device='cuda', dtype=torch.float16)
    w = torch.randn(1728, 288, device='cuda', dtype=torch.float16) / 17
    b = torch.randn(1728, device='cuda')
    variants = [('rw (default)', 0, (0, 0)), ('tiled heuristic', 4, (0, 0)), ('tiled 128x128', 4, (128, 128)),
                ('tiled 64x128', 4, (64, 128)), ('tiled 128x64', 4, (128, 64)), ('row-major rw', 0, None)]
    ref = None
    nbytes = (a.batch * a.rows * (288 + 1728) + 1728 * 288) * 2
    for rep in range(2):
        for name, fl, tile in variants:
            L.kinet_gemm_set_flags(fl)
            L.kinet_gemm_force_tile(*(tile or (0, 0)))
            if tile is None:   # the same GEMM, row-major (B*S, 1728) output
                fn = lambda: K.linear(x, w, b)
            else:
                fn = lambda: K.value_proj_headmajor(x, w, b, 36)
            y = fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / a.iters * 1e3
            L.kinet_gemm_force_tile(0, 0)
            L.kinet_gemm_set_flags(0)
            if tile is None:
                y = y.view(a.batch, a.rows, 48, 36).permute(2, 0, 1, 3)
            same = 'ref' if ref is None else ('bit-identical' if torch.equal(ref, y) else
                                              'max diff %.3g' % (ref.float() - y.float()).abs().max().item())
            ref = y if ref is None else ref
            print(f'{name:18s} {us:8.1f} us {nbytes / us / 1e3:6.0f} GB/s {same}', flush=True)


if __name__ == '__main__':
    main()

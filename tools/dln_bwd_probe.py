#!/usr/bin/env python
"""Time kinet_dropout_add_layernorm_backward at the config-4 encoder rows (2 x 22223 x 288, f32,
p = 0.1): python tools/dln_bwd_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from kinet_amd import kernels as K
    x, r, dy = (torch.randn(2, 22223, 288, device='cuda') for _ in range(3))
    g = torch.rand(288, device='cuda') + 0.5
    seed = torch.tensor([1234], dtype=torch.int64, device='cuda')
    fn = lambda: K.dropout_add_layernorm_backward(dy, x, r, g, 1e-5, 0.1, seed)
    fn()
    torch.cuda.synchronize()
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        print(f'dropout_add_layernorm_backward 2 x 22223 x 288: {us:7.1f} us '
              f'({5 * x.numel() * 4 / us / 1e3:6.0f} GB/s: dy, x, r in; dx, dr out)', flush=True)


if __name__ == '__main__':
    main()

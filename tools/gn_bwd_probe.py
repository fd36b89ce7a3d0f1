#!/usr/bin/env python
"""Time kinet_groupnorm_backward at the config-4 input-projection shapes (2 frames, d = 288,
32 groups, f32): python tools/gn_bwd_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from kinet_amd import kernels as K
    for hw in (16700, 4200, 1050, 273):
        x = torch.randn(2, hw, 288, device='cuda')
        dy = torch.randn(2, hw, 288, device='cuda')
        g = torch.rand(288, device='cuda') + 0.5
        fn = lambda: K.groupnorm_backward(dy, x, g, 32, 1e-5)
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        nbytes = 3 * x.numel() * 4
        print(f'groupnorm_backward 2 x {hw} x 288 f32: {us:7.1f} us ({nbytes / us / 1e3:6.0f} GB/s, x + dy + dx)', flush=True)


if __name__ == '__main__':
    main()

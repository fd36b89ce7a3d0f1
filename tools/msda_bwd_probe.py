#!/usr/bin/env python
"""MSDA backward (kinet_msda_backward, csrc/msda.hip msda_bwd_kernel) at the config-4 training
shapes: encoder call of 2 frames at 800x1333 (levels 100x167, 50x84, 25x42, 13x21; Lq = S =
22,223), 8 heads x 36 channels, 4 levels x 4 points, f32; and the decoder call (Lq = 500 + track
queries, 8 levels of the two frames).  Sampling pattern of the reference init (8-direction grid
offsets) + noise.  Times the backward call.   python tools/msda_bwd_probe.py [--iters 10]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def inputs(B, shapes, Lq, M=8, D=36, P=4, seed=0, decoder=False):
    g = torch.Generator(device='cuda').manual_seed(seed)
    L = len(shapes)
    S = sum(h * w for h, w in shapes)
    ss = torch.tensor(shapes, dtype=torch.int64, device='cuda')
    value = torch.randn(B, S, M, D, device='cuda', generator=g)
    ref = torch.rand(B, Lq, 1, 1, 1, 2, device='cuda', generator=g)
    th = torch.arange(M, device='cuda', dtype=torch.float32) * (2 * math.pi / M)
    grid = torch.stack([th.cos(), th.sin()], -1)[:, None, None, :] * (torch.arange(P, device='cuda') + 1.0)[None, None, :, None]
    wh = torch.tensor([[w, h] for h, w in shapes], device='cuda', dtype=torch.float32)[None, :, None, :]
    off = (grid + 0.5 * torch.randn(B, Lq, M, L, P, 2, device='cuda', generator=g)) / wh
    loc = (ref + off).contiguous()
    attw = torch.softmax(torch.randn(B, Lq, M, L * P, device='cuda', generator=g), -1).view(B, Lq, M, L, P).contiguous()
    gout = torch.randn(B, Lq, M * D, device='cuda', generator=g)
    return value, ss, loc, attw, gout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=10)
    a = ap.parse_args()
    from kinet_amd.MultiScaleDeformableAttention import ms_deform_attn_backward
    lv = [(100, 167), (50, 84), (25, 42), (13, 21)]
    cases = {'encoder': (2, lv, 22223), 'decoder': (2, lv + lv, 520)}
    for name, (B, shapes, Lq) in cases.items():
        v, ss, loc, attw, gout = inputs(B, shapes, Lq)
        ms_deform_attn_backward(v, ss, loc, attw, gout, 64)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            ms_deform_attn_backward(v, ss, loc, attw, gout, 64)
        e.record()
        torch.cuda.synchronize()
        print(f'{name:8s}: {s.elapsed_time(e) / a.iters:8.3f} ms', flush=True)


if __name__ == '__main__':
    main()

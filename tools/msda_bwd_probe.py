#!/usr/bin/env python
"""MSDA backward (kinet_msda_backward, csrc/msda.hip) at the config-4 training shapes: encoder
call of 2 frames at 800x1333 (levels 100x167, 50x84, 25x42, 13x21; Lq = S = 22,223), 8 heads x
36 channels, 4 levels x 4 points, f32; and the decoder call (Lq = 500 + track queries, 8 levels
of the two frames).  Encoder queries are the level pixels in raster order with their pixel
centres as reference points (deformable_transformer.py get_reference_points); decoder queries
have random reference points.  Offsets: the reference init (8-direction grid, point i at
radius i+1 pixels) + N(0, noise) pixels.  Times the direct-atomic kernel (tune mode -1) and the
LDS-table kernel at the given table shapes, and checks they agree.

    python tools/msda_bwd_probe.py [--iters 10] [--noise 0.5] [--sweep] [--phases] [--ab FLAGS]

--ab FLAGS: the default kernel vs the one kinet_msda_backward_debug(FLAGS) selects (result-valid
variants: 16 = DPP row sums in phase 2), interleaved 4 times, with the max difference.

--phases: the on-chip-sum kernel with each timing-only phase knob (kinet_msda_backward_debug:
1 no value loads in the location / weight gradients, 2 no row atomics, 4 no row-sum phase,
8 no hash inserts) -- where the time goes.
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def inputs(B, shapes, Lq, M=8, D=36, P=4, seed=0, encoder=True, noise=0.5):
    g = torch.Generator(device='cuda').manual_seed(seed)
    L = len(shapes)
    S = sum(h * w for h, w in shapes)
    ss = torch.tensor(shapes, dtype=torch.int64, device='cuda')
    value = torch.randn(B, S, M, D, device='cuda', generator=g)
    if encoder:
        refs = []
        for h, w in shapes:
            y, x = torch.meshgrid(torch.arange(h, device='cuda') + 0.5, torch.arange(w, device='cuda') + 0.5, indexing='ij')
            refs.append(torch.stack([x.reshape(-1) / w, y.reshape(-1) / h], -1))
        ref = torch.cat(refs)[None, :, None, None, None, :].expand(B, Lq, 1, 1, 1, 2)
    else:
        ref = torch.rand(B, Lq, 1, 1, 1, 2, device='cuda', generator=g)
    th = torch.arange(M, device='cuda', dtype=torch.float32) * (2 * math.pi / M)
    grid = torch.stack([th.cos(), th.sin()], -1)[:, None, None, :] * (torch.arange(P, device='cuda') + 1.0)[None, None, :, None]
    wh = torch.tensor([[w, h] for h, w in shapes], device='cuda', dtype=torch.float32)[None, :, None, :]
    off = (grid + noise * torch.randn(B, Lq, M, L, P, 2, device='cuda', generator=g)) / wh
    loc = (ref + off).contiguous()
    attw = torch.softmax(torch.randn(B, Lq, M, L * P, device='cuda', generator=g), -1).view(B, Lq, M, L, P).contiguous()
    gout = torch.randn(B, Lq, M * D, device='cuda', generator=g)
    return value, ss, loc, attw, gout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--noise', type=float, default=0.5)
    ap.add_argument('--sweep', action='store_true')
    ap.add_argument('--case', default='encoder,decoder')
    ap.add_argument('--phases', action='store_true')
    ap.add_argument('--ab', type=int, default=0)
    a = ap.parse_args()
    from kinet_amd import _native
    from kinet_amd.MultiScaleDeformableAttention import ms_deform_attn_backward
    tune = _native.lib().kinet_msda_backward_tune
    dbg = _native.lib().kinet_msda_backward_debug
    lv = [(100, 167), (50, 84), (25, 42), (13, 21)]
    cases = {'encoder': (2, lv, 22223, True), 'decoder': (2, lv + lv, 520, False)}
    # (mode, log2 hash rows, queries per block, threads, queries per pass)
    cfgs = [(-1, 0, 0, 0, 0), (0, 0, 0, 0, 0), (2, 0, 0, 0, 0), (3, 0, 0, 0, 0), (4, 0, 0, 0, 0)]
    if a.sweep:
        cfgs += [(0, l2, 0, th, qp) for l2 in (9, 10, 11) for th in (256, 512) for qp in (16, 32, 64)
                 if qp >= th // 32]
    for name, (B, shapes, Lq, enc) in cases.items():
        if name not in a.case.split(','):
            continue
        v, ss, loc, attw, gout = inputs(B, shapes, Lq, encoder=enc, noise=a.noise)
        ref = None
        runs = [(c, 0) for c in cfgs]
        if a.phases:
            runs += [((0, 0, 0, 0, 0), f) for f in (1, 2, 4, 8, 1 | 4, 1 | 8)]
        if a.ab:
            for rep in range(4):
                outs = []
                for flags in (0, a.ab):
                    dbg(flags)
                    out = ms_deform_attn_backward(v, ss, loc, attw, gout, 64)
                    torch.cuda.synchronize()
                    outs.append([t.clone() for t in out])
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.iters):
                        ms_deform_attn_backward(v, ss, loc, attw, gout, 64)
                    e.record()
                    torch.cuda.synchronize()
                    print(f'{name:8s} rep {rep} flags {flags}: {s.elapsed_time(e) / a.iters:8.3f} ms', flush=True)
                dbg(0)
                err = max(((o - r).abs().max() / r.abs().max().clamp_min(1e-30)).item() for o, r in zip(*outs))
                print(f'{name:8s} rep {rep} max rel diff {err:.2e}', flush=True)
            continue
        for cfg, flags in runs:
            tune(*cfg)
            dbg(flags)
            try:
                out = ms_deform_attn_backward(v, ss, loc, attw, gout, 64)
            except RuntimeError as ex:
                print(f'{name:8s} cfg {cfg}: {ex}', flush=True)
                continue
            torch.cuda.synchronize()
            if flags:
                pass
            elif ref is None:
                ref = [t.clone() for t in out]
                err = 0.0
            else:
                err = max(((o - r).abs().max() / r.abs().max().clamp_min(1e-30)).item() for o, r in zip(out, ref))
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                ms_deform_attn_backward(v, ss, loc, attw, gout, 64)
            e.record()
            torch.cuda.synchronize()
            dbg(0)
            if flags:
                print(f'{name:8s} noise {a.noise} cfg {cfg} phase knob {flags}: {s.elapsed_time(e) / a.iters:8.3f} ms',
                      flush=True)
                continue
            print(f'{name:8s} noise {a.noise} cfg {cfg}: {s.elapsed_time(e) / a.iters:8.3f} ms  '
                  f'max rel diff vs direct {err:.2e}', flush=True)
    tune(0, 0, 0, 0, 0)


if __name__ == '__main__':
    main()

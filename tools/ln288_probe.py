#!/usr/bin/env python
"""A/B of the K = 288 resident-weight GEMM with the fused residual + LayerNorm epilogue (the
encoder's output projection + norm1 and the FFN-less LN GEMMs of configs 3-5): per-call time at
the config-3 shape under GEMM flag sets given on the command line, interleaved.
python tools/ln288_probe.py [--m 177784] [--flags 0,4194304] [--reps 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--m', type=int, default=177784)
    ap.add_argument('--flags', default='0,4194304')
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--kind', default='ln', choices=['ln', 'split'],
                    help='ln: output projection + residual + LayerNorm; split: the head_dim-36 value projection')
    args = ap.parse_args()
    from kinet_amd import kernels as K
    from kinet_amd import _native as N
    dt = torch.float16
    M, D = args.m, 288
    x = torch.randn(M, D, device='cuda', dtype=dt)
    r = torch.randn(M, D, device='cuda', dtype=dt)
    w = torch.randn(D, D, device='cuda') / D ** 0.5
    b = torch.randn(D, device='cuda') * 0.1
    g = torch.rand(D, device='cuda') + 0.5
    be = torch.randn(D, device='cuda') * 0.1
    flags = [int(f) for f in args.flags.split(',')]
    if args.kind == 'split':
        ws, bs = K.split_value_weights(w.to(dt), b, 8)

        def call():
            return K.value_proj_headmajor_split(x.view(2, M // 2, D), ws, bs, 8)

        def flat(sv):
            return torch.cat([sv.main.reshape(-1), sv.tail.reshape(-1)])
        nbytes = 2 * M * D * 2
    else:
        call = lambda: K.linear(x, w, b, residual=r, ln=(g, be, 1e-5))
        flat = lambda y: y
        nbytes = 3 * M * D * 2
    outs = {}
    for f in flags:
        N.lib().kinet_gemm_set_flags(f)
        outs[f] = flat(call())
    N.lib().kinet_gemm_set_flags(0)
    torch.cuda.synchronize()
    for f in flags[1:]:
        d = (outs[f].float() - outs[flags[0]].float()).abs().max().item()
        print(f'flags {f}: max |diff| vs flags {flags[0]} = {d:.3g}', flush=True)
    for rep in range(args.reps):
        line = []
        for f in flags:
            N.lib().kinet_gemm_set_flags(f)
            fn = call
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / args.iters * 1e3
            line.append(f'flags {f}: {us:7.1f} us ({nbytes / us / 1e3:6.0f} GB/s)')
        N.lib().kinet_gemm_set_flags(0)
        print(f'rep {rep}: ' + '   '.join(line), flush=True)


if __name__ == '__main__':
    main()

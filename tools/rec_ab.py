"""A/B of the encoder MSDA call at config 2 (800x1333, batch 16): the round-3 pipeline (offsets /
logits projection GEMM -> f16 head-major offsets + logits -> kinet_msda_encoder_forward) against
the sampling-records pipeline (kinet_msda_sample_records -> kinet_msda_encoder_forward_records).
Times each kernel alone (HIP events, interleaved repeats) and prints the max output difference.

usage: python tools/rec_ab.py [--batch 16] [--iters 30] [--reps 3] [--rec-flags 0]
(--rec-flags: time the records GEMM alone under each kinet_gemm_set_flags value, interleaved)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kinet_amd import kernels as K  # noqa: E402
from kinet_amd.msda import MSDeformAttn  # noqa: E402


def time_call(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--iters', type=int, default=30)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--rec-flags', default='')
    a = ap.parse_args()
    shapes = [(100, 167), (50, 84), (25, 42), (13, 21)]
    B, S = a.batch, sum(h * w for h, w in shapes)
    torch.manual_seed(0)
    attn = MSDeformAttn(256, 4, 8, 4).cuda()
    with torch.no_grad():   # reference init (grid offsets in the bias) + trained-like spread
        attn.sampling_offsets.weight.normal_(0, 0.01)
        attn.attention_weights.weight.normal_(0, 0.02)
    src = torch.randn(B, S, 256, device='cuda').bfloat16()
    pos = torch.randn(B, S, 256, device='cuda').bfloat16()
    pts = []
    for h, w in shapes:
        yy, xx = torch.meshgrid(torch.arange(h, dtype=torch.float32) + 0.5, torch.arange(w, dtype=torch.float32) + 0.5,
                                indexing='ij')
        pts.append(torch.stack([xx.reshape(-1) / w, yy.reshape(-1) / h], -1))
    ref = torch.cat(pts, 0)[None, :, None, :].expand(B, -1, 4, -1).contiguous().cuda()
    order = K.encoder_tile_order(shapes, 'cuda')
    with torch.no_grad():
        value = attn.project_value(src)
        w_hm, b_hm = attn.packed_offsets_weights_headmajor()
        w_rec, b_rec = attn.packed_records_weights()
        state = {}

        def proj_old():
            state['hm'] = K.offsets_proj_headmajor(src, w_hm, b_hm, 8, x_add=pos)

        def samp_old():
            state['o_old'] = K.msda_encoder(value, shapes, state['hm'], ref, 8, out_dtype=torch.bfloat16,
                                            query_tile_order=order)

        def proj_rec():
            state['rec'], state['fb'] = K.msda_sample_records(src, w_rec, b_rec, 8, ref, shapes, x_add=pos)

        def samp_rec():
            state['o_rec'] = K.msda_encoder_records(value, shapes, state['rec'], state['fb'],
                                                    out_dtype=torch.bfloat16, query_tile_order=order)
        for f in (proj_old, samp_old, proj_rec, samp_rec):
            f()
        time_call(samp_old, 100)   # clocks up
        for r in range(a.reps):
            t = [time_call(f, a.iters) * 1e3 for f in (proj_old, samp_old, proj_rec, samp_rec)]
            print(f'rep {r}: offlog GEMM {t[0]:.1f} us + sampler {t[1]:.1f} us = {t[0] + t[1]:.1f} | '
                  f'records GEMM {t[2]:.1f} us + sampler {t[3]:.1f} us = {t[2] + t[3]:.1f}  (B={B})', flush=True)
        if a.rec_flags:
            from kinet_amd import _native
            flags = [int(f) for f in a.rec_flags.split(',')]
            for r in range(a.reps):
                t = []
                for f in flags:
                    _native.lib().kinet_gemm_set_flags(f)
                    t.append(time_call(proj_rec, a.iters) * 1e3)
                _native.lib().kinet_gemm_set_flags(0)
                print(f'rep {r}: records GEMM ' + ' | '.join(f'flags {f}: {x:.1f} us' for f, x in zip(flags, t)),
                      flush=True)
        d = (state['o_old'].float() - state['o_rec'].float()).abs()
        print(f'max |old - records| {d.max().item():.4g}  mean {d.mean().item():.3g}  '
              f'max |old| {state["o_old"].float().abs().max().item():.3g}')


if __name__ == '__main__':
    main()

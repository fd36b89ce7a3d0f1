"""Microbenchmark of the fused MSDA sampling kernel at the config2 encoder shape
(4 frames of 800x1333: levels 100x167, 50x84, 25x42, 13x21; 8 heads x 32 channels;
4 levels x 4 points), with the sampling pattern the bench workload has (reference init:
sampling_offsets.weight = 0, bias = the 8-direction grid, ms_deform_attn.py:34-47) plus
optional noise.  Prints the average time per call (HIP events over `iters` calls).

usage: python tools/bench_msda.py [--noise PIXELS] [--iters N] [--decoder]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kinet_amd import kernels as K  # noqa: E402


def make_inputs(B=4, shapes=((100, 167), (50, 84), (25, 42), (13, 21)), M=8, D=32, P=4, noise=0.0,
                decoder=False, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device='cuda').manual_seed(seed)
    L = len(shapes)
    S = sum(h * w for h, w in shapes)
    ss = torch.tensor(shapes, dtype=torch.int64, device='cuda')
    value = torch.randn(M, B, S, D, device='cuda', generator=g).to(dtype)
    if decoder:
        Lq = 300
        ref = torch.rand(B, Lq, L, 2, device='cuda', generator=g)
    else:
        Lq = S
        refs = []
        for h, w in shapes:
            ys, xs = torch.meshgrid(torch.arange(h, device='cuda') + 0.5, torch.arange(w, device='cuda') + 0.5,
                                    indexing='ij')
            refs.append(torch.stack([xs.reshape(-1) / w, ys.reshape(-1) / h], -1))
        ref = torch.cat(refs, 0)[None, :, None, :].expand(B, Lq, L, 2).contiguous()
    thetas = torch.arange(M, dtype=torch.float32) * (2.0 * math.pi / M)
    grid = torch.stack([thetas.cos(), thetas.sin()], -1)
    grid = grid / grid.abs().max(-1, keepdim=True)[0]
    grid = grid.view(M, 1, 1, 2).repeat(1, L, P, 1)
    for i in range(P):
        grid[:, :, i, :] *= i + 1
    off = grid.reshape(1, 1, -1).to('cuda').expand(B, Lq, -1).clone()
    if noise:
        off += noise * torch.randn(off.shape, device='cuda', generator=g)
    logits = 0.1 * torch.randn(B, Lq, M * L * P, device='cuda', generator=g)
    offlog = torch.cat([off, logits], -1).contiguous()
    return value, ss, offlog, ref, (M, L, P)


def time_call(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--noise', type=float, default=0.0)
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--decoder', action='store_true')
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--order', action='store_true', help='encoder tile order (kernels.encoder_tile_order)')
    ap.add_argument('--hm', action='store_true',
                    help='encoder kernel on head-major offsets/logits (kinet_msda_encoder_forward)')
    ap.add_argument('--rec', action='store_true',
                    help='encoder kernel on sampling records (kinet_msda_encoder_forward_records); the records are '
                         'made once by kinet_msda_sample_records from an identity-like projection of the offsets')
    a = ap.parse_args()
    if os.environ.get('KINET_ENC_STRIPS'):   # encoder strips per head map (kinet_msda_encoder_set_strips)
        from kinet_amd import _native
        _native.lib().kinet_msda_encoder_set_strips(int(os.environ['KINET_ENC_STRIPS']))
    value, ss, offlog, ref, (M, L, P) = make_inputs(B=a.batch, noise=a.noise, decoder=a.decoder,
                                                    dtype=torch.float16)
    offlog = offlog.half()
    order = K.encoder_tile_order(ss.tolist(), value.device) if a.order and not a.decoder else None
    fn = lambda: K.msda_fused(value, ss, offlog, ref, M, L, P, head_major=True, out_dtype=torch.bfloat16,   # noqa: E731
                              query_tile_order=order)
    kind = 'fused'
    if a.hm and not a.decoder:
        B_, Lq_ = offlog.shape[:2]
        hm = torch.cat([offlog[..., :M * L * P * 2].reshape(B_, Lq_, M, -1),
                        offlog[..., M * L * P * 2:].reshape(B_, Lq_, M, -1)], -1).permute(2, 0, 1, 3).contiguous()
        shapes = [tuple(s) for s in ss.tolist()]
        fn = lambda: K.msda_encoder(value, shapes, hm, ref, M, out_dtype=torch.bfloat16,   # noqa: E731
                                    query_tile_order=order)
        kind = 'encoder-hm'
    if a.rec and not a.decoder:
        # records from an encoder projection with the reference init (sampling_offsets.bias = the
        # 8-direction grid, ms_deform_attn.py:34-47) plus a small random weight: the sampling
        # pattern of the bench workload (grid + spread), written by kinet_msda_sample_records
        from kinet_amd.msda import MSDeformAttn
        B_, Lq_ = offlog.shape[:2]
        torch.manual_seed(0)
        attn = MSDeformAttn(256, L, M, P).cuda()
        with torch.no_grad():
            attn.sampling_offsets.weight.normal_(0, 0.01 + 0.01 * a.noise)
            attn.attention_weights.weight.normal_(0, 0.02)
            w, bias = attn.packed_records_weights()
            x = torch.randn(B_, Lq_, 256, device='cuda').half()
            shapes = [tuple(s) for s in ss.tolist()]
            rec, fb = K.msda_sample_records(x, w, bias, M, ref, shapes)
        fn = lambda: K.msda_encoder_records(value, shapes, rec, fb, out_dtype=torch.bfloat16,   # noqa: E731
                                            query_tile_order=order)
        kind = 'encoder-records'
    ms = time_call(fn, a.iters)
    B, Lq = offlog.shape[:2]
    S = value.shape[2]
    nsamp = B * Lq * M * L * P
    gathered = nsamp * 4 * value.shape[-1] * value.element_size()
    compulsory = value.numel() * value.element_size() + offlog.numel() * offlog.element_size() + ref.numel() * 4 + \
        B * Lq * M * value.shape[-1] * value.element_size()
    print(f'[{kind}] msda {"decoder" if a.decoder else "encoder"} B={B} Lq={Lq} S={S} noise={a.noise}: {ms * 1e3:.1f} us/call  '
          f'compulsory {compulsory / ms / 1e6:.0f} GB/s  gathered {gathered / ms / 1e6:.0f} GB/s')


if __name__ == '__main__':
    main()

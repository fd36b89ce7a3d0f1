"""A/B of the encoder sampling kernel: kinet_msda_encoder_forward of the in-tree library against
the same entry point of another build (e.g. the previous commit's msda_enc.hip compiled alone
into tools/ab/libenc_old.so), on bench_msda.py's config-2 encoder inputs.  Prints us/call of
both (HIP events, interleaved repeats) and the max output difference.

usage: python tools/enc_ab.py [--lib tools/ab/libenc_old.so] [--batch 16] [--noise 0] [--iters 30]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kinet_amd import _native as N  # noqa: E402
from kinet_amd import kernels as K  # noqa: E402
from tools.bench_msda import make_inputs, time_call  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', action='append', default=None,
                    help='other build(s) to time (repeatable; default tools/ab/libenc_old.so)')
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--noise', type=float, default=0.0)
    ap.add_argument('--iters', type=int, default=30)
    ap.add_argument('--reps', type=int, default=3)
    a = ap.parse_args()
    value, ss, offlog, ref, (M, L, P) = make_inputs(B=a.batch, noise=a.noise, dtype=torch.float16)
    offlog = offlog.half()
    B, Lq = offlog.shape[:2]
    S = value.shape[2]
    hm = torch.cat([offlog[..., :M * L * P * 2].reshape(B, Lq, M, -1),
                    offlog[..., M * L * P * 2:].reshape(B, Lq, M, -1)], -1).permute(2, 0, 1, 3).contiguous()
    shapes = [tuple(s) for s in ss.tolist()]
    order = K.encoder_tile_order(shapes, value.device)
    hs = torch.tensor(shapes, dtype=torch.int64)
    libs = a.lib or [os.path.join(os.path.dirname(os.path.abspath(__file__)), 'ab', 'libenc_old.so')]
    out_o = torch.empty((B, Lq, M * 32), dtype=torch.bfloat16, device=value.device)

    def runner(path):
        fn_o = ctypes.CDLL(path).kinet_msda_encoder_forward
        fn_o.argtypes = N._SIGS['kinet_msda_encoder_forward']

        def run_other():
            rc = fn_o(N.ptr(value), value.stride(1), value.stride(0), N.ptr(hs), N.ptr(hm), N.ptr(ref), ref.shape[-1],
                      None, N.ptr(out_o), B, S, M, 32, 4, Lq, 4, N.dtype_code(torch.bfloat16), N.ptr(order),
                      N.stream(value.device))
            assert rc == 0, rc
        return run_other
    others = [(os.path.basename(p), runner(p)) for p in libs]

    def run_new():
        return K.msda_encoder(value, shapes, hm, ref, M, out_dtype=torch.bfloat16, query_tile_order=order)

    print('plan (fl, nstrip, used, wgs):', K.msda_encoder_plan(shapes, B, M, Lq))
    time_call(run_new, 200)   # clocks up
    for r in range(a.reps):
        line = f'rep {r}: in-tree {time_call(run_new, a.iters) * 1e3:.1f} us'
        for name, fn in others:
            line += f'  {name} {time_call(fn, a.iters) * 1e3:.1f} us'
        print(line + f'  (B={B} noise={a.noise})')
    o_new = run_new()
    for name, fn in others:
        fn()
        torch.cuda.synchronize()
        d = (o_new.float() - out_o.float()).abs()
        print(f'{name}: max |in-tree - it| {d.max().item():.4g}  mean {d.mean().item():.3g}')


if __name__ == '__main__':
    main()

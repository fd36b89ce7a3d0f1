"""Debug aid: the records GEMM (kinet_msda_sample_records) against oracle.sample_records on one
test problem; prints the samples whose decoded locations differ by more than 1 LSB, with the
f64 pixel coordinates of both.  python tools/rec_debug.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))

from kinet_amd import kernels as K  # noqa: E402
from oracle import msda_oracle as O  # noqa: E402
from test_msda_gpu import _host_offlog, _record_problem  # noqa: E402


def main():
    shapes = ((100, 167), (50, 84), (25, 42), (13, 21))
    B, M = 2, 8
    x, pos, w, bias, ref, qmask, raw = _record_problem(shapes, B, 2.0, 43, 2, False)
    rec, fb = K.msda_sample_records(x.cuda(), w.cuda(), bias.cuda(), M, ref.cuda(), shapes, x_add=pos.cuda())
    torch.cuda.synchronize()
    offlog = _host_offlog(x, pos, *raw, torch.bfloat16)
    loc, aw = O.prep(offlog, ref.double(), shapes, None, M, 4, 4)
    exp = O.sample_records(loc, aw, ref, shapes, fb)
    got = rec.cpu()
    l_g, a_g = O.decode_records(got, shapes, fb)
    l_e, a_e = O.decode_records(exp, shapes, fb)
    H = torch.tensor([h for h, _ in shapes], dtype=torch.float64)[None, None, None, :, None]
    W = torch.tensor([w_ for _, w_ in shapes], dtype=torch.float64)[None, None, None, :, None]
    dy = ((l_g[..., 1] - l_e[..., 1]) * H).abs()
    dx = ((l_g[..., 0] - l_e[..., 0]) * W).abs()
    bad = (dy > 1.01 * 2.0 ** -fb) | (dx > 1.01 * 2.0 ** -fb)
    print('bad fraction', bad.double().mean().item(), 'count', int(bad.sum()))
    idx = bad.nonzero()[:40]
    hx = loc[..., 1] * H - 0.5
    wx = loc[..., 0] * W - 0.5
    for b, q, m, l, p in idx.tolist():
        print(f'b{b} q{q} m{m} l{l} p{p}: exact h {hx[b, q, m, l, p]:.5f} w {wx[b, q, m, l, p]:.5f} | '
              f'gpu h {l_g[b, q, m, l, p, 1] * H[0, 0, 0, l, 0] - 0.5:.5f} w {l_g[b, q, m, l, p, 0] * W[0, 0, 0, l, 0] - 0.5:.5f} '
              f'a {a_g[b, q, m, l, p]:.4f} | oracle h {l_e[b, q, m, l, p, 1] * H[0, 0, 0, l, 0] - 0.5:.5f} '
              f'w {l_e[b, q, m, l, p, 0] * W[0, 0, 0, l, 0] - 0.5:.5f} a {a_e[b, q, m, l, p]:.4f}  '
              f'raw gpu {int(got[m, b, q, l * 4 + p]) & 0xffffffff:08x} oracle {int(exp[m, b, q, l * 4 + p]) & 0xffffffff:08x}')
    # where in the query range
    qs = idx[:, 1]
    print('bad query range', qs.min().item() if len(qs) else None, qs.max().item() if len(qs) else None)


if __name__ == '__main__':
    main()

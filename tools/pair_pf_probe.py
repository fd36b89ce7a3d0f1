"""Fused bottleneck pair (kinet_bottleneck_pair) with its weight fragments read further ahead
(kinet_ffn_set_debug 2048 = PF 1, 4096 = PF 2) vs the default, on the config-2 batch-28 stage
shapes: HIP-event time per call, interleaved repeats, outputs compared bit for bit.
usage: python tools/pair_pf_probe.py [--iters 20] [--reps 3] [--knobs 0,2048,4096]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd import _native  # noqa: E402
from kinet_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--iters', type=int, default=20)
ap.add_argument('--reps', type=int, default=3)
ap.add_argument('--knobs', default='0,2048,4096')
ap.add_argument('--shapes', default='128:467600,256:117600,256:32640,128:129600')
a = ap.parse_args()
L = _native.lib()
for sh in a.shapes.split(','):
    D, M = (int(v) for v in sh.split(':'))
    F_ = 4 * D
    g = torch.Generator().manual_seed(D + M)
    x = torch.relu(torch.randn(M, 1, 1, D, generator=g)).bfloat16().cuda()
    res = torch.randn(M, 1, 1, F_, generator=g).bfloat16().cuda()
    w3 = (torch.randn(F_, D, 1, 1, generator=g) * (2.0 / D) ** 0.5).cuda()
    w1 = (torch.randn(D, F_, 1, 1, generator=g) * (2.0 / F_) ** 0.5).cuda()
    s3, b3 = (torch.rand(F_, generator=g) + 0.5).cuda(), (torch.randn(F_, generator=g) * 0.1).cuda()
    s1, b1 = (torch.rand(D, generator=g) + 0.5).cuda(), (torch.randn(D, generator=g) * 0.1).cuda()
    packed = K.bottleneck_pack(w3, w1, s3, s1, torch.bfloat16)
    ref = None
    for _ in range(10):
        K.bottleneck_pair(x, res, packed, b3, b1)
    for r in range(a.reps):
        for knob in (int(k) for k in a.knobs.split(',')):
            old = L.kinet_ffn_set_debug(knob)
            try:
                y, t = K.bottleneck_pair(x, res, packed, b3, b1)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.iters):
                    K.bottleneck_pair(x, res, packed, b3, b1)
                en.record()
                torch.cuda.synchronize()
            finally:
                L.kinet_ffn_set_debug(old)
            us = st.elapsed_time(en) * 1e3 / a.iters
            if ref is None:
                ref = (y.clone(), t.clone())
            same = torch.equal(ref[0], y) and torch.equal(ref[1], t)
            print(f'pair D={D} M={M} knob {knob:5d}: {us:7.1f} us  {"bit-identical" if same else "DIFFERS"}', flush=True)
print('pair_pf_probe done')

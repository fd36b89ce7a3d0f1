"""Run only the fused FFN kernel (config-2 encoder shape at batch 8 unless --rows) a few
times -- a short program for rocprofv3 --pmc passes (tools/pmc_probe.sh)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--rows', type=int, default=8 * 22223)
ap.add_argument('--iters', type=int, default=5)
ap.add_argument('--d', type=int, default=256)
ap.add_argument('--knobs', default='0,2,8', help='kinet_ffn_set_debug values (D = 288: 0 = wave pairs, 32 = 4 waves)')
ap.add_argument('--dtype', default='bf16', choices=['bf16', 'f16'])
a = ap.parse_args()
D = a.d
dt = torch.bfloat16 if a.dtype == 'bf16' else torch.float16
lin1, lin2, norm = torch.nn.Linear(D, 1024).cuda(), torch.nn.Linear(1024, D).cuda(), torch.nn.LayerNorm(D).cuda()
x = torch.randn(a.rows, D, device='cuda', dtype=dt)
from kinet_amd import _native as N  # noqa: E402
ref = None
for knob in [int(k) for k in a.knobs.split(',')]:
    N.lib().kinet_ffn_set_debug(knob)
    for _ in range(2):
        y = K.ffn_fused(x, lin1, lin2, norm)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        y = K.ffn_fused(x, lin1, lin2, norm)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / a.iters
    tf = 4.0 * a.rows * D * 1024 / (us * 1e-6) / 1e12
    same = 'ref' if ref is None else ('bit-identical' if torch.equal(ref, y) else
                                     'max diff %.3g' % (ref.float() - y.float()).abs().max().item())
    ref = y if ref is None else ref
    print('ffn_probe knob %d: rows %d, %.1f us, %.0f TF/s, %s' % (knob, a.rows, us, tf, same))
N.lib().kinet_ffn_set_debug(0)
print('ffn_probe done')

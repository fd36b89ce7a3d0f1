"""Time output_proj + residual + LayerNorm (K.linear with ln) at the config-5 encoder shape
(M = 4 x 43110 rows, d = 288, f16) and the config-2 one (M = 16 x 22223, d = 256, bf16).
usage: python tools/ln_gemm_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd import kernels as K  # noqa: E402
from tools.bench_msda import time_call  # noqa: E402

for M, d, dt in ((4 * 43110, 288, torch.float16), (16 * 22223, 256, torch.bfloat16)):
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randn(M, d, device='cuda', generator=g).to(dt)
    r = torch.randn(M, d, device='cuda', generator=g).to(dt)
    w = (torch.randn(d, d, device='cuda', generator=g) / d ** 0.5).to(dt)
    b = torch.randn(d, device='cuda', generator=g)
    gam, bet = torch.rand(d, device='cuda') + 0.5, torch.randn(d, device='cuda')
    fn = lambda: K.linear(x, w, b, residual=r, ln=(gam, bet, 1e-5))  # noqa: E731
    time_call(fn, 20)
    ms = time_call(fn, 50)
    print(f'LN-GEMM M={M} d={d} {dt}: {ms * 1e3:.1f} us  {2 * M * d * d / ms / 1e9:.0f} TF/s  '
          f'{3 * M * d * 2 / ms / 1e6:.0f} GB/s (x, r, y)')

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
a = ap.parse_args()
lin1, lin2, norm = torch.nn.Linear(256, 1024).cuda(), torch.nn.Linear(1024, 256).cuda(), torch.nn.LayerNorm(256).cuda()
x = torch.randn(a.rows, 256, device='cuda', dtype=torch.bfloat16)
for _ in range(a.iters):
    K.ffn_fused(x, lin1, lin2, norm)
torch.cuda.synchronize()
print('ffn_probe done')

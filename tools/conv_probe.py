"""Run one implicit-GEMM conv shape a few times (default: the layer-3 3x3 256->256 conv at
batch 8) -- a short program for rocprofv3 --pmc passes (tools/pmc_probe.sh)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--shape', default='8,50,84,256,256,3,1', help='B,H,W,Cin,Cout,k,stride')
ap.add_argument('--iters', type=int, default=5)
ap.add_argument('--tile', default='0,0', help='forced BMxBN (kinet_gemm_force_tile), 0,0 = heuristic')
a = ap.parse_args()
B, H, W, Cin, Cout, k, s = (int(v) for v in a.shape.split(','))
x = torch.randn(B, H, W, Cin, device='cuda', dtype=torch.bfloat16)
wp = K.pack_conv_weight(torch.randn(Cout, Cin, k, k, device='cuda') * 0.02, torch.bfloat16)
from kinet_amd import _native  # noqa: E402
_native.lib().kinet_gemm_force_tile(*(int(v) for v in a.tile.split(',')))
for _ in range(a.iters):
    K.conv2d_nhwc(x, wp, s, k // 2)
torch.cuda.synchronize()
print('conv_probe done')

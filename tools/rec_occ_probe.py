"""Records GEMM (kinet_msda_sample_records, batch-16 encoder shape) at 3 / 2 workgroups per
CU (kinet_gemm_set_flags 0 = three per CU, 8192 = two); run under rocprofv3 --kernel-trace --stats for
device times."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd import _native  # noqa: E402
from kinet_amd import kernels as K  # noqa: E402

shapes = ((100, 167), (50, 84), (25, 42), (13, 21))
S = sum(h * w for h, w in shapes)
B = 16
g = torch.Generator().manual_seed(0)
x = torch.randn(B, S, 256, generator=g).bfloat16().cuda()
pos = torch.randn(B, S, 256, generator=g).bfloat16().cuda()
w = (torch.randn(384, 256, generator=g) / 16).cuda()
bias = torch.randn(384, generator=g).cuda()
ref = torch.rand(B, S, 4, 2, generator=g).cuda()
lib = _native.lib()
for flags in (0, 8192, 0, 8192):
    lib.kinet_gemm_set_flags(flags)
    for _ in range(3):
        K.msda_sample_records(x, w, bias, 8, ref, shapes, x_add=pos)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        K.msda_sample_records(x, w, bias, 8, ref, shapes, x_add=pos)
    e1.record()
    torch.cuda.synchronize()
    print(f'flags {flags:6d}: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per call', flush=True)
lib.kinet_gemm_set_flags(0)

"""Checksum of the encoder sampler's output at the config-2 encoder shape (batch 4), for
bit-identity checks between kernel variants run in separate processes (env knobs).
    python tools/enc_sig_probe.py"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd.msda import MSDeformAttn  # noqa: E402


def main():
    torch.manual_seed(0)
    dev = 'cuda'
    shapes = [(100, 167), (50, 84), (25, 42), (13, 21)]
    S = sum(h * w for h, w in shapes)
    B = 4
    m = MSDeformAttn(256, 4, 8, 4).to(dev)
    with torch.no_grad():
        m.sampling_offsets.bias.add_(torch.randn_like(m.sampling_offsets.bias))
        src = torch.randn(B, S, 256, device=dev).to(torch.bfloat16)
        pos = torch.randn(1, S, 256, device=dev).to(torch.bfloat16)
        ref = torch.rand(B, S, 4, 2, device=dev)
        ss = torch.tensor(shapes, device=dev)
        value = m.project_value(src, None, encoder_shapes=shapes)
        out = m.sample(src, ref, value, ss, query_add=pos, shapes_host=shapes)
    torch.cuda.synchronize()
    print('sig', hashlib.sha256(out.cpu().view(torch.int16).numpy().tobytes()).hexdigest()[:16],
          'mean', out.float().abs().mean().item(), flush=True)


if __name__ == '__main__':
    main()

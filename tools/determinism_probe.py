"""Probe: run the batch-8 detection forward twice serially on the same input and report, stage by
stage (backbone features, encoder memory, decoder hs, logits), the largest difference between the
two runs.  Every kernel of the inference path is meant to be deterministic (bit-identical reruns).
    python tools/determinism_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def flat(o):
    out, _, feats, mem, hs = o
    d = {f'feat{i}': (f.tensors if hasattr(f, 'tensors') else f) for i, f in enumerate(feats)}
    d.update({f'mem{i}': m for i, m in enumerate(mem)})
    d['hs'] = hs
    d['logits'] = out['pred_logits']
    return {k: v.detach().float().clone() for k, v in d.items() if torch.is_tensor(v)}


def main():
    import bench
    from kinet_amd.models import nested_tensor_from_tensor_list
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    model = bench.build(dev, torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = nested_tensor_from_tensor_list([torch.randn(3, 800, 1333, generator=g, device=dev) for _ in range(8)])
    with torch.no_grad():
        model(x)
        runs = []
        for _ in range(3):
            runs.append(flat(model(x)))
            torch.cuda.synchronize()
    for k in runs[0]:
        d1 = (runs[1][k] - runs[0][k]).abs().max().item()
        d2 = (runs[2][k] - runs[0][k]).abs().max().item()
        print(f'{k:8s} {tuple(runs[0][k].shape)}: max|run1-run0| = {d1:.3e}  max|run2-run0| = {d2:.3e}')


if __name__ == '__main__':
    main()

"""Experiment: two batches in flight on two HIP streams (serving-style pipelining) vs one
stream.  Also reports host syncs seen in one forward (torch sync debug mode).
    python tools/bench_streams.py [--batch 8] [--steps 10]
"""
import argparse
import os
import sys
import time
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--steps', type=int, default=10)
    a = ap.parse_args()
    from kinet_amd.models import build_model, nested_tensor_from_tensor_list
    from kinet_amd.models.config import load_args
    torch.manual_seed(0)
    model, _, _ = build_model(load_args('train_deformable', device='cuda'))
    model = model.cuda().eval()
    model.set_compute_dtype(torch.bfloat16)
    g = torch.Generator(device='cuda').manual_seed(1)
    samples = [nested_tensor_from_tensor_list([torch.randn(3, 800, 1333, generator=g, device='cuda')
                                               for _ in range(a.batch)]) for _ in range(3)]
    with torch.no_grad():
        for _ in range(3):
            model(samples[0])
        torch.cuda.synchronize()
        torch.cuda.set_sync_debug_mode(1)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter('always')
            model(samples[0])
        torch.cuda.set_sync_debug_mode(0)
        print(f'host syncs in one forward: {len(w)}')
        for x in w[:5]:
            print('  ', str(x.message)[:160], x.filename, x.lineno)

        def run(nstreams):
            streams = [torch.cuda.Stream() for _ in range(nstreams)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                s = streams[i % nstreams]
                with torch.cuda.stream(s):
                    model(samples[i % 3])
            torch.cuda.synchronize()
            return a.batch * a.steps / (time.perf_counter() - t0)
        for ns in (1, 2, 3):
            run(ns)
            print(f'batch {a.batch}, {ns} stream(s): {run(ns):.1f} frames/s')


if __name__ == '__main__':
    main()

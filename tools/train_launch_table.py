"""Per-launch table of one config-4 training step (the model, optimizer and synthetic batch of
tools/train_torch_ops.py): every kinet launch traced with HIP events (kinet_amd._native.trace_begin /
trace_end), aggregated by (entry point, shape) with average us and achieved TFLOP/s / GB/s from
the algorithmic flops / bytes each launch reports, sorted by total time; plus the sum of the
traced kinet time against the step's wall time (the rest: torch kernels, host glue).

    python tools/train_launch_table.py [--top 40]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd import _native  # noqa: E402
from kinet_amd import train as T  # noqa: E402
from kinet_amd.models import build_model  # noqa: E402
from kinet_amd.models.config import load_args  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--top', type=int, default=40)
    a = ap.parse_args()
    torch.set_float32_matmul_precision('high')
    dev = torch.device('cuda', 0)
    args = load_args('train_deformable', 'train_multi_frame', 'train_tracking', 'train_mot17', device='cuda')
    torch.manual_seed(0)
    model, criterion, _ = build_model(args)
    model = model.to(dev).train()
    model.set_compute_dtype(torch.bfloat16)
    opt = T.build_optimizer(model, args)
    g = torch.Generator().manual_seed(1000)
    samples, targets = T.synthetic_mot_batch(2, 800, 1333, dev, g)

    def step():
        tg = [dict(t, prev_target=dict(t['prev_target'])) for t in targets]
        return T.train_step(model, criterion, opt, samples, tg, args.clip_max_norm)[0]

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    _native.trace_begin()
    try:
        step()
    finally:
        trace = _native.trace_end()
    torch.cuda.synchronize()
    agg = {}
    tot = 0.0
    for name, work, s, e in trace:
        ms = s.elapsed_time(e)
        tot += ms
        key = (name, str(work.get('shape', '')))
        r = agg.setdefault(key, [0, 0.0, 0.0, 0.0])
        r[0] += 1
        r[1] += ms
        r[2] += work.get('flops', 0.0)
        r[3] += work.get('bytes', 0.0)
    print(f'step wall {wall:.1f} ms (untraced); traced kinet device time {tot:.1f} ms over {len(trace)} launches')
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    for (name, shape), (n, ms, fl, by) in rows[:a.top]:
        t = ms * 1e-3
        print(f'{ms / tot * 100:5.1f}% {n:4d} x {ms / n * 1e3:8.1f} us  {fl / t / 1e12 if t else 0:7.1f} TF/s '
              f'{by / t / 1e9 if t else 0:7.0f} GB/s  {name} {shape}')


if __name__ == '__main__':
    main()

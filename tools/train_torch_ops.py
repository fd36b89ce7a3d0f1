"""Which torch (non-kinet) device work the config-4 training step still launches, and from where:
torch.profiler over 2 steps (after warm-up), the aten ops that launch device kernels grouped by
(op, input shapes) with counts and device time, plus the Python frames of the top copy / add
sources.  Targets of VERDICT r4 item 5 (non-kinet share of the train step's device time).

    python tools/train_torch_ops.py [--top 25]
"""
import argparse
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd.models import build_model  # noqa: E402
from kinet_amd.models.config import load_args  # noqa: E402
from kinet_amd import train as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--top', type=int, default=25)
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
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    ev = prof.key_averages(group_by_input_shape=True)
    rows = sorted(ev, key=lambda e: -e.self_device_time_total)
    tot = sum(e.self_device_time_total for e in ev)
    print(f'total self device time over 2 steps: {tot / 1e3:.1f} ms')
    # device kernels only (the op-level rows carry the same time again): kinet vs the rest
    from torch.autograd import DeviceType
    kern = [e for e in ev if e.device_type == DeviceType.CUDA]
    kt = sum(e.self_device_time_total for e in kern)
    kin = sum(e.self_device_time_total for e in kern if 'kinet' in e.key)
    print(f'device kernels: {kt / 2e3:.2f} ms per step, kinet {kin / 2e3:.2f} ms, other {(kt - kin) / 2e3:.2f} ms '
          f'= {(kt - kin) / max(kt, 1):.3f} of kernel time')
    other = sorted([e for e in kern if 'kinet' not in e.key], key=lambda e: -e.self_device_time_total)
    for e in other[:15]:
        print(f'   {e.self_device_time_total / 2e3:8.3f} ms/step  {e.count // 2:5d}x  {e.key[:100]}')
    for e in rows[:a.top]:
        print(f'{e.self_device_time_total / 1e3:9.2f} ms  {e.count:6d}x  {e.key[:60]:60s} {str(e.input_shapes)[:90]}')
    # Python sources of the copy / add / fill launches
    src = defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if e.name in ('aten::copy_', 'aten::add_', 'aten::add', 'aten::fill_', 'aten::zero_', 'aten::cat',
                      'aten::contiguous', 'aten::clone') and e.device_time_total > 0:
            frames = [f for f in (e.stack or []) if 'kinet_amd' in f or 'train.py' in f]
            key = (e.name, frames[0] if frames else '?')
            src[key][0] += 1
            src[key][1] += e.device_time_total
    print('\n-- copy / add / fill sources (first kinet_amd frame) --')
    for (n, f), (c, t) in sorted(src.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f'{t / 1e3:9.2f} ms  {c:6d}x  {n:18s} {f}')


if __name__ == '__main__':
    main()

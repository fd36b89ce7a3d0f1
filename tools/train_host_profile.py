"""Where the host time of the config-4 train step goes: cProfile over 2 steps (after warmup),
top functions by own time and by cumulative time, plus the step's wall time vs the device
time of its kernels (torch profiler-free: HIP events around the step).
    python tools/train_host_profile.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kinet_amd.models import build_model  # noqa: E402
from kinet_amd.models.config import load_args  # noqa: E402
from kinet_amd import train as T  # noqa: E402

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
for _ in range(3):
    t0 = time.perf_counter()
    step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'step: host returns after {1e3 * (t1 - t0):.1f} ms, device done at {1e3 * (t2 - t0):.1f} ms', flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(2):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats('tottime').print_stats(25)
st.sort_stats('cumulative').print_stats(45)

#!/usr/bin/env python
"""Training throughput of config 4 (BASELINE.json configs[3], cfgs/train_mot17.yaml:
`mot17 deformable multi_frame tracking`): DeformableDETRTracking, d=288, 500 queries,
multi-frame (8 decoder levels), two-pass track-query training, focal + L1 + GIoU with aux
losses, AdamW, clip 0.1.  Synthetic (current, prev) 3x800x1333 frame pairs with 10-30
boxes each, random-init weights.

    python tools/bench_train.py [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... tools/bench_train.py

One step = one optimiser step over `--batch` current frames per GPU (each with its
previous frame run without grad inside the step).  Gradients are averaged by DDP over
RCCL.  Prints one JSON line on rank 0: frames/s (current frames, whole job) and
images/s (= 2x, both frames of each pair).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--batch', type=int, default=2)
    ap.add_argument('--height', type=int, default=800)
    ap.add_argument('--width', type=int, default=1333)
    ap.add_argument('--prev-dtype', default='bf16', choices=['bf16', 'f32'],
                    help='compute dtype of the no-grad previous-frame pass (HIP path)')
    a = ap.parse_args()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    from kinet_amd.train import build_optimizer, setup_ddp, synthetic_mot_batch, train_step
    args = load_args('train_deformable', 'train_multi_frame', 'train_tracking', 'train_mot17', device='cuda')
    torch.manual_seed(0)
    model, criterion, _ = build_model(args)
    model = model.to(dev).train()
    model.set_compute_dtype(torch.bfloat16 if a.prev_dtype == 'bf16' else torch.float32)
    ddp = setup_ddp(model, dev)
    opt = build_optimizer(ddp, args)
    g = torch.Generator().manual_seed(1000 + rank)
    samples, targets = synthetic_mot_batch(a.batch, a.height, a.width, dev, g)

    def step():
        tg = [dict(t, prev_target=dict(t['prev_target'])) for t in targets]
        return train_step(ddp, criterion, opt, samples, tg, args.clip_max_norm)[0]

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    if rank == 0:
        frames = a.batch * a.steps * world
        print(json.dumps({
            'metric': 'train frames/sec (config 4: mot17 deformable multi_frame tracking, 3x800x1333 pairs)',
            'value': frames / el, 'unit': 'frames/s', 'images_per_s': 2 * frames / el, 'n_gpus': world,
            'steps': a.steps, 'warmup': a.warmup, 's_per_step': el / a.steps, 'loss': float(loss),
            'scaling': 'weak', 'data': 'synthetic frame pairs, 10-30 boxes, random-init weights',
            'config': {'workload': 'config4 two-pass tracking training step', 'batch_per_gpu': a.batch,
                       'hidden_dim': args.hidden_dim, 'num_queries': args.num_queries,
                       'prev_frame_dtype': a.prev_dtype, 'grad_frame_dtype': 'f32',
                       'parallelism': f'ddp{world} (RCCL all-reduce)'}}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

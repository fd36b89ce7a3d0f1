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
    ap.add_argument('--matmul-precision', default='high', choices=['highest', 'high'],
                    help="f32 GEMMs of the grad frame: 'high' = bf16x3 MFMA products, 'highest' = exact f32")
    a = ap.parse_args()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)
    from kinet_amd.train import benchmark_train
    res = benchmark_train(a.steps, a.warmup, a.batch, a.height, a.width,
                          torch.bfloat16 if a.prev_dtype == 'bf16' else torch.float32, dev,
                          matmul_precision=a.matmul_precision)
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

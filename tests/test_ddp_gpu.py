"""Two-rank DistributedDataParallel training step of the REAL tracking detector (config-4
structure at a small size: DeformableDETRTracking, d=288, multi-frame, two-pass track-query
training with the matcher inside forward), train.py:84-91 / engine.py:124-149.

Each rank takes a different synthetic batch.  The DDP gradients (averaged over the two
ranks by DDP's bucketed all-reduce, find_unused_parameters=True as train.py:89-90) must
equal the mean of the two ranks' single-process gradients of the same step (same seeds ->
same track-query sampling).

Runs on the GPU box: the detector's autograd path runs kinet kernels only (the reference's
MSDeformAttn has no CPU path either, ms_deform_attn.h:27), so the two ranks share cuda:0 and
talk over gloo (RCCL refuses two ranks on one device).  Unmeasured on multi-GPU hardware:
the driver's 8-GPU run is the first place RCCL carries it.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, golden_dir, out_path):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, golden_dir)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from weights import make_state_dict
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    from kinet_amd.train import synthetic_mot_batch, weighted_loss
    args = load_args('train_deformable', 'train_multi_frame', 'train_tracking', dataset='mot', dropout=0.0,
                     num_queries=40, enc_layers=2, dec_layers=3, device='cuda')
    model, criterion, _ = build_model(args)
    keys = [ln.split() for ln in open(os.path.join(golden_dir, 'train_step_small.keys.txt'))]
    model.load_state_dict(make_state_dict({k[0]: [int(s) for s in k[1:]] for k in keys}, seed=71))
    model = model.cuda().train()
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(500 + rank)
    samples, targets = synthetic_mot_batch(2, 96, 128, dev, g, num_boxes=(4, 8))

    def loss_of(m):
        torch.manual_seed(900 + rank)
        tg = [dict(t, prev_target=dict(t['prev_target'])) for t in targets]
        out, tg, *_ = m(samples, tg)
        return weighted_loss(criterion(out, tg), criterion.weight_dict)

    # single-process gradients of this rank's batch
    loss_of(model).backward()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    single = {n: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
              for n, p in model.named_parameters() if p.requires_grad}
    model.zero_grad(set_to_none=True)
    # the same step under DDP
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], find_unused_parameters=True)
    loss_of(ddp).backward()
    worst = 0.0
    n_checked = 0
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        mean = single[n].clone()
        dist.all_reduce(mean)
        mean /= world
        got = p.grad if p.grad is not None else torch.zeros_like(p)
        scale = mean.abs().max().item()
        err = (got - mean).abs().max().item()
        if scale > 0:
            worst = max(worst, err / scale)
        n_checked += 1
    if rank == 0:
        with open(out_path, 'w') as f:
            f.write(f'{worst} {n_checked} {len(names)}\n')
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_two_rank_detector_gradients(golden_dir, tmp_path):
    out = str(tmp_path / 'ddp.txt')
    mp.spawn(_worker, args=(2, _free_port(), golden_dir, out), nprocs=2, join=True)
    worst, n_checked, n_params = open(out).read().split()
    assert int(n_checked) == int(n_params) > 100
    # fp32 GEMM / all-reduce summation-order differences only
    assert float(worst) < 1e-4, worst

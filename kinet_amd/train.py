"""Training step of the tracking detector (config 4, cfgs/train_mot17.yaml), mirroring
src/train.py:84-120 (DDP wrap, AdamW parameter groups) and
src/trackformer/engine.py:119-149 (forward -> criterion -> weighted sum -> backward ->
clip -> step).

Compute split:
  * previous-frame forward without grad: the HIP inference path (bf16 or f32) when the
    model has no active dropout, else the op-for-op path (train-mode dropout, as the
    reference runs it) -- on kinet kernels either way;
  * current-frame forward with grad: op-for-op modules in f32 on kinet_amd.autograd
    Functions (backbone convs, Linear, LayerNorm, GroupNorm, attention: forward and backward
    on kinet kernels) and MSDeformAttnFunction (HIP forward / backward);
  * Hungarian matching and track-query sampling on the host (north_star);
  * gradients averaged over ranks by DistributedDataParallel over RCCL ("nccl" backend),
    bucketed and overlapped with backward -- the one exchange step of the path; the
    criterion's num_boxes scalar is all-reduced as in detr.py:845.
"""
import os

import torch
import torch.distributed as dist

from kinet_amd.models.misc import nested_tensor_from_tensor_list


def match_name_keywords(n, name_keywords):
    return any(b in n for b in name_keywords)


def build_optimizer(model, args):
    """train.py:95-120: base lr, backbone lr, linear-projection lr multiplier; AdamW."""
    m = model.module if hasattr(model, 'module') else model
    lp = list(args.lr_linear_proj_names)
    bb = list(args.lr_backbone_names)
    param_dicts = [
        {"params": [p for n, p in m.named_parameters()
                    if not match_name_keywords(n, bb + lp + ['layers_track_attention']) and p.requires_grad],
         "lr": args.lr},
        {"params": [p for n, p in m.named_parameters() if match_name_keywords(n, bb) and p.requires_grad],
         "lr": args.lr_backbone},
        {"params": [p for n, p in m.named_parameters() if match_name_keywords(n, lp) and p.requires_grad],
         "lr": args.lr * args.lr_linear_proj_mult}]
    return torch.optim.AdamW(param_dicts, lr=args.lr, weight_decay=args.weight_decay)


def weighted_loss(loss_dict, weight_dict):
    """engine.py:128."""
    return sum(loss_dict[k] * weight_dict[k] for k in loss_dict.keys() if k in weight_dict)


def reduce_dict(input_dict, average=True):
    """util/misc.py reduce_dict: loss values averaged over ranks (logging only)."""
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    if world < 2:
        return input_dict
    with torch.no_grad():
        names = sorted(input_dict.keys())
        values = torch.stack([input_dict[k].detach().float().reshape(()) for k in names])
        dist.all_reduce(values)
        if average:
            values /= world
        return dict(zip(names, values))


def train_step(model, criterion, optimizer, samples, targets, clip_max_norm=0.1):
    """One optimisation step (engine.py:124-149).  Returns (weighted loss, loss_dict)."""
    outputs, targets, *_ = model(samples, targets)
    defer = hasattr(criterion, 'pop_deferred_checks')
    if defer:
        criterion.defer_box_checks = True
    try:
        loss_dict = criterion(outputs, targets)
    finally:
        if defer:
            criterion.defer_box_checks = False
    losses = weighted_loss(loss_dict, criterion.weight_dict)
    # one host read for the loss-finiteness check (engine.py:131-134) and the criterion's GIoU
    # degenerate-box asserts (util/box_ops.py:44-45, deferred to here)
    flags = [torch.isfinite(losses).reshape(())]
    boxes_ok = criterion.pop_deferred_checks() if hasattr(criterion, 'pop_deferred_checks') else None
    if boxes_ok is not None:
        flags.append(boxes_ok.reshape(()))
    flags = torch.stack(flags).tolist()
    if not flags[0]:
        raise FloatingPointError(f'non-finite loss {losses.item()}: '
                                 + ', '.join(f'{k}={v.item():.4g}' for k, v in loss_dict.items()))
    assert all(flags[1:]), 'degenerate boxes (util/box_ops.py:44-45)'

    optimizer.zero_grad()
    losses.backward()
    if clip_max_norm > 0:
        torch.nn.utils.clip_grad_norm_(model.parameters(), clip_max_norm)
    optimizer.step()
    return losses.detach(), loss_dict


def synthetic_mot_batch(batch, height, width, device, generator, num_boxes=(10, 30), track_overlap=0.8):
    """per sample a (current, prev) frame pair of N(0,1) pixels
    with 10-30 boxes, cxcy ~ U(0.05, 0.95), wh ~ U(0.02, 0.2), labels 0 (person), and track
    ids shared between the two frames for `track_overlap` of the objects."""
    samples, targets = [], []
    lo, hi = num_boxes
    for _ in range(batch):
        n = int(torch.randint(lo, hi + 1, (1,), generator=generator))
        n_prev = int(torch.randint(lo, hi + 1, (1,), generator=generator))
        shared = int(min(n, n_prev) * track_overlap)

        def boxes(k):
            c = torch.rand(k, 2, generator=generator) * 0.9 + 0.05
            wh = torch.rand(k, 2, generator=generator) * 0.18 + 0.02
            return torch.cat([c, wh], -1)
        ids_cur = torch.cat([torch.arange(shared), 1000 + torch.arange(n - shared)])
        ids_prev = torch.cat([torch.arange(shared), 2000 + torch.arange(n_prev - shared)])
        ids_prev = ids_prev[torch.randperm(n_prev, generator=generator)]
        cur = {'boxes': boxes(n), 'labels': torch.zeros(n, dtype=torch.long), 'track_ids': ids_cur}
        prev = {'boxes': boxes(n_prev), 'labels': torch.zeros(n_prev, dtype=torch.long), 'track_ids': ids_prev}
        img = torch.randn(3, height, width, generator=generator)
        prev_img = torch.randn(3, height, width, generator=generator)
        cur = {k: v.to(device) for k, v in cur.items()}
        cur['prev_target'] = {k: v.to(device) for k, v in prev.items()}
        cur['prev_image'] = prev_img.to(device)
        samples.append(img.to(device))
        targets.append(cur)
    return nested_tensor_from_tensor_list(samples), targets


def setup_ddp(model, device, find_unused_parameters=True):
    """train.py:84-91: DistributedDataParallel over the RCCL process group (env:// rendezvous).
    find_unused_parameters=True is the reference's setting (train.py:89-91); every parameter of
    this model receives a gradient in the two-pass step, so False skips DDP's extra traversal of
    the autograd graph per step without changing the result (bench.py --ddp-find-unused 0)."""
    if not (dist.is_available() and dist.is_initialized()):
        return model
    local = int(os.environ.get('LOCAL_RANK', '0'))
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=[local] if device.type == 'cuda' else None,
                                                     find_unused_parameters=find_unused_parameters)


HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 (the KINET_F32_X3 products run on the bf16 MFMA)


def train_rooflines(trace):
    """Per-family rooflines of one traced training step: the MSDA backward launches against HBM
    (SURVEY 8(d) B_bwd per call), split encoder (list kernel) / decoder, and every GEMM / conv /
    weight-gradient launch against the dense MFMA peak."""
    out = {}
    bwd = [(w, s.elapsed_time(e)) for name, w, s, e in trace if w.get('family') == 'msda_bwd']
    if bwd:
        def roof(items, label):
            ms = sum(t for _, t in items)
            by = sum(w['bytes'] for w, _ in items)
            ach = by / (ms * 1e-3) / 1e9
            return {'bound': 'hbm', 'kernel': label, 'achieved': ach, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                    'frac': ach / HBM_PEAK_GBS, 'algorithmic_bytes_per_launch': by / len(items),
                    'avg_launch_ms': ms / len(items), 'launches_per_step': len(items),
                    'bytes_basis': 'SURVEY 8(d) B_bwd: value + grad_out + loc/attw + f32 grad_value + grad loc/attw'}
        enc = [x for x in bwd if x[0]['kernel'] == 'msda_bwd_list_kernel']
        dec = [x for x in bwd if x[0]['kernel'] != 'msda_bwd_list_kernel']
        r = roof(enc or dec, 'msda_bwd_list_kernel (encoder calls, Lq = S)' if enc else 'msda_bwd_kernel')
        if enc and dec:
            r['decoder_kernel'] = roof(dec, 'msda_bwd_kernel (decoder calls)')
        out['msda_bwd'] = r
    gr = [(w, s.elapsed_time(e)) for name, w, s, e in trace
          if w.get('flops') and w.get('family') in ('grad', 'gemm', 'conv')]
    if gr:
        ms = sum(t for _, t in gr)
        fl = sum(w['flops'] for w, _ in gr)
        ach = fl / (ms * 1e-3) / 1e12
        out['grad'] = {'bound': 'mfma', 'kernel': 'every GEMM / conv / weight-gradient launch of the step',
                       'achieved': ach, 'peak': MFMA_BF16_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                       'frac': ach / MFMA_BF16_PEAK_TFLOPS, 'launches_per_step': len(gr), 'device_ms_per_step': ms,
                       'note': 'f32 operands as three bf16 MFMA passes (KINET_F32_X3): algorithmic flops counted '
                               'once, so the MFMA pipe runs 3x the reported rate'}
    return out


def benchmark_train(steps=10, warmup=2, batch=2, height=800, width=1333, prev_dtype=torch.bfloat16, device=None,
                    dropout=None, matmul_precision='high', find_unused_parameters=True):
    """Config-4 training throughput (BASELINE.json configs[3], cfgs/train_mot17.yaml: `mot17
    deformable multi_frame tracking`, d=288, 500 queries, two-pass track-query training,
    focal + L1 + GIoU with aux losses, AdamW, clip 0.1) on synthetic (current, prev) frame
    pairs; DDP over the initialised process group when there is one.  Returns a dict with
    frames/s (current frames of the whole job), images/s (= 2x) and s/step; the timed region
    is bracketed by a barrier + device synchronisation and the elapsed time is the max over
    ranks.  matmul_precision: torch.set_float32_matmul_precision for the run -- 'high' runs
    the f32 grad frame's GEMMs / convs / weight gradients as three bf16 MFMA passes
    (KINET_F32_X3, ~2^-17 relative error per product; the reference's own cuDNN convs run
    TF32, 2^-11, by default), 'highest' on the exact f32 MFMA."""
    prev_prec = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(matmul_precision)
    try:
        return _benchmark_train(steps, warmup, batch, height, width, prev_dtype, device, dropout, matmul_precision,
                                find_unused_parameters)
    finally:
        torch.set_float32_matmul_precision(prev_prec)


def _benchmark_train(steps, warmup, batch, height, width, prev_dtype, device, dropout, matmul_precision,
                     find_unused_parameters=True):
    import statistics
    import time
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    dev = device or torch.device('cuda', torch.cuda.current_device())
    over = {} if dropout is None else {'dropout': dropout}
    args = load_args('train_deformable', 'train_multi_frame', 'train_tracking', 'train_mot17', device='cuda', **over)
    torch.manual_seed(0)
    model, criterion, _ = build_model(args)
    model = model.to(dev).train()
    model.set_compute_dtype(prev_dtype)
    ddp = setup_ddp(model, dev, find_unused_parameters)
    opt = build_optimizer(ddp, args)
    g = torch.Generator().manual_seed(1000 + rank)
    samples, targets = synthetic_mot_batch(batch, height, width, dev, g)

    def step():
        tg = [dict(t, prev_target=dict(t['prev_target'])) for t in targets]
        return train_step(ddp, criterion, opt, samples, tg, args.clip_max_norm)[0]

    for _ in range(max(1, warmup)):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the reported rate: K steps back to back (no extra synchronisation between them, so host
    # work of step i+1 overlaps the device tail of step i as in a real training loop), elapsed
    # time max over ranks -> value = frames / elapsed
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # a separate pass with every step timed on its own (device synchronised on both sides): the
    # median / min / max describe the spread; they are not the reported value
    per_step = []
    for _ in range(steps):
        ts = time.perf_counter()
        step()
        torch.cuda.synchronize()
        per_step.append(time.perf_counter() - ts)
    if world > 1:
        t = torch.tensor([el] + per_step, device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, per_step = t[0].item(), t[1:].tolist()
    med = statistics.median(per_step)
    # host glue of the step (matcher + track-query sampler), measured over
    # two extra steps: wall seconds in those functions, the part of it spent waiting for the
    # device in the one-sync-per-call host copies, and the number of such syncs
    from kinet_amd.models import training as TR
    TR.GLUE.update(on=True, glue_s=0.0, sync_wait_s=0.0, syncs=0)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    glue = dict(TR.GLUE)
    TR.GLUE['on'] = False
    # backward rooflines: HIP events around every kinet launch of one more step (one stream)
    from kinet_amd import _native
    _native.trace_begin()
    try:
        step()
    finally:
        trace = _native.trace_end()
    torch.cuda.synchronize()
    rooflines = train_rooflines(trace)
    frames = batch * steps * world
    from kinet_amd.models.training import _has_dropout
    # with dropout > 0 the previous frame runs op-for-op in f32 (train-mode dropout, as the
    # reference runs it: prepare_track_queries -> reference_path), not the bf16 HIP path
    prev_desc = ('float32 (op-for-op path: train-mode dropout %g, as the reference)' % args.dropout
                 if _has_dropout(model) else str(prev_dtype).replace('torch.', ''))
    fpstep = batch * world
    pg = 'none (single process)'
    if world >= 1 and dist.is_available() and dist.is_initialized():
        pg = f'ddp{world}: DistributedDataParallel over a {world}-rank {dist.get_backend()} process group'
        pg += ', find_unused_parameters=%s' % find_unused_parameters
        if dist.get_backend() == 'nccl':
            pg += ' (RCCL all-reduce)'
    return {'metric': 'train frames/sec (config 4: mot17 deformable multi_frame tracking, 3x%dx%d pairs)'
                      % (height, width),
            'value': frames / el, 'unit': 'frames/s', 'images_per_s': 2 * frames / el, 'n_gpus': world,
            'steps': steps, 'warmup': warmup, 's_per_step': el / steps, 's_per_step_mean': el / steps,
            's_per_step_median_synced': med, 's_per_step_min_synced': min(per_step),
            's_per_step_max_synced': max(per_step), 'frames_per_s_median_synced': fpstep / med,
            'rate_basis': 'frames of all ranks / elapsed time of K back-to-back steps (max over ranks); the '
                          '*_synced fields come from a second pass with each step synchronised and timed alone',
            'loss': float(loss), 'scaling': 'weak',
            'host_glue': {'ms_per_step': glue['glue_s'] / 2 * 1e3,
                          'device_wait_ms_per_step': glue['sync_wait_s'] / 2 * 1e3,
                          'host_only_ms_per_step': (glue['glue_s'] - glue['sync_wait_s']) / 2 * 1e3,
                          'device_to_host_syncs_per_step': glue['syncs'] / 2,
                          'what': 'matcher (prev frame + criterion, all output sets) + track-query sampler'},
            'msda_bwd_roofline': rooflines.get('msda_bwd'), 'dense_grad_roofline': rooflines.get('grad'),
            'dtype': 'f32', 'data': 'synthetic frame pairs, 10-30 boxes, random-init weights',
            'config': {'workload': 'config4 two-pass tracking training step (prev frame no-grad, current frame '
                                   'fwd+bwd, AdamW)', 'batch_per_gpu': batch, 'hidden_dim': args.hidden_dim,
                       'num_queries': args.num_queries, 'dropout': args.dropout,
                       'prev_frame_dtype': prev_desc,
                       'grad_frame_dtype': 'f32', 'f32_matmul_precision': matmul_precision +
                       (' (bf16x3 MFMA products)' if matmul_precision != 'highest' else ' (exact f32 MFMA)'),
                       'parallelism': pg}}

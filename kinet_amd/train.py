"""Training step of the tracking detector (config 4, cfgs/train_mot17.yaml), mirroring
src/train.py:84-120 (DDP wrap, AdamW parameter groups) and
src/trackformer/engine.py:119-149 (forward -> criterion -> weighted sum -> backward ->
clip -> step).

Compute split:
  * previous-frame forward without grad: the HIP inference path (bf16 or f32);
  * current-frame forward with grad: op-for-op modules with the HIP MSDeformAttn
    forward/backward kernels (MSDeformAttnFunction); dense layers via the library GEMMs
    of PyTorch-ROCm;
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
    loss_dict = criterion(outputs, targets)
    losses = weighted_loss(loss_dict, criterion.weight_dict)
    if not torch.isfinite(losses):
        raise FloatingPointError(f'non-finite loss {losses.item()}: '
                                 + ', '.join(f'{k}={v.item():.4g}' for k, v in loss_dict.items()))
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


def setup_ddp(model, device):
    """train.py:84-91: DistributedDataParallel over the RCCL process group (env:// rendezvous)."""
    if not (dist.is_available() and dist.is_initialized()):
        return model
    local = int(os.environ.get('LOCAL_RANK', '0'))
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=[local] if device.type == 'cuda' else None,
                                                     find_unused_parameters=True)

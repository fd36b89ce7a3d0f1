"""Host-side training glue of the tracking detector: track-query sampling and the
two-pass forward (src/trackformer/models/detr_tracking.py:39-283).

Training step of a sample pair (detr_tracking.py:225-265): the previous frame is run
without grad (the HIP inference path), Hungarian-matched to its targets on the host,
a random subset of the matched detections becomes the current frame's track queries
(plus false positives drawn near them), and the current frame runs with grad.

`add_track_queries_to_targets` makes exactly the reference's sequence of torch
global-RNG calls (randint, randint, then per sample randperm / randperm / multinomial or
randperm), so a seeded run draws the same track queries as the reference -- pinned by
tests/golden/train_sampler.npz.  The reference's distance weight uses the x offset twice
(`box_weights[:, 0] ** 2 + box_weights[:, 0] ** 2`, :128); kept for parity.
"""
import contextlib
import math
import time

import torch
from torch import nn

from kinet_amd.models.deformable_transformer import reference_path


def empty_track_queries(model, targets):
    """Evaluation with targets: detection only, no track queries (detr_tracking.py:259-270)."""
    for target in targets:
        device = target['boxes'].device
        target['track_query_hs_embeds'] = torch.zeros(0, model.hidden_dim).float().to(device)
        target['track_queries_mask'] = torch.zeros(model.num_queries).bool().to(device)
        target['track_queries_fal_pos_mask'] = torch.zeros(model.num_queries).bool().to(device)
        target['track_query_boxes'] = torch.zeros(0, 4).to(device)
        target['track_query_match_ids'] = torch.tensor([]).long().to(device)


# host-glue accounting of the training step (kinet_amd/train.py benchmark_train reports it):
# seconds spent in the matcher / sampler, seconds of those spent waiting in to_host for the
# device, and the number of device->host synchronisations
GLUE = {'on': False, 'glue_s': 0.0, 'sync_wait_s': 0.0, 'syncs': 0}


class glue_timer:
    def __enter__(self):
        self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        if GLUE['on']:
            GLUE['glue_s'] += time.perf_counter() - self.t0


def to_host(*tensors):
    """Device -> host copies of several tensors with ONE synchronisation: pinned destinations,
    non-blocking copies queued on the current stream, then a single stream sync.  Host
    tensors pass through."""
    dev = next((t.device for t in tensors if t.is_cuda), None)
    if dev is None:
        return list(tensors)
    t0 = time.perf_counter()
    out = []
    for t in tensors:
        if t.is_cuda:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            out.append(h)
        else:
            out.append(t)
    torch.cuda.current_stream(dev).synchronize()
    if GLUE['on']:
        GLUE['sync_wait_s'] += time.perf_counter() - t0
        GLUE['syncs'] += 1
    return out


def to_device(t, device):
    """Host -> device without a host-side wait (pinned source, non-blocking copy)."""
    if device.type != 'cuda':
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


def add_track_queries_to_targets(model, targets, prev_indices, prev_out, add_false_pos=True):
    with glue_timer():
        _add_track_queries_to_targets(model, targets, prev_indices, prev_out, add_false_pos)


def _add_track_queries_to_targets(model, targets, prev_indices, prev_out, add_false_pos=True):
    """detr_tracking.py:39-218, batched host traffic.

    The reference loops over samples with device tensors, so every `nonzero`, membership
    test and `multinomial(box_weights.cpu())` synchronises with the GPU (≈4 syncs per sample
    plus one per false positive).  Here the sampler's inputs cross to the host ONCE per batch
    (track ids of both frames, the previous frame's boxes when false positives are drawn; one
    stream sync), the per-sample logic runs on host tensors with the reference's exact
    sequence of global-RNG calls, and the results go back in one non-blocking copy per dtype:
    the track-query embeddings / boxes are one gather from the flattened previous-frame
    outputs, split per sample."""
    device = prev_out['pred_boxes'].device
    fp_prob = model._track_query_false_positive_prob
    fn_prob = model._track_query_false_negative_prob
    min_prev_target_ind = min([len(prev_ind[1]) for prev_ind in prev_indices])
    num_prev_target_ind = 0
    if min_prev_target_ind:
        num_prev_target_ind = torch.randint(0, min_prev_target_ind + 1, (1,)).item()
    num_prev_target_ind_for_fps = 0
    if num_prev_target_ind:
        num_prev_target_ind_for_fps = torch.randint(int(math.ceil(fp_prob * num_prev_target_ind)) + 1, (1,)).item()

    B, num_q_all = prev_out['pred_boxes'].shape[:2]
    # one host copy of everything the sampler reads (matcher indices are host tensors already)
    prev_ids = [t['prev_target']['track_ids'] for t in targets]
    cur_ids = [t['track_ids'] for t in targets]
    n_prev, n_cur = [len(x) for x in prev_ids], [len(x) for x in cur_ids]
    ids_dev = torch.cat([x.to(device).long().flatten() for x in prev_ids + cur_ids])
    copies = [ids_dev]
    if add_false_pos and num_prev_target_ind_for_fps:
        copies.append(prev_out['pred_boxes'].detach().float())
    host = to_host(*copies)
    ids_host = host[0].split(n_prev + n_cur)
    boxes_all = host[1] if len(host) > 1 else None
    indices = [(o.cpu(), t.cpu()) for o, t in prev_indices]

    flat_idx, match_ids, tq_masks, fp_masks, counts = [], [], [], [], []
    for i in range(len(targets)):
        prev_out_ind, prev_target_ind = indices[i]
        if fn_prob:
            # random subset of the matched detections (:62-79)
            random_subset_mask = torch.randperm(len(prev_target_ind))[:num_prev_target_ind]
            prev_out_ind = prev_out_ind[random_subset_mask]
            prev_target_ind = prev_target_ind[random_subset_mask]

        # match track ids between frames (:82-94)
        match = ids_host[i][prev_target_ind].unsqueeze(dim=1).eq(ids_host[len(targets) + i])
        target_ind_matching = match.any(dim=1)
        match_ids.append(match.nonzero()[:, 1])

        out_ind = prev_out_ind.tolist()
        if add_false_pos:
            # random false positives next to matched detections (:97-158), on the host copy
            random_false_out_ind = []
            taken = set(out_ind)
            not_prev_out_ind = [ind for ind in range(num_q_all) if ind not in taken]
            prev_target_ind_for_fps = torch.randperm(num_prev_target_ind)[:num_prev_target_ind_for_fps]
            if len(prev_target_ind_for_fps):
                boxes_host = boxes_all[i]
                prev_boxes_matched = boxes_host[prev_out_ind[target_ind_matching]]
            for j in prev_target_ind_for_fps:
                if len(prev_boxes_matched) > j:
                    prev_boxes_unmatched = boxes_host[not_prev_out_ind]
                    box_weights = prev_boxes_matched[j].unsqueeze(dim=0)[:, :2] - prev_boxes_unmatched[:, :2]
                    box_weights = box_weights[:, 0] ** 2 + box_weights[:, 0] ** 2   # (sic, :132)
                    box_weights = torch.sqrt(box_weights)
                    random_false_out_idx = not_prev_out_ind.pop(torch.multinomial(box_weights, 1).item())
                else:
                    random_false_out_idx = not_prev_out_ind.pop(torch.randperm(len(not_prev_out_ind))[0])
                random_false_out_ind.append(random_false_out_idx)
            out_ind = out_ind + random_false_out_ind
            target_ind_matching = torch.cat([target_ind_matching,
                                             torch.zeros(len(random_false_out_ind), dtype=torch.bool)])
        K = len(out_ind)
        counts.append(K)
        flat_idx.append(torch.tensor(out_ind, dtype=torch.long) + i * num_q_all)
        # track query masks (:164-184); queries are prepended to the object queries
        tail = torch.zeros(model.num_queries, dtype=torch.bool)
        tq_masks.append(torch.cat([torch.ones(K, dtype=torch.bool), tail]))
        fp_masks.append(torch.cat([~target_ind_matching, tail]))

    # back to the device: one copy per dtype, then views
    n_match = [len(m) for m in match_ids]
    longs = to_device(torch.cat(flat_idx + match_ids), device)
    bools = to_device(torch.cat(tq_masks + fp_masks), device)
    idx_dev, mid_dev = longs[:sum(counts)], longs[sum(counts):]
    hs = prev_out['hs_embed'].flatten(0, 1)[idx_dev].split(counts)
    bx = prev_out['pred_boxes'].detach().flatten(0, 1)[idx_dev].split(counts)
    mids = mid_dev.split(n_match)
    masks = bools.split([c + model.num_queries for c in counts] * 2)
    for i, target in enumerate(targets):
        target['track_query_match_ids'] = mids[i]
        target['track_query_hs_embeds'] = hs[i]
        target['track_query_boxes'] = bx[i]
        target['track_queries_mask'] = masks[i]
        target['track_queries_fal_pos_mask'] = masks[len(targets) + i]


def _has_dropout(model):
    return any(isinstance(m, (nn.Dropout, nn.MultiheadAttention)) and getattr(m, 'p', getattr(m, 'dropout', 0)) > 0
               for m in model.modules())


def _without_aux(out):
    return {k: v for k, v in out.items() if 'aux_outputs' not in k}


def prepare_track_queries(model, targets, base_forward, prev_features=None):
    """detr_tracking.py:221-270.  `base_forward` is the plain detector forward
    (DeformableDETR.forward of `model`).  Returns the prev_features the current-frame
    forward uses (the previous frame's backbone features in training, else the caller's)."""
    if not model.training:
        empty_track_queries(model, targets)
        return prev_features
    if model._matcher is None:
        raise RuntimeError('training the tracking model needs the Hungarian matcher (build_model sets it)')
    prev_targets = [target['prev_target'] for target in targets]
    grad_ctx = torch.enable_grad() if model._backprop_prev_frame else torch.no_grad()
    # the reference runs the previous frame in train mode, so with dropout > 0 it must take
    # the op-for-op path (dropout included) rather than the HIP inference path
    path_ctx = reference_path() if _has_dropout(model) else contextlib.nullcontext()
    with grad_ctx, path_ctx:
        if 'prev_prev_image' in targets[0]:
            for target, prev_target in zip(targets, prev_targets):
                prev_target['prev_target'] = target['prev_prev_target']
            prev_prev_targets = [target['prev_prev_target'] for target in targets]
            prev_prev_out, _, prev_prev_features, _, _ = base_forward([t['prev_prev_image'] for t in targets])
            prev_prev_indices = model._matcher(_without_aux(prev_prev_out), prev_prev_targets)
            add_track_queries_to_targets(model, prev_targets, prev_prev_indices, prev_prev_out, add_false_pos=False)
            prev_out, _, prev_features, _, _ = base_forward([t['prev_image'] for t in targets], prev_targets,
                                                            prev_prev_features)
        else:
            prev_out, _, prev_features, _, _ = base_forward([t['prev_image'] for t in targets])
        # the matcher's indices stay on the host: the sampler consumes them there (the
        # reference moves them to the device, :262-265, and its sampler reads them back)
        with glue_timer():
            prev_indices = model._matcher(_without_aux(prev_out), prev_targets)
        add_track_queries_to_targets(model, targets, prev_indices, prev_out)
    return prev_features

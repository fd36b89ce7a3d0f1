"""Training-path host logic against reference-generated fixtures (tests/golden/make_golden.py
`train`): Hungarian matcher with track queries (matcher.py:112-202), SetCriterion losses
(detr.py:566-870), the seeded track-query sampler (detr_tracking.py:39-218); and the
distributed pieces on a 2-rank gloo group: the criterion's num_boxes all-reduce
(detr.py:841-846) and DDP gradient averaging of train_step (engine.py:124-149)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def _targets_from(d, n_samples, Q):
    targets = []
    for i in range(n_samples):
        t = {k: torch.from_numpy(d[f't{i}_{k}']) for k in
             ('boxes', 'labels', 'track_query_match_ids', 'track_queries_mask', 'track_queries_fal_pos_mask')}
        t['track_query_boxes'] = torch.zeros(int(t['track_queries_mask'].sum()), 4)
        targets.append(t)
    return targets


@pytest.mark.parametrize('focal', [True, False])
def test_matcher_and_criterion_vs_reference(golden_dir, focal):
    from kinet_amd.models.criterion import SetCriterion
    from kinet_amd.models.matcher import HungarianMatcher
    d = _load(golden_dir, 'train_matcher_criterion.npz')
    tag = 'focal' if focal else 'ce'
    outs = [{'pred_logits': torch.from_numpy(d[f'logits{l}']), 'pred_boxes': torch.from_numpy(d[f'boxes{l}'])}
            for l in range(3)]
    outputs = dict(outs[-1], aux_outputs=outs[:-1])
    targets = _targets_from(d, 2, 40)
    matcher = HungarianMatcher(cost_class=1.0, cost_bbox=5.0, cost_giou=2.0, focal_loss=focal,
                               focal_alpha=0.25, focal_gamma=2)
    idx = matcher({k: v for k, v in outputs.items() if k != 'aux_outputs'}, targets)
    for i, (a, b) in enumerate(idx):
        np.testing.assert_array_equal(a.numpy(), d[f'{tag}_match{i}_pred'])
        np.testing.assert_array_equal(b.numpy(), d[f'{tag}_match{i}_tgt'])
    # track queries are forced onto their targets (matcher.py:186-190)
    for t, (a, b) in zip(targets, idx):
        K = int(t['track_queries_mask'].sum())
        fp = t['track_queries_fal_pos_mask'][:K]
        for j in range(K):
            if fp[j]:
                assert j not in a.tolist()
    crit = SetCriterion(20 if focal else 19, matcher=matcher, weight_dict={}, eos_coef=0.1,
                        losses=['labels', 'boxes', 'cardinality'], focal_loss=focal, focal_alpha=0.25,
                        focal_gamma=2, tracking=True, track_query_false_positive_eos_weight=True)
    losses = crit(outputs, targets)
    ref_keys = sorted(k[len(tag) + 6:] for k in d.files if k.startswith(f'{tag}_loss_'))
    assert sorted(losses.keys()) == ref_keys
    for k in ref_keys:
        np.testing.assert_allclose(losses[k].item(), float(d[f'{tag}_loss_{k}']), rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_track_query_sampler_vs_reference(golden_dir, seed):
    """Same global-RNG call sequence as the reference -> the same track queries."""
    from types import SimpleNamespace
    from kinet_amd.models.training import add_track_queries_to_targets
    d = _load(golden_dir, 'train_sampler.npz')
    prev_out = {'pred_boxes': torch.from_numpy(d['prev_boxes']), 'hs_embed': torch.from_numpy(d['prev_hs'])}
    targets, prev_indices = [], []
    for i in range(2):
        targets.append({'track_ids': torch.from_numpy(d[f's{i}_cur_ids']),
                        'prev_target': {'track_ids': torch.from_numpy(d[f's{i}_prev_ids'])}})
        prev_indices.append((torch.from_numpy(d[f's{i}_prev_out_ind']), torch.from_numpy(d[f's{i}_prev_target_ind'])))
    model = SimpleNamespace(_track_query_false_positive_prob=0.1, _track_query_false_negative_prob=0.4, num_queries=30)
    torch.manual_seed(1000 + seed)
    add_track_queries_to_targets(model, targets, prev_indices, prev_out)
    for i, t in enumerate(targets):
        for k in ('track_query_match_ids', 'track_queries_mask', 'track_queries_fal_pos_mask',
                  'track_query_boxes', 'track_query_hs_embeds'):
            np.testing.assert_array_equal(t[k].numpy(), d[f'seed{seed}_s{i}_{k}'], err_msg=f'{k} sample {i}')


# ---- distributed pieces on gloo -----------------------------------------------------------

class _ToyDetector(torch.nn.Module):
    """Stand-in with the detector's output contract (pred_logits / pred_boxes / aux) so the
    criterion + train_step + DDP plumbing runs on CPU."""

    def __init__(self, Q=12, C=5):
        super().__init__()
        self.q = torch.nn.Parameter(torch.randn(Q, 16, generator=torch.Generator().manual_seed(5)))
        self.cls = torch.nn.Linear(16, C)
        self.box = torch.nn.Linear(16, 4)
        torch.nn.init.normal_(self.cls.weight, generator=torch.Generator().manual_seed(6))
        torch.nn.init.normal_(self.box.weight, generator=torch.Generator().manual_seed(7))

    def forward(self, samples, targets):
        h = self.q[None] * samples.mean(dim=(1, 2, 3))[:, None, None]
        out = {'pred_logits': self.cls(h), 'pred_boxes': self.box(h).sigmoid() * 0.5 + 0.25}
        out['aux_outputs'] = [{'pred_logits': out['pred_logits'] * 0.5, 'pred_boxes': out['pred_boxes']}]
        return out, targets


def _toy_batch(rank):
    g = torch.Generator().manual_seed(100 + rank)
    samples = torch.randn(2, 3, 8, 8, generator=g)
    targets = []
    for n in (2 + rank, 3):
        c = torch.rand(n, 2, generator=g) * 0.5 + 0.25
        targets.append({'boxes': torch.cat([c, torch.full((n, 2), 0.1)], -1), 'labels': torch.zeros(n, dtype=torch.long)})
    return samples, targets


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from kinet_amd.models.criterion import SetCriterion
    from kinet_amd.models.matcher import HungarianMatcher
    from kinet_amd.train import reduce_dict, setup_ddp, train_step
    torch.manual_seed(0)
    model = setup_ddp(_ToyDetector(), torch.device('cpu'))
    matcher = HungarianMatcher(cost_class=2.0, cost_bbox=5.0, cost_giou=2.0, focal_loss=True)
    crit = SetCriterion(5, matcher, {'loss_ce': 1.0, 'loss_bbox': 5.0, 'loss_giou': 2.0, 'loss_ce_0': 1.0,
                                     'loss_bbox_0': 5.0, 'loss_giou_0': 2.0}, 0.1, ['labels', 'boxes', 'cardinality'],
                        True, 0.25, 2.0, False, False)
    samples, targets = _toy_batch(rank)
    nb = crit.num_boxes({'x': samples}, targets)
    opt = torch.optim.SGD(model.parameters(), lr=0.0)     # lr 0: keep params, inspect grads
    loss, ld = train_step(model, crit, opt, samples, targets, clip_max_norm=0.0)
    red = reduce_dict({k: v for k, v in ld.items() if k.startswith('loss_')})
    torch.save({'num_boxes': nb, 'grads': {n: p.grad.clone() for n, p in model.module.named_parameters()},
                'loss': loss, 'reduced': {k: v for k, v in red.items()}}, os.path.join(outdir, f'r{rank}.pt'))
    dist.destroy_process_group()


def test_ddp_train_step_gloo(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(os.path.join(tmp_path, f'r{r}.pt'), weights_only=True) for r in range(world)]
    # num_boxes: (5 + 6) summed over ranks / world (detr.py:845-846)
    assert res[0]['num_boxes'] == res[1]['num_boxes'] == pytest.approx((5 + 6) / 2)
    # DDP averaged the gradients: identical on both ranks ...
    for n in res[0]['grads']:
        torch.testing.assert_close(res[0]['grads'][n], res[1]['grads'][n])
    # ... and equal to the mean of the single-process gradients of each rank's batch
    from kinet_amd.models.criterion import SetCriterion
    from kinet_amd.models.matcher import HungarianMatcher
    from kinet_amd.train import weighted_loss
    single = []
    for r in range(world):
        torch.manual_seed(0)
        m = _ToyDetector()
        matcher = HungarianMatcher(cost_class=2.0, cost_bbox=5.0, cost_giou=2.0, focal_loss=True)
        crit = SetCriterion(5, matcher, {'loss_ce': 1.0, 'loss_bbox': 5.0, 'loss_giou': 2.0, 'loss_ce_0': 1.0,
                                         'loss_bbox_0': 5.0, 'loss_giou_0': 2.0}, 0.1, ['labels', 'boxes', 'cardinality'],
                            True, 0.25, 2.0, False, False)
        crit.num_boxes = lambda outputs, targets: (5 + 6) / 2     # the value the group all-reduce gives
        s, t = _toy_batch(r)
        out, t = m(s, t)
        weighted_loss(crit(out, t), crit.weight_dict).backward()
        single.append({n: p.grad.clone() for n, p in m.named_parameters()})
    for n in res[0]['grads']:
        torch.testing.assert_close(res[0]['grads'][n], (single[0][n] + single[1][n]) / 2, rtol=1e-5, atol=1e-6)
    # reduce_dict averages the logged losses over ranks
    for k, v in res[0]['reduced'].items():
        torch.testing.assert_close(v, res[1]['reduced'][k])

"""Checkpoint compatibility (kinet_amd/checkpoint.py) against the reference's resume rules
(src/train.py:166-233) and detector loading (src/track.py:80-87).  Host-only."""
import argparse

import pytest
import torch


def _sd(**shapes):
    g = torch.Generator().manual_seed(0)
    return {k.replace('__', '.'): torch.randn(*s, generator=g) for k, s in shapes.items()}


def test_resume_rules_match_train_py():
    from kinet_amd.checkpoint import resume_state_dict
    model = _sd(norm1__weight=(8,), layers__0__self_attn__in_proj_weight=(12, 8),
                transformer__reference_points__weight=(4, 8), layers__0__linear1__weight=(16, 8),
                layers__0__linear2__weight=(8, 16), input_proj__0__0__weight=(8, 4, 1, 1),
                class_embed__0__weight=(20, 8), same__weight=(3, 3), fresh__weight=(2,))
    ckpt = _sd(norm1__weight=(4,), layers__0__self_attn__in_proj_weight=(6, 4),
               transformer__reference_points__weight=(2, 8), layers__0__linear1__weight=(16, 4),
               layers__0__linear2__weight=(4, 16), input_proj__0__0__weight=(4, 4, 1, 1),
               class_embed__0__weight=(92, 8), same__weight=(3, 3), stale__weight=(5,))
    ckpt = {'detr.' + k: v for k, v in ckpt.items()}            # tracking-wrapper prefix (:175-176)
    logs = []
    out = resume_state_dict(model, ckpt, log=logs.append)
    c = {k[5:]: v for k, v in ckpt.items()}
    assert torch.equal(out['norm1.weight'], c['norm1.weight'].repeat(2))
    assert torch.equal(out['layers.0.self_attn.in_proj_weight'], c['layers.0.self_attn.in_proj_weight'].repeat(2, 2))
    rp = out['transformer.reference_points.weight']
    assert torch.equal(rp[:2], c['transformer.reference_points.weight'])
    assert torch.equal(rp[2:], model['transformer.reference_points.weight'][2:])
    assert torch.equal(out['layers.0.linear1.weight'], model['layers.0.linear1.weight'])       # from scratch
    assert torch.equal(out['layers.0.linear2.weight'], c['layers.0.linear2.weight'].repeat(2, 1))
    assert torch.equal(out['input_proj.0.0.weight'], c['input_proj.0.0.weight'].repeat(2, 1, 1, 1))
    assert torch.equal(out['class_embed.0.weight'], c['class_embed.0.weight'][:20])
    assert torch.equal(out['same.weight'], c['same.weight'])
    assert torch.equal(out['fresh.weight'], model['fresh.weight'])
    assert any('Where is stale.weight' in m for m in logs)
    assert any('Load fresh.weight' in m and 'from scratch' in m for m in logs)


def test_resume_shift_neuron_and_unknown_rule():
    from kinet_amd.checkpoint import resume_state_dict
    model = _sd(class_embed__weight=(5, 3))
    ckpt = _sd(class_embed__weight=(5, 3))
    out = resume_state_dict(model, ckpt, resume_shift_neuron=True, log=lambda m: None)
    c = ckpt['class_embed.weight']
    exp = c.clone()
    exp[:-1] = c[1:]
    exp[-2] = c[0]
    assert torch.equal(out['class_embed.weight'], exp)
    with pytest.raises(NotImplementedError):
        resume_state_dict(_sd(backbone__x=(4,)), _sd(backbone__x=(3,)), log=lambda m: None)


def test_detector_state_dict_like_track_py():
    from kinet_amd.checkpoint import detector_state_dict
    sd = {'detr.a.weight': torch.ones(2), 'detr.track_encoding.w': torch.ones(1), 'b': torch.zeros(1)}
    out = detector_state_dict(sd)
    assert set(out) == {'a.weight', 'b'}


def test_resume_round_trip_through_a_file(tmp_path):
    """A reference-format checkpoint ({'model': 'detr.'-prefixed state, 'args': Namespace,
    'epoch'}) written to disk and resumed into a fresh model reproduces every tensor."""
    from kinet_amd.checkpoint import resume
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    args = load_args('train_deformable', 'train_multi_frame', 'train_tracking', dataset='mot', enc_layers=1,
                     dec_layers=1, num_queries=10)
    torch.manual_seed(1)
    src, _, _ = build_model(args)
    torch.manual_seed(2)
    dst, _, _ = build_model(args)
    path = tmp_path / 'checkpoint.pth'
    torch.save({'model': {'detr.' + k: v for k, v in src.state_dict().items()}, 'epoch': 7,
                'args': argparse.Namespace(lr=2e-4)}, path)
    ck = resume(dst, str(path), log=lambda m: None)
    assert ck['epoch'] == 7 and ck['args'].lr == 2e-4
    for k, v in src.state_dict().items():
        assert torch.equal(dst.state_dict()[k], v), k


def test_load_full_train_py_checkpoint(tmp_path):
    """train.py:322-330 saves model, optimizer, lr_scheduler (MultiStepLR: a Counter of
    milestones), epoch, args, vis_win_names and best_val_stats -- with tracking_eval on
    (cfgs/train.yaml:68) the latter holds numpy.float64 MOTA / IDF1 values (engine.py:343).
    weights_only loading must accept all of it without unpickling code."""
    import numpy as np
    from kinet_amd.checkpoint import load_checkpoint
    m = torch.nn.Linear(3, 2)
    opt = torch.optim.AdamW(m.parameters(), lr=2e-4)
    sched = torch.optim.lr_scheduler.MultiStepLR(opt, [40, 50])
    ck = {'model': {'detr.' + k: v for k, v in m.state_dict().items()}, 'optimizer': opt.state_dict(),
          'lr_scheduler': sched.state_dict(), 'epoch': 7, 'args': argparse.Namespace(lr=2e-4, hidden_dim=288),
          'vis_win_names': {'train_loss': 'w1', 'val_mota': 'w2'},
          'best_val_stats': [np.float64(0.61), np.float64(0.70), np.float32(0.5), np.int64(12)]}
    p = tmp_path / 'checkpoint.pth'
    torch.save(ck, p)
    got = load_checkpoint(str(p))
    assert got['epoch'] == 7 and got['args'].hidden_dim == 288
    assert got['best_val_stats'][0] == np.float64(0.61) and isinstance(got['best_val_stats'][3], np.int64)
    assert dict(got['lr_scheduler']['milestones']) == {40: 1, 50: 1}
    assert torch.equal(got['model']['detr.weight'], m.weight)
    # the allow-list is scoped to the call, not registered process-wide
    with pytest.raises(Exception):
        torch.load(p, weights_only=True)


def test_load_checkpoint_refuses_code(tmp_path):
    import os
    from kinet_amd.checkpoint import load_checkpoint

    class Evil:
        def __reduce__(self):
            return (os.getcwd, ())
    p = tmp_path / 'evil.pth'
    torch.save({'model': {}, 'x': Evil()}, p)
    with pytest.raises(Exception):
        load_checkpoint(str(p))

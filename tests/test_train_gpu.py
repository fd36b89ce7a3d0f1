"""Training step of the tracking detector on the GPU vs the reference (config-4 structure
at a small size, tests/golden/train_step_small.npz): two-pass forward with the seeded
track-query sampler, Hungarian matching, SetCriterion with aux losses, backward through
the HIP MSDeformAttn forward/backward kernels.  fp32, dropout 0."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _build(golden_dir):
    sys.path.insert(0, golden_dir)
    from weights import make_state_dict
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    args = load_args('train_deformable', 'train_multi_frame', 'train_tracking', dataset='mot', dropout=0.0,
                     num_queries=40, enc_layers=2, dec_layers=3, device='cuda')
    model, criterion, _ = build_model(args)
    keys = [ln.split() for ln in open(os.path.join(golden_dir, 'train_step_small.keys.txt'))]
    model.load_state_dict(make_state_dict({k[0]: [int(s) for s in k[1:]] for k in keys}, seed=71))
    return args, model.cuda().train(), criterion


def _batch(d):
    imgs, targets = [], []
    for i in range(2):
        imgs.append(torch.from_numpy(d[f'img{i}']).cuda())
        t = {'boxes': torch.from_numpy(d[f't{i}_boxes']).cuda(),
             'labels': torch.zeros(len(d[f't{i}_boxes']), dtype=torch.long).cuda(),
             'track_ids': torch.from_numpy(d[f't{i}_track_ids']).cuda(),
             'prev_image': torch.from_numpy(d[f'prev_img{i}']).cuda(),
             'prev_target': {'boxes': torch.from_numpy(d[f't{i}_prev_boxes']).cuda(),
                             'labels': torch.zeros(len(d[f't{i}_prev_boxes']), dtype=torch.long).cuda(),
                             'track_ids': torch.from_numpy(d[f't{i}_prev_track_ids']).cuda()}}
        targets.append(t)
    return imgs, targets


@pytest.fixture(params=['highest', 'high'])
def matmul_precision(request):
    # 'high': every f32 GEMM / conv / weight-gradient GEMM as three bf16 MFMA passes
    # (KINET_F32_X3) -- the training benchmark's setting; same tolerances as exact f32
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(request.param)
    yield request.param
    torch.set_float32_matmul_precision(prev)


def test_train_step_matches_reference(golden_dir, matmul_precision):
    from kinet_amd.models import nested_tensor_from_tensor_list
    from kinet_amd.train import weighted_loss
    d = np.load(os.path.join(golden_dir, 'train_step_small.npz'))
    args, model, criterion = _build(golden_dir)
    imgs, targets = _batch(d)
    torch.manual_seed(73)
    out, targets, *_ = model(nested_tensor_from_tensor_list(imgs), targets)
    # the seeded sampler drew the same track queries as the reference
    for i, t in enumerate(targets):
        np.testing.assert_array_equal(t['track_query_match_ids'].cpu().numpy(), d[f't{i}_track_query_match_ids'])
        np.testing.assert_array_equal(t['track_queries_fal_pos_mask'].cpu().numpy(),
                                      d[f't{i}_track_queries_fal_pos_mask'])
    np.testing.assert_allclose(out['pred_logits'].detach().cpu().numpy(), d['pred_logits'], atol=1e-3)
    np.testing.assert_allclose(out['pred_boxes'].detach().cpu().numpy(), d['pred_boxes'], atol=1e-3)
    losses = criterion(out, targets)
    total = weighted_loss(losses, criterion.weight_dict)
    for k, v in losses.items():
        np.testing.assert_allclose(v.item(), float(d[f'loss_{k}']), rtol=1e-3, atol=1e-4, err_msg=k)
    np.testing.assert_allclose(total.item(), float(d['loss_total']), rtol=1e-3)
    total.backward()
    params = dict(model.named_parameters(remove_duplicate=False))
    bad = []
    for k in d.files:
        if not k.startswith('grad:'):
            continue
        g = params[k[5:]].grad
        assert g is not None, k
        ref = torch.from_numpy(d[k])
        err = (g.cpu() - ref).abs().max().item()
        print(f'[grad] {matmul_precision} {k}: max err {err:.3e} rel {err / (ref.abs().max().item() + 1e-12):.3e}')
        # gradients below the encoder pass the MSDA location derivative, which is one-sided at
        # integer pixel coordinates (a 1-ulp location difference can flip it), and then ~10
        # conv layers: the backbone's deepest trainable weight lands at ~2e-3 of its scale
        # (heads / decoder: ~1e-7 .. 1e-6; encoder / input_proj: ~1.5e-4; measured on MI355X)
        rel = 5e-3 if 'backbone' in k else 2e-3
        if matmul_precision != 'highest' and ('backbone' in k or 'sampling_offsets' in k):
            # bf16x3 products move the forward by ~1e-5 relative, enough to carry a few sampling
            # locations across a pixel knot; measured 5.7e-3 (encoder sampling_offsets) and
            # 4.2e-3 (backbone) of scale vs <= 2e-6 on the exact path, everything else <= 4e-4
            rel = 1e-2
        if err > rel * ref.abs().max().item() + 1e-5:
            bad.append((k, err, ref.abs().max().item()))
    assert not bad, bad


def test_train_steps_reduce_loss(golden_dir):
    """A few AdamW steps (train.py param groups, clip 0.1) on one synthetic MOT batch."""
    from kinet_amd.train import build_optimizer, synthetic_mot_batch, train_step
    args, model, criterion = _build(golden_dir)
    g = torch.Generator().manual_seed(3)
    samples, targets = synthetic_mot_batch(2, 96, 128, torch.device('cuda'), g, num_boxes=(4, 8))
    opt = build_optimizer(model, args)
    assert [len(pg['params']) for pg in opt.param_groups][1] > 0          # backbone group (layer2-4)
    losses = []
    for _ in range(4):
        torch.manual_seed(5)
        tg = [dict(t, prev_target=dict(t['prev_target'])) for t in targets]
        loss, _ = train_step(model, criterion, opt, samples, tg, args.clip_max_norm)
        losses.append(loss.item())
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0], losses

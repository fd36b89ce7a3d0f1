"""Parity at the BENCHMARKED sizes (the timed workload was pinned only at
128x160).  Fixtures come from the reference model run in the build container
(tests/golden/make_golden.py `full` / `config5`) with the same name-seeded weights; the
frames are regenerated here from CPU generator seeds, so only outputs are committed.

  * config 2 (cfgs/train_deformable.yaml): one 3x800x1333 frame.
      - HIP fp32 vs reference: pred_logits / pred_boxes / hs_embed / aux / memory within
        1e-3 abs (the BASELINE north_star gate).
      - HIP bf16 (the mode bench.py times) vs HIP fp32, per-tensor max-abs bounds BF16_TOL.
      - HIP bf16 vs the REFERENCE's outputs directly (closing the chain timed kernels ->
        reference): within BF16_TOL + 1e-3 per tensor (the fp32 gate plus the 16-bit bound).
  * config 5 (cfgs/train_full_res.yaml: ResNet-101, d=288, 500 queries, separate
    per-frame encoders, 8-level decoder, tracking step with prev_features + K track
    queries): at 96x128 and at 1080x1920.
      - HIP fp32 vs reference within 1e-3 abs, both frames of the step.
      - HIP fp16 (the config's compute dtype) vs HIP fp32, per-tensor bounds F16_TOL, and vs
        the reference's outputs within F16_TOL + 1e-3.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-3
# 16-bit compute vs the fp32 HIP path on the same frame and weights: max |diff| per tensor.
# Logits/hs are O(1..10) (random-init weights keep activations O(1)); boxes are in [0, 1].
# Measured on MI355X on the round-5 timed path (records sampling with 1/256-px locations, folded
# bottleneck pairs, the stem from the f32 image; config 5 on the split head_dim-36 strip kernel),
# profiles/r05b_fullsize_tolerances.log: bf16 0.1945 / 0.0182 / 0.2878, fp16 0.0509 / 0.0062 /
# 0.0813 (round 2: bf16 0.188 / 0.0167 / 0.192, fp16 0.054 / 0.0038 / 0.058); the bounds are
# ~1.6x the measured max.
BF16_TOL = {'pred_logits': 0.3, 'pred_boxes': 0.03, 'hs_embed': 0.45}
F16_TOL = {'pred_logits': 0.08, 'pred_boxes': 0.01, 'hs_embed': 0.13}


def _frame(seed, h, w):
    return torch.randn(3, h, w, generator=torch.Generator().manual_seed(seed))


def _build(golden_dir, keyfile, seed, *cfgs, **over):
    from weights import make_state_dict
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    model, _, _ = build_model(load_args(*cfgs, **over))
    shapes = {}
    for ln in open(os.path.join(golden_dir, keyfile)):
        k, *s = ln.split()
        shapes[k] = [int(x) for x in s]
    model.load_state_dict(make_state_dict(shapes, seed=seed))
    return model.cuda().eval()


def _check_outputs(out, d, prefix='', n_aux=5):
    np.testing.assert_allclose(out['pred_logits'].float().cpu().numpy(), d['pred_logits' + prefix], atol=TOL, rtol=0)
    np.testing.assert_allclose(out['pred_boxes'].float().cpu().numpy(), d['pred_boxes' + prefix], atol=TOL, rtol=0)
    np.testing.assert_allclose(out['hs_embed'].float().cpu().numpy(), d['hs_embed' + prefix], atol=TOL, rtol=0)
    if prefix == '':
        for i, aux in enumerate(out['aux_outputs'][:n_aux]):
            np.testing.assert_allclose(aux['pred_logits'].cpu().numpy(), d[f'aux{i}_logits'], atol=TOL, rtol=0)
            np.testing.assert_allclose(aux['pred_boxes'].cpu().numpy(), d[f'aux{i}_boxes'], atol=TOL, rtol=0)


def _max_diffs(a, b):
    return {k: (a[k].float() - b[k].float()).abs().max().item() for k in ('pred_logits', 'pred_boxes', 'hs_embed')}


def _report(tag, diffs):
    print(f'[fullsize] {tag}: ' + ' '.join(f'{k}={v:.4g}' for k, v in diffs.items()))


# ---------------------------------------------------------------------------------- config 2
@pytest.fixture(scope='module')
def config2_full(golden_dir):
    d = dict(np.load(os.path.join(golden_dir, 'detr_config2_full.npz')))
    model = _build(golden_dir, 'detr_config2_small.keys.txt', 21, 'train_deformable')
    img = _frame(2002, 800, 1333).cuda()
    return d, model, img


def _fwd(model, imgs, dtype, targets=None, prev=None):
    model.set_compute_dtype(dtype)
    try:
        with torch.no_grad():
            r = model(imgs, targets, prev) if targets is not None or prev is not None else model(imgs)
        torch.cuda.synchronize()
        return r
    finally:
        model.set_compute_dtype(torch.float32)


def test_config2_full_fp32_parity(config2_full):
    d, model, img = config2_full
    out, _, _, memory, _ = _fwd(model, [img], torch.float32)
    _check_outputs(out, d)
    for i, m in enumerate(memory):
        np.testing.assert_allclose(m[:, :, ::7, ::7].float().cpu().numpy(), d[f'memory{i}_sub'], atol=TOL, rtol=0)


def test_config2_full_bf16_vs_fp32(config2_full):
    d, model, img = config2_full
    ref = _fwd(model, [img], torch.float32)[0]
    got = _fwd(model, [img], torch.bfloat16)[0]
    diffs = _max_diffs(got, ref)
    _report('config2 800x1333 bf16 vs HIP fp32', diffs)
    for k, tol in BF16_TOL.items():
        assert diffs[k] < tol, (k, diffs[k], tol)
    # and the boxes the bench produces stay boxes
    assert torch.isfinite(got['pred_boxes']).all() and (got['pred_boxes'] >= 0).all() and (got['pred_boxes'] <= 1).all()


def _vs_reference(out, d, prefix=''):
    """max / mean |HIP - reference| per tensor against the fixture."""
    r = {}
    for k in ('pred_logits', 'pred_boxes', 'hs_embed'):
        diff = np.abs(out[k].float().cpu().numpy() - d[k + prefix])
        r[k] = (float(diff.max()), float(diff.mean()))
    return r


def test_config2_full_bf16_vs_reference(config2_full):
    """The timed bf16 path (records sampler, bf16 GEMM / conv kernels, 1/256-px sampling
    locations) against the reference model's own fp32 outputs at 800x1333: per-tensor max |diff|
    within BF16_TOL + TOL (the bf16-vs-HIP-fp32 bound plus the fp32 gate)."""
    d, model, img = config2_full
    got = _fwd(model, [img], torch.bfloat16)[0]
    r = _vs_reference(got, d)
    print('[fullsize] config2 800x1333 bf16 vs reference: ' +
          ' '.join(f'{k}=max {a:.4g} mean {m:.3g}' for k, (a, m) in r.items()))
    for k, tol in BF16_TOL.items():
        assert r[k][0] < tol + TOL, (k, r[k], tol + TOL)


# ---------------------------------------------------------------------------------- config 5
def _config5_model(golden_dir):
    model = _build(golden_dir, 'config5.keys.txt', 81, 'train_deformable', 'train_multi_frame', 'train_tracking',
                   'train_full_res', dataset='mot', backbone='resnet101')
    model.tracking()
    return model


def _config5_step(model, f0, f1, top, dtype):
    out0, _, feat0, _, _ = _fwd(model, [f0], dtype)
    target = {'track_query_hs_embeds': out0['hs_embed'][0, top].float(),
              'track_query_boxes': out0['pred_boxes'][0, top].float()}
    out1 = _fwd(model, [f1], dtype, [target], feat0)[0]
    return out0, out1


@pytest.fixture(scope='module')
def config5_model(golden_dir):
    return _config5_model(golden_dir)


@pytest.mark.parametrize('tag,hw', [('small', (96, 128)), ('full', (1080, 1920))])
def test_config5_fp32_parity(golden_dir, config5_model, tag, hw):
    d = dict(np.load(os.path.join(golden_dir, f'config5_{tag}.npz')))
    f0, f1 = _frame(5001, *hw).cuda(), _frame(5002, *hw).cuda()
    top = torch.from_numpy(d['top_idx']).cuda()
    out0, out1 = _config5_step(config5_model, f0, f1, top, torch.float32)
    _check_outputs(out0, d, prefix='0')
    _check_outputs(out1, d)


def test_config5_full_fp16_vs_fp32(golden_dir, config5_model):
    d = dict(np.load(os.path.join(golden_dir, 'config5_full.npz')))
    f0, f1 = _frame(5001, 1080, 1920).cuda(), _frame(5002, 1080, 1920).cuda()
    top = torch.from_numpy(d['top_idx']).cuda()   # same track-query selection in both dtypes
    _, ref = _config5_step(config5_model, f0, f1, top, torch.float32)
    _, got = _config5_step(config5_model, f0, f1, top, torch.float16)
    diffs = _max_diffs(got, ref)
    _report('config5 1080x1920 fp16 vs HIP fp32', diffs)
    for k, tol in F16_TOL.items():
        assert diffs[k] < tol, (k, diffs[k], tol)


def test_config5_full_fp16_vs_reference(golden_dir, config5_model):
    """config 5's timed fp16 path against the reference model's fp32 outputs at 1080x1920
    (both frames of the tracking step): within F16_TOL + TOL per tensor."""
    d = dict(np.load(os.path.join(golden_dir, 'config5_full.npz')))
    f0, f1 = _frame(5001, 1080, 1920).cuda(), _frame(5002, 1080, 1920).cuda()
    top = torch.from_numpy(d['top_idx']).cuda()
    out0, out1 = _config5_step(config5_model, f0, f1, top, torch.float16)
    for tag, out, prefix in (('frame 0', out0, '0'), ('frame 1', out1, '')):
        r = _vs_reference(out, d, prefix)
        print(f'[fullsize] config5 1080x1920 fp16 vs reference, {tag}: ' +
              ' '.join(f'{k}=max {a:.4g} mean {m:.3g}' for k, (a, m) in r.items()))
        for k, tol in F16_TOL.items():
            assert r[k][0] < tol + TOL, (tag, k, r[k], tol + TOL)

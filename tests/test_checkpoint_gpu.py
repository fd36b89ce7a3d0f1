"""SURVEY.md §8(f)4 on the GPU: a checkpoint in the reference's own format (the train.py:322-330
dict, 'detr.'-prefixed state keys + a track_encoding entry as track.py:80-87 expects, the
reference's AdamW / MultiStepLR states, argparse args, numpy best_val_stats), written from the
reference-built config-3 model by tests/golden/make_golden.py `checkpoint`, is loaded through
kinet_amd.checkpoint exactly as track.py loads an object detector (build_model(checkpoint args)
-> detector_state_dict -> load_state_dict) and the detector's outputs match the reference
model's on a frame pair (tracking step with track queries) within 1e-3 (fp32).

The committed skeleton holds the dict with each model tensor replaced by its shape; the
tensors are regenerated here from (key, shape, seed) by weights.py -- the same generator
make_golden.py loaded into the reference model -- and the full dict is torch.saved again, so
the file read back is byte-for-byte a torch.save of the reference's checkpoint dict."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _write_full_checkpoint(golden_dir, path):
    from weights import make_tensor
    from kinet_amd.checkpoint import load_checkpoint
    sk = load_checkpoint(os.path.join(golden_dir, 'checkpoint_skeleton.pth'))
    seed = sk['model']['seed']
    state = {k: make_tensor(k[len('detr.'):], shape, seed) for k, shape in sk['model']['shapes'].items()}
    state.update({k: torch.zeros(shape) for k, shape in sk['model']['extra'].items()})
    ckpt = dict(sk, model=state)
    torch.save(ckpt, path)
    return ckpt


def test_reference_checkpoint_drives_detector(golden_dir, tmp_path):
    from argparse import Namespace
    from kinet_amd.checkpoint import detector_state_dict, load_checkpoint
    from kinet_amd.models import build_model
    from kinet_amd.models.misc import nested_tensor_from_tensor_list
    path = str(tmp_path / 'checkpoint.pth')
    _write_full_checkpoint(golden_dir, path)
    ckpt = load_checkpoint(path)                                   # weights_only, numpy / Namespace allowed
    assert ckpt['epoch'] == 7 and isinstance(ckpt['best_val_stats'][0], np.float64)
    assert len(ckpt['optimizer']['param_groups']) == 3 and ckpt['lr_scheduler']['last_epoch'] == 1
    args = Namespace(**dict(vars(ckpt['args']), device='cuda'))    # track.py builds from the run's args
    model, _, post = build_model(args)
    model.load_state_dict(detector_state_dict(ckpt['model']))     # strict: every key mapped
    model = model.cuda().eval()
    model.tracking()
    d = dict(np.load(os.path.join(golden_dir, 'checkpoint.npz')))
    f0, f1 = torch.from_numpy(d['frame0']).cuda(), torch.from_numpy(d['frame1']).cuda()
    with torch.no_grad():
        out0, _, feat0, _, _ = model(nested_tensor_from_tensor_list([f0]))
        top = torch.from_numpy(d['top_idx']).cuda()
        target = {'track_query_hs_embeds': out0['hs_embed'][0, top], 'track_query_boxes': out0['pred_boxes'][0, top]}
        out1 = model(nested_tensor_from_tensor_list([f1]), [target], feat0)[0]
    torch.cuda.synchronize()
    for k, got in (('pred_logits0', out0['pred_logits']), ('pred_boxes0', out0['pred_boxes']),
                   ('pred_logits1', out1['pred_logits']), ('pred_boxes1', out1['pred_boxes']),
                   ('hs_embed1', out1['hs_embed'])):
        np.testing.assert_allclose(got.cpu().numpy(), d[k], atol=TOL, rtol=0, err_msg=k)


def test_reference_checkpoint_resume_into_training_model(golden_dir, tmp_path):
    """train.py:166-233 resume of the same checkpoint into the config-4 training model
    (identical shapes: every tensor taken from the checkpoint, no rule fires)."""
    from kinet_amd.checkpoint import resume
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    path = str(tmp_path / 'checkpoint.pth')
    ckpt = _write_full_checkpoint(golden_dir, path)
    model, _, _ = build_model(load_args('train_deformable', 'train_multi_frame', 'train_tracking', dataset='mot',
                                        device='cuda'))
    logs = []
    back = resume(model, path, log=logs.append)
    assert back['epoch'] == 7
    sd = model.state_dict()
    for k, v in ckpt['model'].items():
        if 'track_encoding' in k:
            continue
        assert torch.equal(sd[k[len('detr.'):]], v), k
    assert not any('from scratch' in m for m in logs)

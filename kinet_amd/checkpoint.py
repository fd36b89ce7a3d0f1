"""Checkpoint compatibility with the reference's TrackFormer / KineT checkpoints (SURVEY.md
§8(f)4): load a reference `checkpoint.pth` into kinet_amd's model, whose state_dict keys and
shapes equal the reference's (tests/test_host_cpu.py pins the key lists).

  * load_checkpoint(path)                 torch.load(map_location='cpu') as train.py:171 /
                                          track.py:73, but never executing pickled code
                                          (weights_only=True; argparse.Namespace `args`
                                          entries allowed)
  * detector_state_dict(ckpt['model'])    track.py:80-87: strip the 'detr.' prefix of tracking
                                          wrappers, drop 'track_encoding' keys
  * resume_state_dict(model_sd, ckpt_sd)  train.py:172-233: the shape-adapting resume rules
                                          (norm x2, attention x2 per dim, reference_points
                                          [:2], linear1 / query_embed from scratch, linear2 /
                                          input_proj x2 along dim 0, class_embed first 20
                                          rows, optional class-neuron shift)
  * resume(model, path, ...)              the two above + model.load_state_dict
"""
import argparse

import torch


def _safe_globals():
    """The non-tensor types a reference checkpoint holds (train.py:322-330): the argparse
    `args`, and numpy scalars in `best_val_stats` (MOTA / IDF1 from the motmetrics summary,
    engine.py:343) -- numpy.float64 etc. pickle as numpy's `scalar` reconstructor plus a dtype
    object of one of numpy's DType classes.  Data-only reconstructors, no code."""
    import numpy as np
    try:
        from numpy._core.multiarray import scalar
    except ImportError:   # pragma: no cover (numpy < 2)
        from numpy.core.multiarray import scalar
    dts = {type(np.dtype(t)) for t in (np.float16, np.float32, np.float64, np.int8, np.int16, np.int32, np.int64,
                                       np.uint8, np.uint16, np.uint32, np.uint64, np.bool_)}
    return [argparse.Namespace, scalar, np.dtype] + sorted(dts, key=lambda c: c.__name__)


def load_checkpoint(path, map_location='cpu'):
    """The checkpoint dict ('model', and optionally 'optimizer', 'lr_scheduler', 'epoch',
    'args', 'vis_win_names', 'best_val_stats').  weights_only=True with a scoped allow-list
    (torch.serialization.safe_globals, not the process-wide registry)."""
    with torch.serialization.safe_globals(_safe_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def strip_detr_prefix(state_dict):
    """train.py:175-176 / track.py:83-86: keys of a tracking wrapper's inner `detr` module."""
    return {k.replace('detr.', ''): v for k, v in state_dict.items()}


def detector_state_dict(state_dict):
    """track.py:83-86: the object detector's state for tracking (no track_encoding keys)."""
    return {k.replace('detr.', ''): v for k, v in state_dict.items() if 'track_encoding' not in k}


def resume_state_dict(model_state_dict, checkpoint_state_dict, resume_shift_neuron=False, log=print):
    """train.py:172-233.  model_state_dict: the model's current state (keys and target shapes);
    checkpoint_state_dict: checkpoint['model'].  Returns the dict to load_state_dict."""
    ckpt = strip_detr_prefix(checkpoint_state_dict)
    for k, v in ckpt.items():
        if k not in model_state_dict:
            log(f'Where is {k} {tuple(v.shape)}?')
    out = {}
    for k, v in model_state_dict.items():
        if k not in ckpt:
            value = v
            log(f'Load {k} {tuple(v.shape)} from scratch.')
        elif v.shape != ckpt[k].shape:
            cv = ckpt[k]
            nd = len(cv.shape)
            if 'norm' in k:
                value = cv.repeat(2)
            elif 'multihead_attn' in k or 'self_attn' in k:
                value = cv.repeat(nd * (2,))
            elif 'reference_points' in k and cv.shape[0] * 2 == v.shape[0]:
                value = v.clone()
                value[:2] = cv.clone()
            elif 'linear1' in k or 'query_embed' in k:
                out[k] = v
                log(f'Load {k} {tuple(v.shape)} from scratch.')
                continue
            elif 'linear2' in k or 'input_proj' in k:
                value = cv.repeat((2,) + (nd - 1) * (1,))
            elif 'class_embed' in k:
                value = cv[list(range(0, 20))]          # person + the first 19 classes (:213-219)
            else:
                raise NotImplementedError(f'No rule for {k} with shape {v.shape}.')
            log(f'Load {k} {tuple(v.shape)} from resume model {tuple(cv.shape)}.')
        elif resume_shift_neuron and 'class_embed' in k:
            cv = ckpt[k]
            value = cv.clone()
            value[:-1] = cv[1:].clone()
            value[-2] = cv[0].clone()
            log(f'Load {k} {tuple(v.shape)} from resume model and shift class embed neurons to start with '
                'label=0 at neuron=0.')
        else:
            value = ckpt[k]
        out[k] = value
    return out


def resume(model, path, resume_shift_neuron=False, log=print):
    """train.py:167-233 for a local checkpoint: load, adapt, load_state_dict.  Returns the
    checkpoint dict (optimizer / lr_scheduler / epoch entries for the caller, train.py:235-256)."""
    ckpt = load_checkpoint(path)
    m = model.module if hasattr(model, 'module') else model
    m.load_state_dict(resume_state_dict(m.state_dict(), ckpt['model'], resume_shift_neuron, log))
    return ckpt

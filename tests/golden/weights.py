"""Deterministic, name-keyed parameter generator shared by the golden-fixture
generator (which loads it into the reference model) and the tests (which load it
into kinet_amd's model).  Every tensor depends only on (seed, state_dict key, shape),
so fixtures need not carry the ~40 M weights of a full Deformable-DETR: the GPU box
regenerates bit-identical weights from the key list.

Value ranges are chosen to keep activations O(1) through ResNet + 6/6 transformer
layers with non-trivial (query-dependent, partly out-of-bounds) sampling offsets.
"""
import zlib

import numpy as np
import torch


def _rng(seed, name):
    return np.random.default_rng((zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)) & 0xFFFFFFFF)


def canonical(name):
    """Shared modules appear under two keys (deformable_detr.py:103 aliases the box
    heads into the decoder); give both keys the same tensor."""
    for head in ('bbox_embed', 'class_embed'):
        name = name.replace('transformer.decoder.' + head, head)
    return name


def make_tensor(name, shape, seed=0):
    shape = tuple(int(s) for s in shape)
    name = canonical(name)
    r = _rng(seed, name)
    n = len(shape)
    leaf = name.rsplit('.', 1)[-1]
    if leaf == 'running_mean':
        a = r.normal(0.0, 0.1, shape)
    elif leaf == 'running_var':
        a = r.uniform(0.5, 1.5, shape)
    elif n == 1 and 'backbone' in name and leaf == 'weight':            # FrozenBatchNorm2d
        a = r.uniform(0.5, 1.0, shape)
    elif n == 1 and 'backbone' in name and leaf == 'bias':
        a = r.normal(0.0, 0.1, shape)
    elif n == 1 and leaf == 'weight':                                    # LayerNorm / GroupNorm
        a = r.uniform(0.5, 1.5, shape)
    elif n == 1 and ('norm' in name or '.1.bias' in name) and leaf == 'bias':
        a = r.normal(0.0, 0.1, shape)
    elif 'level_embed' in name or 'query_embed' in name:
        a = r.normal(0.0, 1.0, shape)
    elif n == 4:                                                         # conv, kaiming normal
        fan_in = shape[1] * shape[2] * shape[3]
        a = r.normal(0.0, np.sqrt(2.0 / fan_in), shape)
    elif n == 2:                                                         # linear, xavier uniform
        fan_out, fan_in = shape
        lim = np.sqrt(6.0 / (fan_in + fan_out))
        a = r.uniform(-lim, lim, shape)
    elif 'sampling_offsets.bias' in name:
        a = r.normal(0.0, 2.0, shape)
    elif n == 1:
        a = r.normal(0.0, 0.02, shape)
    else:
        a = r.normal(0.0, 0.02, shape)
    return torch.from_numpy(np.asarray(a, dtype=np.float32))


def make_state_dict(shapes: dict, seed=0):
    """shapes: {key: shape}; returns {key: fp32 tensor}."""
    return {k: make_tensor(k, s, seed) for k, s in shapes.items()}


def randomize(module: torch.nn.Module, seed=0):
    sd = module.state_dict()
    new = make_state_dict({k: v.shape for k, v in sd.items()}, seed)
    module.load_state_dict(new)
    return module

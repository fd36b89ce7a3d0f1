"""CPU-only checks of the host side: the C-ABI library exports every declared symbol,
the model's state_dict keys/shapes equal the reference's, the config values equal the
reference YAMLs, and host utilities (postprocess) reproduce the reference fixtures."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(REPO, 'include', '*.h')):
        src = open(h).read()
        src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
        names |= set(re.findall(r'\b(kinet_[a-z0-9_]+)\s*\(', src))
    return names


def test_library_exports_every_declared_symbol():
    from kinet_amd import _native
    lib = _native.lib()
    declared = _declared_symbols()
    assert len(declared) >= 15
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    assert b'gfx950' in lib.kinet_version()


def _check_library_matches_sources():
    from kinet_amd import _native
    from kinet_amd.build import source_hash
    ver = _native.lib().kinet_version().decode()
    assert ver.endswith('src ' + source_hash()), (ver, source_hash())


def test_library_built_from_these_sources():
    """kinet_version() embeds the hash of csrc/ + include/ it was compiled from."""
    _check_library_matches_sources()


@pytest.mark.gpu
def test_library_built_from_these_sources_on_gpu_box():
    """Same check in the GPU tier: the .so the box loads was built from the shipped sources."""
    _check_library_matches_sources()


def test_ctypes_signatures_cover_declarations():
    from kinet_amd import _native
    assert _declared_symbols() <= set(_native._SIGS)


def test_ops_refuse_cpu_tensors():
    import kinet_amd  # noqa: F401
    import MultiScaleDeformableAttention as M
    v = torch.zeros(1, 4, 1, 4)
    with pytest.raises(RuntimeError):
        M.ms_deform_attn_forward(v, torch.tensor([[2, 2]]), torch.zeros(1, 1, 1, 1, 1, 2), torch.zeros(1, 1, 1, 1, 1), 1)


def _keys(golden_dir, name):
    out = {}
    for ln in open(os.path.join(golden_dir, name)):
        k, *s = ln.split()
        out[k] = tuple(int(x) for x in s)
    return out


@pytest.mark.parametrize('fixture,cfgs,over', [
    ('detr_config2_small.keys.txt', ('train_deformable',), {}),
    ('detr_tracking_mf_small.keys.txt', ('train_deformable', 'train_multi_frame', 'train_tracking'), {'dataset': 'mot'}),
])
def test_state_dict_matches_reference(golden_dir, fixture, cfgs, over):
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    ref = _keys(golden_dir, fixture)
    model, _, post = build_model(load_args(*cfgs, **over))
    mine = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    assert mine == ref
    assert 'bbox' in post


@pytest.mark.skipif(not os.path.isdir('/root/reference/cfgs'), reason='reference configs only in the build container')
def test_config_values_match_reference_yaml():
    import yaml
    from kinet_amd.models.config import DEFAULTS, NAMED
    with open('/root/reference/cfgs/train.yaml') as f:
        base = yaml.safe_load(f)
    for k, v in DEFAULTS.items():
        if k in base:
            assert base[k] == v, k
    for name, vals in NAMED.items():
        with open(f'/root/reference/cfgs/{name}.yaml') as f:
            y = yaml.safe_load(f)
        for k, v in vals.items():
            assert y[k] == v, (name, k)


def test_postprocess_matches_reference(golden_dir):
    from kinet_amd.models import DeformablePostProcess
    d = np.load(os.path.join(golden_dir, 'postprocess_matcher.npz'))
    res = DeformablePostProcess()({'pred_logits': torch.from_numpy(d['logits']),
                                   'pred_boxes': torch.from_numpy(d['boxes'])}, torch.from_numpy(d['sizes']))
    for i, r in enumerate(res):
        for k, v in r.items():
            np.testing.assert_allclose(v.numpy(), d[f'post{i}_{k}'], atol=1e-5)


def test_nested_tensor_padding_and_sizes():
    from kinet_amd.models import nested_tensor_from_tensor_list
    a, b = torch.randn(3, 10, 12), torch.randn(3, 8, 14)
    nt = nested_tensor_from_tensor_list([a, b])
    assert nt.tensors.shape == (2, 3, 10, 14) and nt.sizes == ((10, 12), (8, 14))
    assert nt.mask[0, :, 12:].all() and not nt.mask[0, :, :12].any()
    assert nt.mask[1, 8:].all() and not nt.mask[1, :8, :14].any()
    assert torch.equal(nt.tensors[1, :, :8, :14], b)


def test_track_reset_last_pos_compat_switch():
    """Track.reset_last_pos: by default the relative-position history survives a
    re-identification; with the reference-compatibility switch it is cleared as in the
    reference (tracker.py:1120-1124), whose next repeat_last_pos then raises IndexError."""
    from kinet_amd.tracker import Track
    t = Track(torch.tensor([0., 0., 2., 2.]), 0.9, 1, torch.zeros(4), 0, pos_rel=torch.tensor([0., 0., .1, .1]))
    t.reset_last_pos()
    t.repeat_last_pos()
    assert len(t.last_pos_relative) == 2
    t.reset_last_pos(clear_relative=True)
    assert len(t.last_pos_relative) == 0
    with pytest.raises(IndexError):
        t.repeat_last_pos()


def test_train_glue_entry_points_validate_arguments():
    """The training-glue C ABI (include/kinet_grad.h, csrc/train_ops.hip) rejects bad arguments
    with KINET_ERR_ARG and a message before touching the device (no GPU needed)."""
    from kinet_amd import _native
    L = _native.lib()
    fake = 4096   # never dereferenced: every call below fails validation first

    def err(rc):
        assert rc != 0
        return L.kinet_last_error().decode()

    assert 'p must be in [0, 1)' in err(L.kinet_dropout_add_layernorm(fake, fake, fake, fake, fake, 10, 288, 1e-5, 1.0,
                                                                       fake, None))
    assert 'd must be in [1, 1024]' in err(L.kinet_dropout_add_layernorm(fake, fake, fake, fake, fake, 10, 2048, 1e-5,
                                                                         0.1, fake, None))
    assert 'bad arguments' in err(L.kinet_dropout_act(fake, fake, 64, 1, 0.5, None, None))   # p > 0 needs a seed
    assert 'bad arguments' in err(L.kinet_msda_prep(fake, 384, fake, fake, None, fake, fake, 10, 8, 4, 4, 3, None))
    assert 'power of two' in err(L.kinet_msda_prep_backward(fake, fake, fake, fake, 288, fake, fake, fake, None, 10, 3,
                                                            4, 4, 2, None))
    assert 'bad arguments' in err(L.kinet_inverse_sigmoid(None, fake, 10, 1e-5, None))

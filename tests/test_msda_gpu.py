"""GPU parity of the HIP MSDeformAttn operator (through the C-ABI drop-in module) against
the reference's own outputs (tests/golden, generated from ms_deform_attn_core_pytorch)
and the C oracle (oracle/msda_oracle.c, pinned in test_oracle_golden.py).

Tolerances follow the reference op tests: fp32 forward/backward allclose(rtol=1e-2,
atol=1e-3) (ops/test.py:31, :55); the gate requested by BASELINE is 1e-3 abs fp32.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = ['msda_kat_f32.npz', 'msda_kat_f64.npz', 'msda_mid_d32.npz', 'msda_mid_d36.npz']


def _load(golden_dir, name):
    d = dict(np.load(os.path.join(golden_dir, name)))
    t = {k: torch.from_numpy(v).cuda() for k, v in d.items()}
    return d, t


def _on_knot(d):
    from test_oracle_golden import _on_knot as k
    return k(d)


@pytest.fixture(scope='module')
def MSDA():
    import kinet_amd  # noqa: F401
    import MultiScaleDeformableAttention as M
    assert M.__file__.endswith('kinet_amd/MultiScaleDeformableAttention.py')
    return M


@pytest.mark.parametrize('name', CASES)
def test_forward_matches_reference(MSDA, golden_dir, name):
    d, t = _load(golden_dir, name)
    out = MSDA.ms_deform_attn_forward(t['value'], t['shapes'], t['loc'], t['attw'], 2)
    torch.cuda.synchronize()
    ref = d['out']
    atol = 1e-10 if ref.dtype == np.float64 else 1e-5
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=atol, rtol=1e-4)


@pytest.mark.parametrize('name', CASES)
def test_backward_matches_reference(MSDA, golden_dir, name):
    from oracle import msda_oracle
    d, t = _load(golden_dir, name)
    go = d.get('grad_out')
    if go is None:
        go = np.sign(d['out'])
    gv, gl, ga = MSDA.ms_deform_attn_backward(t['value'], t['shapes'], t['loc'], t['attw'],
                                              torch.from_numpy(go).cuda(), 2)
    torch.cuda.synchronize()
    f64 = d['value'].dtype == np.float64
    atol = 1e-10 if f64 else 1e-4
    np.testing.assert_allclose(gv.cpu().numpy(), d['grad_value'], atol=atol, rtol=1e-3)
    np.testing.assert_allclose(ga.cpu().numpy(), d['grad_attw'], atol=atol, rtol=1e-3)
    keep = ~_on_knot(d)
    np.testing.assert_allclose(gl.cpu().numpy()[keep], d['grad_loc'][keep], atol=atol * 10, rtol=1e-3)
    # on the derivative knots compare with the C restatement of the CUDA kernel instead
    ogv, ogl, oga = msda_oracle.bwd(d['value'], d['shapes'], d['loc'], d['attw'], go)
    np.testing.assert_allclose(gl.cpu().numpy(), ogl, atol=atol * 10, rtol=1e-3)


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_half_value_forward_backward(MSDA, golden_dir, dtype):
    d, t = _load(golden_dir, 'msda_mid_d32.npz')
    v = t['value'].to(dtype)
    out = MSDA.ms_deform_attn_forward(v, t['shapes'], t['loc'], t['attw'], 64)
    assert out.dtype == dtype
    ref = torch.from_numpy(d['out'])
    err = (out.float().cpu() - ref).abs().max().item()
    assert err < 0.05 * ref.abs().max().item(), err
    gv, gl, ga = MSDA.ms_deform_attn_backward(v, t['shapes'], t['loc'], t['attw'], t['grad_out'].to(dtype), 64)
    assert gv.dtype == dtype and gl.dtype == torch.float32
    gref = torch.from_numpy(d['grad_value'])
    assert (gv.float().cpu() - gref).abs().max().item() < 0.05 * gref.abs().max().item()


def test_large_encoder_shape_vs_oracle(MSDA):
    """config-2 level geometry at 1/4 resolution, checked against the C oracle."""
    from oracle import msda_oracle
    g = torch.Generator().manual_seed(0)
    shapes = torch.tensor([[25, 42], [13, 21], [7, 11], [4, 6]], dtype=torch.int64)
    S = int((shapes[:, 0] * shapes[:, 1]).sum())
    N, M, D, L, P, Lq = 2, 8, 32, 4, 4, 300
    value = torch.randn(N, S, M, D, generator=g)
    loc = torch.rand(N, Lq, M, L, P, 2, generator=g) * 1.2 - 0.1
    attw = torch.rand(N, Lq, M, L, P, generator=g)
    attw /= attw.sum((-1, -2), keepdim=True)
    out = MSDA.ms_deform_attn_forward(value.cuda(), shapes.cuda(), loc.cuda(), attw.cuda(), 64).cpu()
    ref = msda_oracle.fwd(value.numpy(), shapes.numpy(), loc.numpy(), attw.numpy())
    np.testing.assert_allclose(out.numpy(), ref, atol=1e-5, rtol=1e-4)


def test_errors_like_reference(MSDA, golden_dir):
    d, t = _load(golden_dir, 'msda_kat_f32.npz')
    with pytest.raises(RuntimeError, match='must divide im2col_step'):
        # N=2, step=3 -> min(2,3)=2 divides; use N=2 with step... reference: batch % min(batch, step)
        v = torch.cat([t['value'], t['value'][:1]], 0)
        MSDA.ms_deform_attn_forward(v, t['shapes'], torch.cat([t['loc'], t['loc'][:1]]),
                                    torch.cat([t['attw'], t['attw'][:1]]), 2)
    with pytest.raises(RuntimeError, match='contiguous'):
        nc = t['value'].transpose(0, 1).contiguous().transpose(0, 1)   # same shape, not contiguous
        MSDA.ms_deform_attn_forward(nc, t['shapes'], t['loc'], t['attw'], 2)
    with pytest.raises(RuntimeError):
        MSDA.ms_deform_attn_forward(t['value'].cpu(), t['shapes'], t['loc'], t['attw'], 2)


def test_function_gradcheck_f64(golden_dir):
    """ops/test_double_precision.py:111-119: gradcheck of the Function in fp64."""
    from torch.autograd import gradcheck
    from kinet_amd.msda import MSDeformAttnFunction
    d, t = _load(golden_dir, 'msda_kat_f64.npz')
    # keep locations away from the derivative knots, as gradcheck's finite differences need
    value = t['value'].clone().requires_grad_()
    loc = (t['loc'] * 0.9 + 0.05).clone().requires_grad_()
    attw = t['attw'].clone().requires_grad_()
    assert gradcheck(MSDeformAttnFunction.apply, (value, t['shapes'], loc, attw, 2), eps=1e-6, atol=1e-6)


def test_fused_module_path_matches_reference(golden_dir):
    """MSDeformAttn module (fused softmax/location/sampling kernel) vs the reference module."""
    from weights import randomize
    from kinet_amd.msda import MSDeformAttn
    d, t = _load(golden_dir, 'msda_module.npz')
    mod = randomize(MSDeformAttn(256, 4, 8, 4), seed=5).cuda().eval()
    with torch.no_grad():
        out2 = mod(t['query'], t['ref2'], t['input_flatten'], t['shapes'], t['padding_mask'])
        out4 = mod(t['query'], t['ref4'], t['input_flatten'], t['shapes'], None)
    np.testing.assert_allclose(out2.cpu().numpy(), d['out_ref2_masked'], atol=1e-3, rtol=0)
    np.testing.assert_allclose(out4.cpu().numpy(), d['out_ref4'], atol=1e-3, rtol=0)

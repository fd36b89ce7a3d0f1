"""Training-path operators (kinet_amd/autograd.py): forward and backward on kinet kernels vs
the same op in plain PyTorch fp32 autograd (the reference trains with torch's modules,
engine.py:145-149), on the GPU.  Tolerances: fp32 with different summation orders --
relative 1e-4 of the tensor's scale (GEMM reductions of up to ~10^4 terms)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _close(a, b, rel=1e-4, name=''):
    scale = b.abs().max().item() + 1e-12
    err = (a.float() - b.float()).abs().max().item()
    assert err <= rel * scale, f'{name}: max err {err:.3e} vs scale {scale:.3e}'


def _g(*shape, seed=0):
    g = torch.Generator(device='cuda').manual_seed(seed)
    return torch.randn(*shape, generator=g, device='cuda')


@pytest.mark.parametrize('M,Kin,Nout,bias', [(1000, 256, 288, True), (37, 288, 1024, True), (5000, 64, 20, False)])
def test_linear_fwd_bwd(M, Kin, Nout, bias):
    from kinet_amd import autograd as A
    x = _g(M, Kin, seed=1).requires_grad_()
    w = (_g(Nout, Kin, seed=2) * Kin ** -0.5).requires_grad_()
    b = _g(Nout, seed=3).requires_grad_() if bias else None
    go = _g(M, Nout, seed=4)
    y = A.linear(x, w, b)
    (y * go).sum().backward()
    got = [y.detach(), x.grad, w.grad] + ([b.grad] if bias else [])
    x2, w2 = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    b2 = b.detach().clone().requires_grad_() if bias else None
    y2 = F.linear(x2, w2, b2)
    (y2 * go).sum().backward()
    ref = [y2.detach(), x2.grad, w2.grad] + ([b2.grad] if bias else [])
    for n, a, r in zip(['y', 'dx', 'dw', 'db'], got, ref):
        _close(a, r, name=n)


@pytest.mark.parametrize('cin,cout,k,stride,pad,bn,relu,res,bias', [
    (64, 128, 3, 1, 1, True, True, False, False),     # bottleneck conv2 (stride 1)
    (128, 128, 3, 2, 1, True, True, False, False),    # first block conv2 of a stage (stride 2)
    (256, 512, 1, 2, 0, True, False, False, False),   # downsample 1x1/2
    (128, 512, 1, 1, 0, True, True, True, False),     # conv3 + residual + ReLU
    (512, 256, 1, 1, 0, False, False, False, True),   # input_proj 1x1 with bias
    (256, 256, 3, 2, 1, False, False, False, True),   # input_proj extra level 3x3/2 with bias
])
def test_conv_fwd_bwd(cin, cout, k, stride, pad, bn, relu, res, bias):
    from kinet_amd import autograd as A
    B, H, W = 2, 13, 18
    x = _g(B, H, W, cin, seed=5).requires_grad_()
    w = (_g(cout, cin, k, k, seed=6) * (cin * k * k) ** -0.5).requires_grad_()
    b = _g(cout, seed=7).requires_grad_() if bias else None
    scale = (torch.rand(cout, generator=torch.Generator(device='cuda').manual_seed(11), device='cuda') + 0.5) \
        if bn else None
    shift = _g(cout, seed=8) * 0.1 if bn else None
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    r = _g(B, Ho, Wo, cout, seed=9).requires_grad_() if res else None
    go = _g(B, Ho, Wo, cout, seed=10)
    y = A.conv_nhwc(x, w, b, stride, pad, scale, shift, relu, r)
    (y * go).sum().backward()
    # torch reference on NCHW
    x2 = x.detach().permute(0, 3, 1, 2).clone().requires_grad_()
    w2 = w.detach().clone().requires_grad_()
    b2 = b.detach().clone().requires_grad_() if bias else None
    r2 = r.detach().permute(0, 3, 1, 2).clone().requires_grad_() if res else None
    z = F.conv2d(x2, w2, b2, stride, pad)
    if bn:
        z = z * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)
    if res:
        z = z + r2
    if relu:
        # the reference applies the KERNEL's ReLU mask (y > 0, what its backward uses): an output
        # within fp32 rounding of 0 may land on opposite sides of the ReLU in the two forwards (the
        # round-4 one-off dx failure, profiles/r04ab_flake_note.log), and one flipped element moves
        # dx by a whole weight row; the forward values are still compared element by element
        zr = F.relu(z)
        _close(y.detach(), zr.detach().permute(0, 2, 3, 1), name='y')
        flips = ((y.detach() > 0).permute(0, 3, 1, 2) != (z.detach() > 0)) & (z.detach().abs() > 1e-4)
        assert not flips.any(), f'{int(flips.sum())} ReLU mask flips away from 0'
        z = z * (y.detach() > 0).permute(0, 3, 1, 2).to(z.dtype)
    (z * go.permute(0, 3, 1, 2)).sum().backward()
    _close(y.detach(), z.detach().permute(0, 2, 3, 1), name='y')
    _close(x.grad, x2.grad.permute(0, 2, 3, 1), name='dx')
    _close(w.grad, w2.grad, name='dw')
    # the parameter's own strides (DDP's bucket views copy a gradient whose strides differ)
    assert w.grad.stride() == w.stride(), (w.grad.stride(), w.stride())
    if bias:
        _close(b.grad, b2.grad, name='db')
    if res:
        _close(r.grad, r2.grad.permute(0, 2, 3, 1), name='dres')


@pytest.mark.parametrize('d', [256, 288])
def test_layer_norm_fwd_bwd(d):
    from kinet_amd import autograd as A
    ln = torch.nn.LayerNorm(d).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.normal_()
    x = (_g(3, 517, d, seed=11) * 2 + 0.5).requires_grad_()
    go = _g(3, 517, d, seed=12)
    y = A.layer_norm(x, ln)
    (y * go).sum().backward()
    got = [y.detach(), x.grad, ln.weight.grad.clone(), ln.bias.grad.clone()]
    ln.zero_grad()
    x2 = x.detach().clone().requires_grad_()
    y2 = ln(x2)
    (y2 * go).sum().backward()
    for n, a, r in zip(['y', 'dx', 'dg', 'db'], got, [y2.detach(), x2.grad, ln.weight.grad, ln.bias.grad]):
        _close(a, r, name=n)


@pytest.mark.parametrize('C,G,H,W', [(288, 32, 25, 42), (288, 32, 100, 167), (256, 32, 13, 21), (36, 12, 7, 9),
                                     (30, 6, 5, 7)])
def test_group_norm_fwd_bwd(C, G, H, W):
    """GroupNorm forward / backward (the input projections' norms) vs torch: 4-channel vector
    partial sums over 64-row blocks (C % 4 == 0, incl. the config-4 level-0 map 100 x 167 x 288)
    and the scalar path (C = 30)."""
    from kinet_amd import autograd as A
    gn = torch.nn.GroupNorm(G, C).cuda()
    with torch.no_grad():
        gn.weight.uniform_(0.5, 1.5)
        gn.bias.normal_()
    B = 2
    x = (_g(B, H * W, C, seed=13) * 3 + 1).requires_grad_()
    go = _g(B, H * W, C, seed=14)
    y = A.group_norm_nhwc(x, gn)
    (y * go).sum().backward()
    got = [y.detach(), x.grad, gn.weight.grad.clone(), gn.bias.grad.clone()]
    gn.zero_grad()
    x2 = x.detach().permute(0, 2, 1).reshape(B, C, H, W).clone().requires_grad_()
    y2 = gn(x2)
    (y2 * go.permute(0, 2, 1).reshape(B, C, H, W)).sum().backward()
    ref = [y2.detach().reshape(B, C, H * W).permute(0, 2, 1), x2.grad.reshape(B, C, H * W).permute(0, 2, 1),
           gn.weight.grad, gn.bias.grad]
    for n, a, r in zip(['y', 'dx', 'dg', 'db'], got, ref):
        _close(a, r, name=n)


@pytest.mark.parametrize('E,heads,Lq,mask', [(256, 8, 300, False), (288, 8, 520, True), (512, 8, 77, True),
                                            (288, 8, 65, False)])
def test_mha_core_fwd_bwd(E, heads, Lq, mask):
    from kinet_amd import autograd as A
    B = 2
    q = _g(B, Lq, E, seed=15).requires_grad_()
    k = _g(B, Lq, E, seed=16).requires_grad_()
    v = _g(B, Lq, E, seed=17).requires_grad_()
    km = None
    if mask:
        km = torch.zeros(B, Lq, dtype=torch.bool, device='cuda')
        km[1, -40:] = True
    go = _g(B, Lq, E, seed=18)
    D = E // heads
    o = A.mha_core(q, k, v, heads, D ** -0.5, km)
    (o * go).sum().backward()
    q2, k2, v2 = (t.detach().clone().requires_grad_() for t in (q, k, v))

    def split(t):
        return t.view(B, -1, heads, D).transpose(1, 2)
    am = None if km is None else km[:, None, None, :]
    o2 = F.scaled_dot_product_attention(split(q2), split(k2), split(v2),
                                        attn_mask=None if am is None else ~am).transpose(1, 2).reshape(B, Lq, E)
    (o2 * go).sum().backward()
    for n, a, r in zip(['o', 'dq', 'dk', 'dv'], [o.detach(), q.grad, k.grad, v.grad], [o2.detach(), q2.grad, k2.grad,
                                                                                     v2.grad]):
        _close(a, r, rel=2e-4, name=n)


@pytest.mark.parametrize('E,heads,Lq,Lk,mask,p', [(288, 8, 520, 520, True, 0.1), (256, 8, 77, 130, False, 0.5)])
def test_mha_dropout_fixed_mask(E, heads, Lq, Lk, mask, p):
    """Attention-probability dropout (nn.MultiheadAttention(dropout=p), deformable_transformer.py:345):
    forward and gradients equal torch fp32 autograd of softmax -> (P * Z) @ V with the SAME keep
    mask Z, materialised by kinet_dropout_mask from the seed the kernels used."""
    from kinet_amd import autograd as A
    from kinet_amd import kernels as K
    B = 2
    q = _g(B, Lq, E, seed=31).requires_grad_()
    k = _g(B, Lk, E, seed=32).requires_grad_()
    v = _g(B, Lk, E, seed=33).requires_grad_()
    km = None
    if mask:
        km = torch.zeros(B, Lk, dtype=torch.bool, device='cuda')
        km[1, -40:] = True
    go = _g(B, Lq, E, seed=34)
    D = E // heads
    seed = torch.tensor([123456789], dtype=torch.int64, device='cuda')
    o = A.mha_core(q, k, v, heads, D ** -0.5, km, dropout_p=p, seed=seed)
    (o * go).sum().backward()
    keep = K.dropout_mask(seed, B * heads * Lq * Lk, p).view(B, heads, Lq, Lk).float()
    q2, k2, v2 = (t.detach().clone().requires_grad_() for t in (q, k, v))

    def split(t):
        return t.view(B, -1, heads, D).transpose(1, 2)
    s = split(q2) @ split(k2).transpose(-1, -2) * D ** -0.5
    if km is not None:
        s = s.masked_fill(km[:, None, None, :], float('-inf'))
    prob = s.softmax(-1) * keep / (1 - p)
    o2 = (prob @ split(v2)).transpose(1, 2).reshape(B, Lq, E)
    (o2 * go).sum().backward()
    for n, a, r in zip(['o', 'dq', 'dk', 'dv'], [o.detach(), q.grad, k.grad, v.grad], [o2.detach(), q2.grad, k2.grad,
                                                                                     v2.grad]):
        _close(a, r, rel=2e-4, name=n)


def test_dropout_mask_statistics():
    """The keep mask is Bernoulli(1 - p): keep rate within 5 sigma, no correlation between
    neighbouring elements or between two seeds, and reproducible from its seed."""
    from kinet_amd import kernels as K
    n = 1 << 22
    for p in (0.1, 0.5):
        s1 = torch.tensor([7], dtype=torch.int64, device='cuda')
        s2 = torch.tensor([8], dtype=torch.int64, device='cuda')
        a = K.dropout_mask(s1, n, p).double()
        b = K.dropout_mask(s2, n, p).double()
        q = 1 - p
        sig = (q * p / n) ** 0.5
        assert abs(a.mean().item() - q) < 5 * sig
        # P(both kept) = q^2 for independent draws (neighbours, other seed)
        assert abs((a[1:] * a[:-1]).mean().item() - q * q) < 5 * (q * q * (1 - q * q) / n) ** 0.5
        assert abs((a * b).mean().item() - q * q) < 5 * (q * q * (1 - q * q) / n) ** 0.5
        assert torch.equal(a, K.dropout_mask(s1, n, p).double())


def test_multihead_attention_train_dropout_reproducible():
    """Training-mode multihead_attention drops probabilities (the output differs from eval
    mode) with a seed from torch's CUDA generator: torch.manual_seed reproduces it."""
    from kinet_amd import autograd as A
    E, H, B, L = 288, 8, 2, 64
    mod = torch.nn.MultiheadAttention(E, H, dropout=0.1).cuda().train()
    x = _g(B, L, E, seed=35)
    torch.manual_seed(3)
    y1 = A.multihead_attention(mod, x, x, x)
    torch.manual_seed(3)
    y2 = A.multihead_attention(mod, x, x, x)
    y3 = A.multihead_attention(mod, x, x, x)
    mod.eval()
    y0 = A.multihead_attention(mod, x, x, x)
    assert torch.equal(y1, y2)
    assert not torch.equal(y1, y3) and not torch.equal(y1, y0)


def test_multihead_attention_matches_module():
    """in_proj split + core + out_proj == nn.MultiheadAttention (batch-first by transposes)."""
    from kinet_amd import autograd as A
    E, H, B, L = 288, 8, 2, 120
    mod = torch.nn.MultiheadAttention(E, H, dropout=0.0).cuda()
    x = _g(B, L, E, seed=19).requires_grad_()
    pos = _g(B, L, E, seed=20)
    go = _g(B, L, E, seed=21)
    y = A.multihead_attention(mod, x + pos, x + pos, x)
    (y * go).sum().backward()
    got = [y.detach(), x.grad, mod.in_proj_weight.grad.clone(), mod.out_proj.weight.grad.clone()]
    mod.zero_grad()
    x2 = x.detach().clone().requires_grad_()
    qk = (x2 + pos).transpose(0, 1)
    y2 = mod(qk, qk, x2.transpose(0, 1))[0].transpose(0, 1)
    (y2 * go).sum().backward()
    for n, a, r in zip(['y', 'dx', 'dWin', 'dWout'], got, [y2.detach(), x2.grad, mod.in_proj_weight.grad,
                                                           mod.out_proj.weight.grad]):
        _close(a, r, rel=2e-4, name=n)


@pytest.mark.parametrize('rows,cols', [(44446, 288), (1000, 1024), (777, 90), (5, 12), (70000, 256)])
def test_colsum_vs_f64_and_deterministic(rows, cols):
    from kinet_amd import kernels as K
    g = torch.Generator().manual_seed(rows + cols)
    a = torch.randn(rows, cols, generator=g, dtype=torch.float64)
    out = K.colsum(a.float().cuda())
    out2 = K.colsum(a.float().cuda())
    torch.cuda.synchronize()
    ref = a.sum(0)
    assert torch.equal(out, out2)
    assert ((out.double().cpu() - ref).abs() <= 1e-6 * a.abs().sum(0) + 1e-6).all()


# ------------------------------------------------- training glue (csrc/train_ops.hip)
def _leaf(t):
    return t.detach().clone().requires_grad_()


@pytest.mark.parametrize('rows,d,p', [(3001, 288, 0.1), (517, 256, 0.5), (64, 256, 0.0), (7, 90, 0.3), (22223, 288, 0.1)])
def test_dropout_add_layernorm_fixed_mask(rows, d, p):
    """LayerNorm(x + dropout(r)) (deformable_transformer.py:100,108,186,196,199) and its
    gradients equal torch fp32 autograd of F.layer_norm(x + r * Z) with the SAME keep mask Z
    (kinet_dropout_mask of the seed the kernels used)."""
    from kinet_amd import autograd as A
    from kinet_amd import kernels as K
    ln = torch.nn.LayerNorm(d).cuda()
    with torch.no_grad():
        ln.weight.copy_(1 + 0.1 * _g(d, seed=40))
        ln.bias.copy_(0.1 * _g(d, seed=41))
    drop = torch.nn.Dropout(p).train()
    x, r = _g(2, rows, d, seed=42).requires_grad_(), _g(2, rows, d, seed=43).requires_grad_()
    go = _g(2, rows, d, seed=44)
    torch.manual_seed(5)
    y = A.dropout_add_layer_norm(x, r, ln, drop)
    (y * go).sum().backward()
    got = [y.detach(), x.grad, r.grad, ln.weight.grad.clone(), ln.bias.grad.clone()]
    torch.manual_seed(5)
    seed = A._seed(x.device, p)     # the same draw from the CUDA generator
    keep = (K.dropout_mask(seed, x.numel(), p).view(x.shape).float() if p > 0 else torch.ones_like(x))
    ln.zero_grad()
    x2, r2 = _leaf(x), _leaf(r)
    y2 = F.layer_norm(x2 + r2 * keep / (1 - p), (d,), ln.weight, ln.bias, ln.eps)
    (y2 * go).sum().backward()
    for n, a, b in zip(['y', 'dx', 'dr', 'dg', 'db'], got, [y2.detach(), x2.grad, r2.grad, ln.weight.grad,
                                                           ln.bias.grad]):
        _close(a, b, rel=2e-5 if n in ('y', 'dx', 'dr') else 1e-4, name=n)
    if p > 0:
        rate = keep.mean().item()
        assert abs(rate - (1 - p)) < 5 * (p * (1 - p) / keep.numel()) ** 0.5
        drop.eval()
        y0 = A.dropout_add_layer_norm(x.detach(), r.detach(), ln, drop)
        _close(y0, F.layer_norm(x + r, (d,), ln.weight, ln.bias, ln.eps).detach(), rel=2e-5, name='eval')


@pytest.mark.parametrize('n,p,relu', [(4096 * 1024 + 3, 0.1, True), (1000, 0.0, True), (999, 0.5, False)])
def test_dropout_act_fixed_mask(n, p, relu):
    from kinet_amd import autograd as A
    from kinet_amd import kernels as K
    drop = torch.nn.Dropout(p).train()
    x = _g(n, seed=45).requires_grad_()
    go = _g(n, seed=46)
    torch.manual_seed(6)
    y = A.dropout_act(x, drop, relu=relu)
    (y * go).sum().backward()
    torch.manual_seed(6)
    seed = A._seed(x.device, p)
    keep = K.dropout_mask(seed, n, p).float() if p > 0 else torch.ones_like(x)
    x2 = _leaf(x)
    y2 = (F.relu(x2) if relu else x2) * keep / (1 - p)
    (y2 * go).sum().backward()
    assert torch.equal(y.detach(), y2.detach())
    assert torch.equal(x.grad, x2.grad)


@pytest.mark.gpu
@pytest.mark.parametrize('relu', [False, True])
def test_dropout_act_nan_like_torch(relu):
    """NaN inputs stay NaN in the output (relu(NaN) = NaN; a dropped NaN is NaN * 0 = NaN) and
    the gradients follow torch's (relu threshold_backward on the output, the mask product)."""
    from kinet_amd import autograd as A
    from kinet_amd import kernels as K
    n, p = 4099, 0.25
    drop = torch.nn.Dropout(p).train()
    x0 = _g(n, seed=47)
    x0[::97] = float('nan')
    x = x0.clone().requires_grad_()
    go = _g(n, seed=48)
    if not relu:
        # (with relu the backward sees only y = relu(x) * mask: for a DROPPED unit it cannot tell
        # x > 0 from x <= 0, so a NaN incoming gradient there gives 0 where torch's
        # threshold_backward(x) gives NaN -- the one documented difference; finite gradients match)
        go[5::211] = float('nan')
    torch.manual_seed(7)
    y = A.dropout_act(x, drop, relu=relu)
    (y * go).sum().backward()
    torch.manual_seed(7)
    keep = K.dropout_mask(A._seed(x.device, p), n, p).float()
    x2 = _leaf(x)
    y2 = (F.relu(x2) if relu else x2) * keep / (1 - p)
    (y2 * go).sum().backward()
    assert y.isnan().sum() >= x0.isnan().sum()
    torch.testing.assert_close(y.detach(), y2.detach(), rtol=0, atol=0, equal_nan=True)
    torch.testing.assert_close(x.grad, x2.grad, rtol=0, atol=0, equal_nan=True)


@pytest.mark.gpu
def test_inverse_sigmoid_nan_like_torch():
    """A NaN input gives a NaN output and a zero gradient, as the torch clamp chain does."""
    from kinet_amd import autograd as A
    x = torch.tensor([0.3, float('nan'), 0.7, float('nan')], device='cuda').requires_grad_()
    y = A.inverse_sigmoid(x)
    y.sum().backward()
    x2 = _leaf(x)
    xc = x2.clamp(min=0, max=1)
    y2 = torch.log(xc.clamp(min=1e-5) / (1 - xc).clamp(min=1e-5))
    y2.sum().backward()
    torch.testing.assert_close(y.detach(), y2.detach(), equal_nan=True)
    torch.testing.assert_close(x.grad, x2.grad, equal_nan=True)


def _msda_prep_torch(off, logit, ref, shapes, qmask, M, L, P):
    # ms_deform_attn.py:70-82 op for op
    Nb, Lq = off.shape[:2]
    so = off.view(Nb, Lq, M, L, P, 2)
    aw = F.softmax(logit.view(Nb, Lq, M, L * P), -1).view(Nb, Lq, M, L, P)
    if qmask is not None:
        aw = aw.masked_fill(qmask[..., None, None, None], 0.0)
    if ref.shape[-1] == 2:
        loc = ref[:, :, None, :, None, :] + so / shapes[None, None, None, :, None, :]
    else:
        loc = ref[:, :, None, :, None, :2] + so / P * ref[:, :, None, :, None, 2:] * 0.5
    return loc, aw


@pytest.mark.parametrize('refd,mask,M,L,P', [(2, True, 8, 4, 4), (4, False, 8, 4, 4), (4, True, 8, 8, 4),
                                             (2, False, 4, 3, 2)])
def test_msda_prep_vs_torch(refd, mask, M, L, P):
    """Sampling locations + softmaxed attention weights (ms_deform_attn.py:70-82) from the packed
    [offsets | logits] projection, and their gradients w.r.t. it and the reference points, vs
    torch fp32 autograd of the reference's op sequence."""
    from kinet_amd import autograd as A
    Nb, Lq = 2, 777
    C2, C1 = M * L * P * 2, M * L * P
    shapes = torch.tensor([[100 // (2 ** i), 150 // (2 ** i)] for i in range(L)], dtype=torch.int64, device='cuda')
    offlog = torch.cat([_g(Nb, Lq, C2, seed=47) * 3, _g(Nb, Lq, C1, seed=48)], -1).requires_grad_()
    ref = torch.rand(Nb, Lq, L, refd, device='cuda').requires_grad_()
    qm = (torch.rand(Nb, Lq, device='cuda') < 0.2) if mask else None
    gl = _g(Nb, Lq, M, L, P, 2, seed=49)
    ga = _g(Nb, Lq, M, L, P, seed=50)
    loc, aw = A.msda_prep(offlog, ref, shapes, qm, M, L, P)
    ((loc * gl).sum() + (aw * ga).sum()).backward()
    got = [loc.detach(), aw.detach(), offlog.grad, ref.grad]
    ol2, ref2 = _leaf(offlog), _leaf(ref)
    loc2, aw2 = _msda_prep_torch(ol2[..., :C2], ol2[..., C2:], ref2, shapes, qm, M, L, P)
    ((loc2 * gl).sum() + (aw2 * ga).sum()).backward()
    for n, a, b in zip(['loc', 'attw', 'doffl', 'dref'], got, [loc2.detach(), aw2.detach(), ol2.grad, ref2.grad]):
        _close(a, b, rel=1e-5, name=n)


def test_inverse_sigmoid_vs_torch():
    """util/misc.py:609-613 forward and gradient (through the clamps' masks) incl. values at
    and outside [0, 1] and inside the eps band."""
    from kinet_amd import autograd as A
    x = torch.cat([torch.rand(10000, device='cuda'), torch.tensor([0.0, 1.0, -0.5, 1.5, 1e-6, 1 - 1e-6, 0.5, 1e-5],
                                                                    device='cuda')]).requires_grad_()
    go = _g(x.numel(), seed=51)
    y = A.inverse_sigmoid(x)
    (y * go).sum().backward()
    x2 = _leaf(x)
    xc = x2.clamp(min=0, max=1)
    y2 = torch.log(xc.clamp(min=1e-5) / (1 - xc).clamp(min=1e-5))
    (y2 * go).sum().backward()
    _close(y.detach(), y2.detach(), rel=1e-6, name='y')
    _close(x.grad, x2.grad, rel=1e-6, name='dx')


def test_multihead_attention_packed_qk_matches_module():
    """q = k (the decoder self-attention, deformable_transformer.py:370): the packed q|k
    projection path (one GEMM each way) == nn.MultiheadAttention, incl. the in_proj gradient."""
    from kinet_amd import autograd as A
    E, H, B, L = 288, 8, 2, 300
    mod = torch.nn.MultiheadAttention(E, H, dropout=0.0).cuda()
    x = _g(B, L, E, seed=52).requires_grad_()
    pos = _g(B, L, E, seed=53)
    go = _g(B, L, E, seed=54)
    km = torch.zeros(B, L, dtype=torch.bool, device='cuda')
    km[0, -17:] = True
    qk = x + pos
    y = A.multihead_attention(mod, qk, qk, x, key_padding_mask=km)
    (y * go).sum().backward()
    got = [y.detach(), x.grad, mod.in_proj_weight.grad.clone(), mod.in_proj_bias.grad.clone()]
    mod.zero_grad()
    x2 = _leaf(x)
    qk2 = (x2 + pos).transpose(0, 1)
    y2 = mod(qk2, qk2, x2.transpose(0, 1), key_padding_mask=km)[0].transpose(0, 1)
    (y2 * go).sum().backward()
    for n, a, r in zip(['y', 'dx', 'dWin', 'dbin'], got, [y2.detach(), x2.grad, mod.in_proj_weight.grad,
                                                         mod.in_proj_bias.grad]):
        _close(a, r, rel=2e-4, name=n)

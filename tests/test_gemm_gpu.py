"""GPU numerics of the MFMA GEMM / implicit-GEMM conv / norm kernels vs plain PyTorch fp32
on the CPU (the op the reference delegates to cuBLAS/cuDNN)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).abs().max() / (b.float().abs().max() + 1e-6)).item()


@pytest.fixture(scope='module')
def K():
    from kinet_amd import kernels
    return kernels


@pytest.mark.parametrize('M,N,Kd', [(1, 4, 8), (37, 91, 256), (300, 256, 256), (300, 768, 256),
                                    (1000, 1024, 256), (513, 256, 1024), (4200, 384, 256), (64, 64, 64)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_linear_epilogue(K, M, N, Kd, dtype):
    g = torch.Generator().manual_seed(M * 7 + N)
    x = torch.randn(M, Kd, generator=g)
    w = torch.randn(N, Kd, generator=g) / Kd ** 0.5
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g)
    mask = torch.rand(M, generator=g) < 0.2
    ref = F.relu(F.linear(x, w, b) + r).masked_fill(mask[:, None], 0)
    y = K.linear(x.cuda().to(dtype), w.cuda(), b.cuda(), relu=True, residual=r.cuda().to(dtype),
                 row_mask=mask.cuda())
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert _rel(y, ref) < tol


def test_linear_f32_out_from_bf16(K):
    x = torch.randn(300, 256)
    w = torch.randn(384, 256) / 16
    b = torch.randn(384)
    y = K.linear(x.cuda().bfloat16(), w.cuda(), b.cuda(), out_dtype=torch.float32)
    assert y.dtype == torch.float32
    assert _rel(y, F.linear(x, w, b)) < 2e-2


@pytest.mark.parametrize('B,H,W,Cin,Cout,k,s,p', [
    (2, 17, 23, 64, 64, 3, 1, 1), (1, 32, 40, 256, 128, 1, 1, 0), (2, 33, 41, 64, 256, 1, 2, 0),
    (1, 21, 30, 128, 128, 3, 2, 1), (2, 64, 80, 8, 64, 7, 2, 3), (1, 9, 11, 2048, 256, 3, 2, 1)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_conv2d_nhwc_bn_residual_relu(K, B, H, W, Cin, Cout, k, s, p, dtype):
    g = torch.Generator().manual_seed(H * W + Cin)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) * (2.0 / (Cin * k * k)) ** 0.5
    scale = torch.rand(Cout, generator=g) + 0.5
    bias = torch.randn(Cout, generator=g) * 0.1
    y_ref = F.conv2d(x, w, stride=s, padding=p) * scale[None, :, None, None] + bias[None, :, None, None]
    res = torch.randn_like(y_ref)
    y_ref = F.relu(y_ref + res)
    xn = x.permute(0, 2, 3, 1).contiguous().cuda().to(dtype)
    wp = K.pack_conv_weight(w.cuda(), dtype)
    rn = res.permute(0, 2, 3, 1).contiguous().cuda().to(dtype)
    y = K.conv2d_nhwc(xn, wp, s, p, scale=scale.cuda(), bias=bias.cuda(), relu=True, residual=rn)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert _rel(y.permute(0, 3, 1, 2), y_ref) < tol


def test_stem_packed_image(K):
    g = torch.Generator().manual_seed(3)
    img = torch.randn(2, 3, 50, 66, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    ref = F.conv2d(img, w, stride=2, padding=3)
    xp = K.pack_image(img.cuda(), torch.float32, 8)
    y = K.conv2d_nhwc(xp, K.pack_conv_weight(w.cuda(), torch.float32, cin_pad=8), 2, 3)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 2e-5
    mp = K.maxpool_3x3s2(y)
    assert _rel(mp.permute(0, 3, 1, 2), F.max_pool2d(ref, 3, 2, 1)) < 1e-6


@pytest.mark.parametrize('d', [256, 288])
def test_layernorm(K, d):
    x = torch.randn(777, d)
    r = torch.randn(777, d)
    g = torch.rand(d) + 0.5
    b = torch.randn(d)
    y = K.layernorm(x.cuda(), g.cuda(), b.cuda(), residual=r.cuda())
    assert _rel(y, F.layer_norm(x + r, (d,), g, b)) < 1e-5


def test_groupnorm_into_flat_buffer(K):
    B, H, W, C = 2, 13, 21, 256
    x = torch.randn(B, C, H, W) * 2 + 0.3
    g = torch.rand(C) + 0.5
    b = torch.randn(C)
    ref = F.group_norm(x, 32, g, b)
    flat = torch.zeros(B, 1000, C).cuda()
    xn = x.permute(0, 2, 3, 1).reshape(B, H * W, C).contiguous().cuda()
    K.groupnorm_nhwc(xn, g.cuda(), b.cuda(), 32, out=flat[:, 100:], out_batch_stride=1000 * C)
    got = flat[:, 100:100 + H * W].reshape(B, H, W, C).permute(0, 3, 1, 2).cpu()
    assert _rel(got, ref) < 1e-4
    assert flat[:, :100].abs().max().item() == 0


@pytest.mark.parametrize('D,Lq', [(32, 300), (36, 507)])
def test_mha_core(K, D, Lq):
    heads, B = 8, 2
    E = heads * D
    q = torch.randn(B, Lq, E)
    k = torch.randn(B, Lq, E)
    v = torch.randn(B, Lq, E)
    def split(t):
        return t.view(B, Lq, heads, D).transpose(1, 2)
    ref = F.scaled_dot_product_attention(split(q), split(k), split(v)).transpose(1, 2).reshape(B, Lq, E)
    y = K.mha_core(q.cuda(), k.cuda(), v.cuda(), heads, D ** -0.5)
    assert _rel(y, ref) < 1e-5

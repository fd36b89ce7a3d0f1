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


@pytest.mark.parametrize('N,C,H,W', [(3, 64, 101, 167), (1, 64, 5, 7), (2, 32, 400, 667)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_maxpool_exact(K, N, C, H, W, dtype):
    """3x3/2 max-pool (XCD-banded row kernel, incl. fewer rows than XCDs): bit-exact."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, C, H, W, generator=g).to(dtype)
    ref = F.max_pool2d(x.float(), 3, 2, 1).to(dtype)
    got = K.maxpool_3x3s2(x.permute(0, 2, 3, 1).contiguous().cuda()).permute(0, 3, 1, 2).cpu()
    assert torch.equal(got, ref)


@pytest.mark.parametrize('H,W', [(50, 66), (37, 41), (800, 1333)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16, torch.float32])
def test_stem_kwfold(K, H, W, dtype):
    """Tap-folded stem: the packed layout is exactly the strided horizontal unfold of the
    image, and the 7x1 (2, 1)-strided conv over it equals torchvision's 7x7/2 conv1."""
    g = torch.Generator().manual_seed(H + W)
    B = 2 if H < 800 else 1
    img = torch.randn(B, 3, H, W, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    scale = torch.rand(64, generator=g) + 0.5
    bias = torch.randn(64, generator=g) * 0.1
    xp = K.pack_image_kwfold(img.cuda(), dtype, 7, 2, 3, 24)
    Wo = (W + 6 - 7) // 2 + 1
    assert xp.shape == (B, H, Wo, 24)
    # expected fold: column ow holds x[c][h][2*ow - 3 + kw] at channel kw*3 + c
    pad = F.pad(img, (3, 3))
    cols = torch.stack([pad[..., kw: kw + 2 * (Wo - 1) + 1: 2] for kw in range(7)], -1)   # (B, 3, H, Wo, 7)
    exp = torch.zeros(B, H, Wo, 24)
    exp[..., :21] = cols.permute(0, 2, 3, 4, 1).reshape(B, H, Wo, 21)
    assert torch.equal(xp.cpu(), exp.to(dtype))
    y = K.conv2d_nhwc(xp, K.pack_stem_weight(w.cuda(), dtype, 24), (2, 1), (3, 0), scale=scale.cuda(),
                      bias=bias.cuda(), relu=True)
    ref = F.relu(F.conv2d(img, w, stride=2, padding=3) * scale[None, :, None, None] + bias[None, :, None, None])
    torch.cuda.synchronize()
    assert y.shape == (B, (H - 1) // 2 + 1, Wo, 64)
    assert _rel(y.permute(0, 3, 1, 2), ref) < (2e-5 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize('k,s,p', [((3, 1), (2, 1), (1, 0)), ((5, 1), (1, 1), (2, 0)), ((1, 3), (1, 2), (0, 1))])
def test_conv2d_asymmetric_stride_pad(K, k, s, p):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 16, 23, 29, generator=g)
    w = torch.randn(48, 16, k[0], k[1], generator=g) * 0.2
    ref = F.conv2d(x, w, stride=s, padding=p)
    y = K.conv2d_nhwc(x.permute(0, 2, 3, 1).contiguous().cuda().bfloat16(), K.pack_conv_weight(w.cuda(), torch.bfloat16),
                      s, p)
    torch.cuda.synchronize()
    assert _rel(y.permute(0, 3, 1, 2), ref) < 2e-2


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


@pytest.mark.parametrize('C,groups,dt', [(256, 32, torch.bfloat16), (256, 32, torch.float32), (36, 6, torch.float32),
                                         (288, 32, torch.bfloat16), (288, 32, torch.float16), (288, 32, torch.float32),
                                         (36, 12, torch.float32)])
def test_groupnorm_deterministic(K, C, groups, dt):
    """Fixed-order reductions (no float atomics): reruns are bit-identical, on the 16-byte vector
    path (C/groups a multiple of the vector), the vector path whose vectors straddle two groups
    (d = 288 in 32 groups of 9 -- configs 3-5; 36 / 6 in f32) and the scalar path (groups of 3,
    fewer channels than a vector)."""
    B, H, W = 3, 100, 167
    x = (torch.randn(B, C, H, W) * 2 + 0.3)
    g = torch.rand(C) + 0.5
    b = torch.randn(C)
    ref = F.group_norm(x.to(dt).float(), groups, g, b)
    xn = x.permute(0, 2, 3, 1).reshape(B, H * W, C).contiguous().to(dt).cuda()
    y0 = K.groupnorm_nhwc(xn, g.cuda(), b.cuda(), groups)
    got = y0.float().reshape(B, H, W, C).permute(0, 3, 1, 2).cpu()
    assert _rel(got, ref) < {torch.bfloat16: 1e-2, torch.float16: 1e-3, torch.float32: 1e-5}[dt]
    for _ in range(5):
        y = K.groupnorm_nhwc(xn, g.cuda(), b.cuda(), groups)
        assert torch.equal(y, y0)


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


@pytest.mark.parametrize('D,Lq,Lk', [(32, 300, 300), (32, 57, 333), (32, 130, 37), (36, 520, 520), (36, 57, 333),
                                    (36, 130, 37), (36, 500, 640)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_mha_core_mfma(K, D, Lq, Lk, dtype):
    """head_dim 32 / 36, 16-bit: the MFMA kernels (attn.hip; 36 = the d = 288 decoder's
    500 + 20 queries, head dim padded to two K-steps) vs fp32 SDPA with a key padding mask, and
    vs the FMA kernel on the same 16-bit inputs."""
    from kinet_amd import _native
    heads, B = 8, 3
    E = heads * D
    g = torch.Generator().manual_seed(Lq + Lk)
    q, k, v = (torch.randn(B, n, E, generator=g).to(dtype) for n in (Lq, Lk, Lk))
    mask = torch.rand(B, Lk, generator=g) < 0.2
    mask[:, 0] = False

    def split(t, n):
        return t.float().view(B, n, heads, D).transpose(1, 2)
    ref = F.scaled_dot_product_attention(split(q, Lq), split(k, Lk), split(v, Lk),
                                         attn_mask=~mask[:, None, None, :]).transpose(1, 2).reshape(B, Lq, E)
    y = K.mha_core(q.cuda(), k.cuda(), v.cuda(), heads, D ** -0.5, key_mask=mask.cuda())
    lib = _native.lib()
    old = lib.kinet_mha_set_mfma(0)
    try:
        y_fma = K.mha_core(q.cuda(), k.cuda(), v.cuda(), heads, D ** -0.5, key_mask=mask.cuda())
    finally:
        lib.kinet_mha_set_mfma(old)
    torch.cuda.synchronize()
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    assert _rel(y, ref) < tol
    assert _rel(y, y_fma) < tol


# ---- the 512-thread LDS-DMA kernel (M >= 16384, N >= 128, 16-bit operands) ----------------

@pytest.fixture
def gemm_flags():
    """Select the GEMM kernel family for one test and restore the default afterwards."""
    from kinet_amd import _native
    lib = _native.lib()
    yield lib.kinet_gemm_set_flags
    lib.kinet_gemm_set_flags(0)


@pytest.fixture
def big(gemm_flags):
    gemm_flags(2)
    yield


@pytest.mark.parametrize('M,N,Kd,mode', [
    (20000, 256, 256, 'ln'),          # output_proj + residual + LayerNorm (256x256 tiles)
    (16411, 1024, 256, 'relu'),       # FFN linear1, ragged M
    (17000, 384, 264, 'plain'),       # K tail inside a 64-wide K-step
    (16390, 128, 1024, 'relu'),       # BN = 128 tiles
    (18000, 200, 256, 'ln'),          # ragged N inside one 256-wide tile, LN over 200 columns
    (16500, 160, 512, 'residual'),    # ragged N on the 256-wide tile without LN
])
def test_big_gemm_vs_fp32(K, big, M, N, Kd, mode):
    g = torch.Generator().manual_seed(M + N + Kd)
    x = torch.randn(M, Kd, generator=g).bfloat16()
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).bfloat16()
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    mask = torch.rand(M, generator=g) < 0.1
    ref = F.linear(x.float(), w.float(), b)
    kw = {}
    if mode in ('ln', 'residual'):
        ref = ref + r.float()
        kw['residual'] = r.cuda()
    if mode == 'relu':
        ref = F.relu(ref)
        kw['relu'] = True
    if mode == 'ln':
        gam, bet = torch.rand(N, generator=g) + 0.5, torch.randn(N, generator=g)
        ref = F.layer_norm(ref, (N,), gam, bet, 1e-5)
        kw['ln'] = (gam.cuda(), bet.cuda(), 1e-5)
    ref = ref.masked_fill(mask[:, None], 0)
    y = K.linear(x.cuda(), w.cuda(), b.cuda(), row_mask=mask.cuda(), **kw)
    torch.cuda.synchronize()
    # bf16 output rounding only (fp32 accumulation of bf16 products)
    err = (y.float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('M,N', [(20011, 288), (9000, 320), (8192, 300)])
def test_wide_layernorm_gemm_vs_fp32(K, M, N, dtype):
    """output_proj + residual + LayerNorm over rows wider than 256 (d = 288 of configs 3-5) at
    encoder sizes (the 128 x 320 LDS-DMA tile with the fused LayerNorm epilogue), against torch
    fp32 on the same 16-bit operands: f32 accumulation and normalisation, one output rounding
    (bound stated with slack for the accumulation order)."""
    g = torch.Generator().manual_seed(M + N)
    Kd = N
    x = torch.randn(M, Kd, generator=g).to(dtype)
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to(dtype)
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).to(dtype)
    gam, bet = torch.rand(N, generator=g) + 0.5, torch.randn(N, generator=g)
    pre = F.linear(x.float(), w.float(), b) + r.float()
    ref = F.layer_norm(pre, (N,), gam, bet, 1e-5)
    y = K.linear(x.cuda(), w.cuda(), b.cuda(), residual=r.cuda(), ln=(gam.cuda(), bet.cuda(), 1e-5))
    torch.cuda.synchronize()
    u = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    rstd = 1.0 / pre.std(-1, unbiased=False, keepdim=True)
    err = (y.float().cpu() - ref).abs()
    bound = (pre.abs() * rstd * gam.abs() * 2 * u) + ref.abs() * 2 * u + 1e-3
    assert (err <= bound).all(), (err / bound).max().item()


@pytest.mark.parametrize('M,N,Kd', [(20000, 256, 256), (16411, 1024, 264), (16390, 128, 1024)])
def test_big_gemm_matches_small_kernel(K, gemm_flags, M, N, Kd):
    """Both kernels accumulate the same bf16 products in the same K-step order in f32, so
    they must agree to the last bit of the bf16 output (or within one rounding step)."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, Kd, generator=g).bfloat16().cuda()
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).bfloat16().cuda()
    b = torch.randn(N, generator=g).cuda()
    gemm_flags(2)
    y_big = K.linear(x, w, b, relu=True)
    gemm_flags(0)
    y_small = K.linear(x, w, b, relu=True)
    torch.cuda.synchronize()
    d = (y_big.float() - y_small.float()).abs()
    tol = y_small.float().abs() * 2.0 ** -7 + 1e-6
    assert (d <= tol).all(), d.max().item()
    assert (d == 0).float().mean().item() > 0.95


def test_big_gemm_headmajor(K, big):
    B, S, d, hd = 2, 9000, 256, 32
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, S, d, generator=g).bfloat16()
    w = (torch.randn(d, d, generator=g) / 16).bfloat16()
    b = torch.randn(d, generator=g)
    mask = torch.rand(B, S, generator=g) < 0.2
    ref = F.linear(x.float(), w.float(), b).masked_fill(mask[..., None], 0)      # (B, S, d)
    ref = ref.view(B, S, d // hd, hd).permute(2, 0, 1, 3)                         # (heads, B, S, hd)
    y = K.value_proj_headmajor(x.cuda(), w.cuda(), b.cuda(), hd, row_mask=mask.cuda())
    torch.cuda.synchronize()
    assert tuple(y.shape) == tuple(ref.shape)
    err = (y.float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()


@pytest.mark.parametrize('B,H,W,Cin,Cout,k,s,p', [
    (2, 96, 96, 64, 256, 1, 1, 0),      # 1x1, BN = 256 tiles
    (2, 100, 100, 64, 128, 3, 1, 1),    # 3x3 padded, BN = 128 tiles
    (2, 190, 190, 64, 128, 3, 2, 1),    # strided
    (1, 260, 260, 8, 128, 7, 2, 3),     # stem-like: K = 392 (tail), Cin = 8
    (4, 100, 168, 256, 512, 1, 2, 0),   # strided 1x1 downsample
])
def test_big_conv_vs_fp32(K, big, B, H, W, Cin, Cout, k, s, p):
    g = torch.Generator().manual_seed(H * W + Cin + Cout)
    x = torch.randn(B, Cin, H, W, generator=g).bfloat16()
    w = (torch.randn(Cout, Cin, k, k, generator=g) * (2.0 / (Cin * k * k)) ** 0.5).bfloat16()
    scale = torch.rand(Cout, generator=g) + 0.5
    bias = torch.randn(Cout, generator=g) * 0.1
    y_ref = F.conv2d(x.float(), w.float(), stride=s, padding=p) * scale[None, :, None, None] + bias[None, :, None, None]
    res = torch.randn_like(y_ref).bfloat16()
    y_ref = F.relu(y_ref + res.float())
    xn = x.permute(0, 2, 3, 1).contiguous().cuda()
    wp = K.pack_conv_weight(w.cuda(), torch.bfloat16)
    rn = res.permute(0, 2, 3, 1).contiguous().cuda()
    y = K.conv2d_nhwc(xn, wp, s, p, scale=scale.cuda(), bias=bias.cuda(), relu=True, residual=rn)
    torch.cuda.synchronize()
    assert y.shape[0] * y.shape[1] * y.shape[2] >= 16384        # really on the big-tile path
    err = (y.permute(0, 3, 1, 2).float().cpu() - y_ref).abs()
    assert (err <= 1e-2 * y_ref.abs() + 2e-2).all(), err.max().item()


# ---- resident-weight streaming kernel (gemm_rw.hip: 16-bit, K in {64, 128, 256, 512}, M >= 4096) ----

def _rw_case(M, N, Kd, mode, seed, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(M, Kd, generator=g).to(dtype)
    x2 = torch.randn(M, Kd, generator=g).to(dtype)
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to(dtype)
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).to(dtype)
    mask = torch.rand(M, generator=g) < 0.1
    gam, bet = torch.rand(N, generator=g) + 0.5, torch.randn(N, generator=g)
    xin = (x.float() + x2.float()).to(dtype) if 'add' in mode else x
    ref = F.linear(xin.float(), w.float(), b)
    kw = {}
    if 'res' in mode:
        ref = ref + r.float()
        kw['residual'] = r.cuda()
    if 'relu' in mode:
        ref = F.relu(ref)
        kw['relu'] = True
    if 'ln' in mode:
        ref = F.layer_norm(ref, (N,), gam, bet, 1e-5)
        kw['ln'] = (gam.cuda(), bet.cuda(), 1e-5)
    if 'mask' in mode:
        ref = ref.masked_fill(mask[:, None], 0)
        kw['row_mask'] = mask.cuda()
    if 'add' in mode:
        kw['x_add'] = x2.cuda()
    if 'f32' in mode:
        kw['out_dtype'] = torch.float32
    return x, w, b, kw, ref


@pytest.mark.parametrize('M,N,Kd,mode', [
    (8192, 256, 256, 'plain'), (10001, 256, 256, 'res_ln'), (9999, 256, 256, 'ln_mask'),
    (12345, 1024, 256, 'relu'), (8200, 384, 256, 'add_f32'), (8200, 384, 256, 'add'),
    (8197, 200, 256, 'res_ln'), (8197, 200, 128, 'relu_mask'), (16800, 256, 64, 'res_relu'),
    (16800, 512, 128, 'res'), (5000, 64, 64, 'plain'), (4099, 1032, 256, 'f32'),
    (20001, 256, 256, 'res_relu_mask'),
    (9001, 128, 512, 'relu'), (8200, 256, 512, 'plain'), (8197, 200, 512, 'f32'),   # K = 512: 128-column groups
])
def test_rw_gemm_vs_fp32(K, M, N, Kd, mode):
    x, w, b, kw, ref = _rw_case(M, N, Kd, mode, M + N + Kd)
    y = K.linear(x.cuda(), w.cuda(), b.cuda(), **kw)
    torch.cuda.synchronize()
    assert y.dtype == (torch.float32 if 'f32' in mode else torch.bfloat16)
    err = (y.float().cpu() - ref).abs()
    tol = (1e-4 * ref.abs() + 2e-3) if 'f32' in mode else (1e-2 * ref.abs() + 2e-2)
    assert (err <= tol).all(), err.max().item()


@pytest.mark.parametrize('M,N,Kd,mode', [(10001, 256, 256, 'res_ln_mask'), (12345, 1024, 256, 'relu'),
                                         (8200, 384, 256, 'add_f32'), (16800, 256, 64, 'res_relu'),
                                         (9001, 128, 512, 'relu'), (8200, 256, 512, 'mask')])
def test_rw_matches_tiled_kernel(K, gemm_flags, M, N, Kd, mode):
    """Same bf16 products summed in the same K order in f32: the two kernels agree to
    (nearly) the last bit."""
    x, w, b, kw, _ = _rw_case(M, N, Kd, mode, 7)
    args = (x.cuda(), w.cuda(), b.cuda())
    gemm_flags(0)
    y_rw = K.linear(*args, **kw)
    gemm_flags(4)
    y_tiled = K.linear(*args, **kw)
    torch.cuda.synchronize()
    d = (y_rw.float() - y_tiled.float()).abs()
    tol = y_tiled.float().abs() * 2.0 ** -7 + 1e-5
    assert (d <= tol).all(), d.max().item()
    assert (d == 0).float().mean().item() > 0.9


def test_rw_headmajor_value_proj(K):
    B, S, d, hd = 2, 4500, 256, 32
    g = torch.Generator().manual_seed(12)
    x = torch.randn(B, S, d, generator=g).bfloat16()
    w = (torch.randn(d, d, generator=g) / 16).bfloat16()
    b = torch.randn(d, generator=g)
    mask = torch.rand(B, S, generator=g) < 0.2
    ref = F.linear(x.float(), w.float(), b).masked_fill(mask[..., None], 0)
    ref = ref.view(B, S, d // hd, hd).permute(2, 0, 1, 3)
    y = K.value_proj_headmajor(x.cuda(), w.cuda(), b.cuda(), hd, row_mask=mask.cuda())
    torch.cuda.synchronize()
    err = (y.float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()


@pytest.mark.parametrize('Cin,Cout,res', [(64, 256, True), (256, 64, True), (128, 512, True), (256, 1024, True),
                                          (512, 128, False), (512, 256, False)])
def test_rw_conv1x1(K, Cin, Cout, res):
    B, H, W = 4, 60, 70
    g = torch.Generator().manual_seed(Cin + Cout)
    x = torch.randn(B, Cin, H, W, generator=g).bfloat16()
    w = (torch.randn(Cout, Cin, 1, 1, generator=g) * (2.0 / Cin) ** 0.5).bfloat16()
    scale = torch.rand(Cout, generator=g) + 0.5
    bias = torch.randn(Cout, generator=g) * 0.1
    r = torch.randn(B, Cout, H, W, generator=g).bfloat16() if res else None
    ref = F.conv2d(x.float(), w.float()) * scale[None, :, None, None] + bias[None, :, None, None]
    ref = F.relu(ref + r.float() if res else ref)
    y = K.conv2d_nhwc(x.permute(0, 2, 3, 1).contiguous().cuda(), K.pack_conv_weight(w.cuda(), torch.bfloat16), 1, 0,
                      scale=scale.cuda(), bias=bias.cuda(), relu=True,
                      residual=r.permute(0, 2, 3, 1).contiguous().cuda() if res else None)
    torch.cuda.synchronize()
    err = (y.permute(0, 3, 1, 2).float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()


# ---- K = 288 (d = 288, configs 3-5): 16-row tiles, 12 columns per lane; LayerNorm rows on 6-wave
# 288-column groups, the other epilogues on 4-wave 192-column groups ----

@pytest.mark.parametrize('M,N,mode', [(20011, 288, 'res_ln'), (9000, 288, 'res_ln_mask'), (8197, 280, 'res_ln'),
                                      (9001, 288, 'ln'), (8200, 384, 'add'), (8200, 384, 'add_f32'),
                                      (8197, 288, 'plain'), (8197, 1728, 'relu'), (5000, 288, 'res_relu_mask'),
                                      (4099, 200, 'f32'), (12000, 296, 'res_mask')])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_rw288_vs_fp32(K, M, N, mode, dtype):
    """The K = 288 projections (value / offsets / output + LayerNorm of a d = 288 layer, the
    decoder's concatenated value projections) against torch fp32 on the same 16-bit operands:
    f32 accumulation, one output rounding."""
    x, w, b, kw, ref = _rw_case(M, N, 288, mode, M + N, dtype)
    y = K.linear(x.cuda(), w.cuda(), b.cuda(), **kw)
    torch.cuda.synchronize()
    assert y.dtype == (torch.float32 if 'f32' in mode else dtype)
    err = (y.float().cpu() - ref).abs()
    tol = (1e-4 * ref.abs() + 2e-3) if 'f32' in mode else (1e-2 * ref.abs() + 2e-2)
    assert (err <= tol).all(), err.max().item()


@pytest.mark.parametrize('M,N,mode', [(10001, 288, 'res_ln_mask'), (8200, 384, 'add'), (8197, 1728, 'relu'),
                                      (9001, 288, 'ln'), (8200, 384, 'add_f32')])
def test_rw288_matches_tiled_kernel(K, gemm_flags, M, N, mode):
    """K = 288 on the resident-weight kernel vs the tiled kernels (flag 1048576): the same
    16-bit products summed in the same K order in f32 -- (nearly) the last bit."""
    x, w, b, kw, _ = _rw_case(M, N, 288, mode, 9, torch.float16)
    args = (x.cuda(), w.cuda(), b.cuda())
    gemm_flags(0)
    y_rw = K.linear(*args, **kw)
    gemm_flags(1048576)
    y_tiled = K.linear(*args, **kw)
    torch.cuda.synchronize()
    d = (y_rw.float() - y_tiled.float()).abs()
    tol = y_tiled.float().abs() * 2.0 ** -9 + 1e-5
    assert (d <= tol).all(), d.max().item()
    assert (d == 0).float().mean().item() > 0.9


@pytest.mark.parametrize('M,N', [(20011, 256), (9001, 1536), (4103, 512), (8200, 256)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_rw_headmajor32_transpose_bit_identical(K, gemm_flags, M, N, dtype):
    """32-column head-major stores of the resident-weight kernel through its LDS transpose (one
    1 KiB head-plane piece per store, the default) vs the direct 16-byte unit stores (flag
    1073741824): the same values at the same places, ragged row counts included; and against fp32."""
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(1, M, 256, generator=g).to(dtype)
    w = (torch.randn(N, 256, generator=g) / 16).to(dtype)
    b = torch.randn(N, generator=g)
    mask = torch.rand(1, M, generator=g) < 0.1
    gemm_flags(0)
    y0 = K.value_proj_headmajor(x.cuda(), w.cuda(), b.cuda(), 32, row_mask=mask.cuda())
    gemm_flags(1073741824)
    y1 = K.value_proj_headmajor(x.cuda(), w.cuda(), b.cuda(), 32, row_mask=mask.cuda())
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    ref = F.linear(x.float(), w.float(), b).masked_fill(mask[..., None], 0).view(1, M, N // 32, 32).permute(2, 0, 1, 3)
    err = (y0.float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()


@pytest.mark.parametrize('M,N,Kd,mode', [(9001, 1728, 288, 'plain'), (4099, 500, 288, 'relu'), (8197, 400, 288, 'relu_mask')])
def test_rw_wide_group_variants_bit_identical(K, gemm_flags, M, N, Kd, mode):
    """K = 288 plain epilogues with N > 384 (the d = 288 decoder's six value projections in one
    launch): 8-wave 384-column groups (default) vs 4-wave groups (flag 268435456), row-major and
    head-major stores: bit-identical."""
    x, w, b, kw, ref = _rw_case(M, N, Kd, mode, 12, torch.bfloat16)
    args = (x.cuda(), w.cuda(), b.cuda())
    gemm_flags(0)
    y8 = K.linear(*args, **kw)
    gemm_flags(268435456)
    y4 = K.linear(*args, **kw)
    torch.cuda.synchronize()
    assert torch.equal(y8, y4)
    err = (y8.float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()
    if mode == 'plain':
        hd = 36
        gemm_flags(0)
        h8 = K.value_proj_headmajor(x.cuda().view(1, M, Kd), w.cuda(), b.cuda(), hd)
        gemm_flags(268435456)
        h4 = K.value_proj_headmajor(x.cuda().view(1, M, Kd), w.cuda(), b.cuda(), hd)
        torch.cuda.synchronize()
        assert torch.equal(h8, h4)


@pytest.mark.parametrize('M,N,Kd,mode', [(20011, 512, 128, 'res_relu'), (8197, 1024, 256, 'res_relu'),
                                         (9000, 512, 64, 'res_mask'), (4099, 400, 128, 'res')])
def test_rw_res_group_variants_bit_identical(K, gemm_flags, M, N, Kd, mode):
    """+ residual with N > 256 (the stage-end conv3s): 8-wave 512-column groups (default) vs
    4-wave 256-column groups (flag 268435456): the same products and epilogue per column, so
    bit-identical."""
    x, w, b, kw, ref = _rw_case(M, N, Kd, mode, 11, torch.bfloat16)
    args = (x.cuda(), w.cuda(), b.cuda())
    gemm_flags(0)
    y8 = K.linear(*args, **kw)
    gemm_flags(268435456)
    y4 = K.linear(*args, **kw)
    torch.cuda.synchronize()
    assert torch.equal(y8, y4)
    err = (y8.float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()


@pytest.mark.parametrize('M,N,mode', [(20011, 256, 'plain'), (8197, 200, 'relu'), (9000, 256, 'f32')])
def test_rw512_group_variants_bit_identical(K, gemm_flags, M, N, mode):
    """K = 512 with 128 < N <= 256 (config 2's level-0 input projection): one 8-wave 256-column
    group per row tile (default) vs two 4-wave 128-column groups (flag 268435456): the same
    products in the same K order per column, so bit-identical."""
    x, w, b, kw, ref = _rw_case(M, N, 512, mode, 3, torch.bfloat16)
    args = (x.cuda(), w.cuda(), b.cuda())
    gemm_flags(0)
    y8 = K.linear(*args, **kw)
    gemm_flags(268435456)
    y4 = K.linear(*args, **kw)
    torch.cuda.synchronize()
    assert torch.equal(y8, y4)
    err = (y8.float().cpu() - ref).abs()
    tol = (1e-4 * ref.abs() + 2e-3) if 'f32' in mode else (1e-2 * ref.abs() + 2e-2)
    assert (err <= tol).all(), err.max().item()


@pytest.mark.parametrize('M,N,mode', [(8200, 384, 'add'), (8200, 384, 'add_f32'), (20011, 288, 'add'), (4099, 200, 'add')])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_rw288_add_group_variants_bit_identical(K, gemm_flags, M, N, mode, dtype):
    """K = 288 with the second operand added on load and 192 < N <= 384: one 8-wave group of up
    to 384 columns per row tile (default) vs two 4-wave 192-column groups (flag 268435456): the
    same products in the same K order per column, so bit-identical."""
    x, w, b, kw, _ = _rw_case(M, N, 288, mode, 5, dtype)
    args = (x.cuda(), w.cuda(), b.cuda())
    gemm_flags(0)
    y8 = K.linear(*args, **kw)
    gemm_flags(268435456)
    y4 = K.linear(*args, **kw)
    torch.cuda.synchronize()
    assert torch.equal(y8, y4)


@pytest.mark.parametrize('M,N,mode', [(10001, 288, 'res_ln_mask'), (20011, 288, 'res_ln'), (8197, 280, 'res_ln'),
                                      (9001, 288, 'ln')])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_rw288_ln_wave_variants(K, gemm_flags, M, N, mode, dtype):
    """The LayerNorm rows of the K = 288 kernel on 9 waves x 32 columns (the default) vs 6 waves
    x 48 columns (flag 4194304): the same products in the same K order per column; only the row
    statistics' partial sums are grouped differently (f32) -- within one output rounding, mostly
    equal."""
    x, w, b, kw, ref = _rw_case(M, N, 288, mode, 21, dtype)
    args = (x.cuda(), w.cuda(), b.cuda())
    gemm_flags(0)
    y9 = K.linear(*args, **kw)
    gemm_flags(4194304)
    y6 = K.linear(*args, **kw)
    torch.cuda.synchronize()
    d = (y9.float() - y6.float()).abs()
    tol = y6.float().abs() * (2.0 ** -7 if dtype == torch.bfloat16 else 2.0 ** -10) + 1e-5
    assert (d <= tol).all(), d.max().item()
    assert (d == 0).float().mean().item() > 0.9
    err = (y9.float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()


@pytest.mark.parametrize('hd', [36, 48, 'split'])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_rw288_headmajor(K, hd, dtype):
    """Head-major stores of the K = 288 kernel in 4-column units: the d = 288 value projection
    (8 heads x 36), the offsets / logits projection layout (8 x 48) and the split planes
    (32-channel + 4-channel) of the head_dim-36 strip encoder."""
    B, S, d = 2, 4700, 288
    Nout = 384 if hd == 48 else 288
    g = torch.Generator().manual_seed(13)
    x = torch.randn(B, S, d, generator=g).to(dtype)
    w = (torch.randn(Nout, d, generator=g) / 17).to(dtype)
    b = torch.randn(Nout, generator=g)
    mask = torch.rand(B, S, generator=g) < 0.2
    ref = F.linear(x.float(), w.float(), b).masked_fill(mask[..., None], 0)      # (B, S, Nout)
    if hd == 'split':
        ws, bs = K.split_value_weights(w.cuda(), b.cuda(), 8)
        sv = K.value_proj_headmajor_split(x.cuda(), ws, bs, 8, row_mask=mask.cuda())
        torch.cuda.synchronize()
        y = torch.cat([sv.main, sv.tail], -1)                                     # (8, B, S, 36)
        ref = ref.view(B, S, 8, 36).permute(2, 0, 1, 3)
    else:
        y = K.value_proj_headmajor(x.cuda(), w.cuda(), b.cuda(), hd, row_mask=mask.cuda())
        torch.cuda.synchronize()
        ref = ref.view(B, S, Nout // hd, hd).permute(2, 0, 1, 3)
    assert tuple(y.shape) == tuple(ref.shape)
    err = (y.float().cpu() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), err.max().item()


@pytest.mark.parametrize('case', ['plain128', 'relu_mask256', 'f32_256', 'f16out_256', 'headmajor', 'conv1x1_128',
                                  'conv1x1_s2'])
def test_rw_row_tile_variants_bit_identical(K, gemm_flags, case):
    """The resident-weight kernel's shipped 32-row tiles (two MFMA row tiles per wave, TMR = 2:
    plain / masked / head-major GEMMs with K = 128 / 256 and no residual or LayerNorm, the 1x1
    convs, the strided conv-row downsample) give the 16-row tiles' results bit for bit
    (kinet_gemm_set_flags 131072) -- the 32-row SAMPLING-RECORDS tile of round 4 differed from
    its 16-row tile, and these share its ring, counted waits and pending stores."""
    g = torch.Generator().manual_seed(hash(case) % 1000)
    def run(flags):
        gemm_flags(flags)
        if case.startswith('conv1x1'):
            st = 2 if case.endswith('s2') else 1
            cin, cout = (256, 512) if st == 2 else (128, 256)
            x = torch.randn(2, 80 if st == 2 else 60, 130, cin, generator=torch.Generator().manual_seed(3)).bfloat16()
            w = (torch.randn(cout, cin, 1, 1, generator=torch.Generator().manual_seed(4)) / cin ** 0.5).bfloat16()
            sc = torch.rand(cout, generator=torch.Generator().manual_seed(5)) + 0.5
            bi = torch.randn(cout, generator=torch.Generator().manual_seed(6))
            return K.conv2d_nhwc(x.cuda(), K.pack_conv_weight(w.cuda(), torch.bfloat16), st, 0, scale=sc.cuda(),
                                 bias=bi.cuda(), relu=True)
        if case == 'headmajor':
            x = torch.randn(2, 4500, 256, generator=torch.Generator().manual_seed(7)).bfloat16()
            w = (torch.randn(256, 256, generator=torch.Generator().manual_seed(8)) / 16).bfloat16()
            b = torch.randn(256, generator=torch.Generator().manual_seed(9))
            m = torch.rand(2, 4500, generator=torch.Generator().manual_seed(10)) < 0.2
            return K.value_proj_headmajor(x.cuda(), w.cuda(), b.cuda(), 32, row_mask=m.cuda(), out_dtype=torch.float16)
        Kd = 128 if case.endswith('128') else 256
        M, N = 10007, 384
        x, w, b, kw, _ = _rw_case(M, N, Kd, {'plain128': 'plain', 'relu_mask256': 'relu_mask', 'f32_256': 'f32',
                                             'f16out_256': 'plain'}[case], 21)
        if case == 'f16out_256':
            kw['out_dtype'] = torch.float16
        return K.linear(x.cuda(), w.cuda(), b.cuda(), **kw)
    y32 = run(0)
    y16 = run(131072)
    gemm_flags(0)
    torch.cuda.synchronize()
    assert y32.shape == y16.shape
    assert torch.equal(y32, y16), (y32.float() - y16.float()).abs().max().item()


# ---- split-K (few output tiles, long K): f32 slice partials + finalize epilogue ----------------

@pytest.mark.parametrize('M,N,Kd,mode', [(1200, 256, 1024, 'res_ln_mask'), (4200, 256, 2048, 'plain'),
                                         (1000, 91, 2048, 'relu'), (300, 1100, 1024, 'res')])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_splitk_linear_vs_fp32(K, M, N, Kd, mode, dtype):
    assert K.ksplit_for(M, N, Kd, 'ln' in mode) > 1
    x, w, b, kw, ref = _rw_case(M, N, Kd, mode, M + Kd)
    xx = x.float().to(dtype) if dtype == torch.float32 else x
    if dtype == torch.float32 and 'res' in mode:
        kw['residual'] = kw['residual'].float()
    y = K.linear(xx.cuda(), w.cuda().to(dtype), b.cuda(), **kw)
    torch.cuda.synchronize()
    err = (y.float().cpu() - ref).abs()
    tol = (1e-4 * ref.abs() + 1e-4) if dtype == torch.float32 else (1e-2 * ref.abs() + 2e-2)
    assert (err <= tol).all(), err.max().item()


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_splitk_conv_vs_fp32(K, dtype):
    """input_proj of the last level: 3x3 stride-2 conv 2048 -> 256 on a small map (M ~ 1k, K 18k)."""
    B, H, W, Cin, Cout = 2, 25, 42, 2048, 256
    assert K.ksplit_for(B * 13 * 21, Cout, 9 * Cin) > 1
    g = torch.Generator().manual_seed(17)
    x = torch.randn(B, Cin, H, W, generator=g).to(dtype)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (Cin * 9)) ** 0.5).to(dtype)
    bias = torch.randn(Cout, generator=g) * 0.1
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=1) + bias[None, :, None, None]
    y = K.conv2d_nhwc(x.permute(0, 2, 3, 1).contiguous().cuda(), K.pack_conv_weight(w.cuda(), dtype), 2, 1,
                      bias=bias.cuda())
    torch.cuda.synchronize()
    err = (y.permute(0, 3, 1, 2).float().cpu() - ref).abs()
    tol = (1e-4 * ref.abs() + 1e-4) if dtype == torch.float32 else (1e-2 * ref.abs() + 2e-2)
    assert (err <= tol).all(), err.max().item()


@pytest.mark.parametrize('M,D', [(1, 256), (200, 256), (2400, 256), (20000, 256), (777, 288), (17000, 288)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_ffn_fused_vs_fp32(K, M, D, dtype):
    """Fused FFN sub-layer (kinet_ffn_fused) vs fp32 LN(x + W2 relu(W1 x + b1) + b2) on the
    16-bit inputs/weights, hidden rounded to the 16-bit type like the unfused path stores it."""
    Fh = 1024
    g = torch.Generator().manual_seed(M + D)
    lin1, lin2, norm = torch.nn.Linear(D, Fh), torch.nn.Linear(Fh, D), torch.nn.LayerNorm(D)
    with torch.no_grad():
        for p in (norm.weight, norm.bias):
            p.copy_(torch.randn(p.shape, generator=g) * 0.5 + (1.0 if p is norm.weight else 0.0))
    x = torch.randn(M, D, generator=g).to(dtype)
    w1, w2 = lin1.weight.detach().to(dtype).float(), lin2.weight.detach().to(dtype).float()
    h = F.relu(F.linear(x.float(), w1, lin1.bias.detach())).to(dtype).float()
    ref = F.layer_norm(x.float() + F.linear(h, w2, lin2.bias.detach()), (D,), norm.weight.detach(), norm.bias.detach())
    lin1, lin2, norm = lin1.cuda(), lin2.cuda(), norm.cuda()
    y = K.ffn_fused(x.cuda(), lin1, lin2, norm)
    torch.cuda.synchronize()
    assert y.shape == (M, D) and y.dtype == dtype
    err = (y.float().cpu() - ref).abs().max().item()
    assert err < (6e-2 if dtype == torch.bfloat16 else 8e-3), err
    # the unfused kinet path (two GEMMs, LN in the second epilogue) agrees to output rounding:
    # one 16-bit ulp of the larger magnitude (bf16: 2^-7 relative; 0.0625 for |y| in [8, 16))
    hk = K.linear(x.cuda(), lin1.weight, lin1.bias, relu=True)
    yk = K.linear(hk, lin2.weight, lin2.bias, residual=x.cuda(), ln=(norm.weight, norm.bias, norm.eps))
    d = (y.float() - yk.float()).abs()
    ulp = 2.0 ** -7 if dtype == torch.bfloat16 else 2.0 ** -10
    assert (d <= ulp * torch.maximum(y.float().abs(), yk.float().abs()) + 3 * ulp).all(), d.max().item()


def test_ffn_fused_no_norm_and_errors(K):
    lin1, lin2 = torch.nn.Linear(256, 1024).cuda(), torch.nn.Linear(1024, 256).cuda()
    x = torch.randn(300, 256, device='cuda').bfloat16()
    y = K.ffn_fused(x, lin1, lin2, None)
    ref = x.float() + lin2(torch.relu(lin1(x.float())).bfloat16().float())
    assert (y.float() - ref).abs().max().item() < 5e-2
    lin1b, lin2b = torch.nn.Linear(128, 1024).cuda(), torch.nn.Linear(1024, 128).cuda()
    with pytest.raises(RuntimeError, match='D must be 256 or 288'):
        K.ffn_fused(torch.randn(10, 128, device='cuda').bfloat16(), lin1b, lin2b, None)


@pytest.mark.parametrize('B,H,W,Cin,Cout,k,s,p', [
    (16, 50, 84, 256, 256, 3, 1, 1),    # 263 tiles of 256x256: one full round + a 4-wave remainder launch
    (8, 50, 84, 256, 256, 3, 1, 1),     # 132 tiles: one partial round of 8-wave tiles
    (16, 25, 42, 512, 512, 3, 1, 1),    # layer-4 3x3 (N = 2 tile columns)
    (4, 68, 120, 256, 256, 3, 1, 1),    # config-5 stage 3: 128 tiles of 256x256 -> 255 of 128x256
])
def test_conv_full_rounds_split_vs_fp32(K, B, H, W, Cin, Cout, k, s, p):
    """Multi-tap convs split into whole rounds of 8-wave 256x256 tiles + the remainder rows on
    the 4-wave tiles (csrc/gemm.hip launch): fused BN / residual / ReLU epilogue vs fp32."""
    g = torch.Generator().manual_seed(H * W + Cin + Cout + B)
    x = torch.randn(B, Cin, H, W, generator=g).bfloat16()
    w = (torch.randn(Cout, Cin, k, k, generator=g) * (2.0 / (Cin * k * k)) ** 0.5).bfloat16()
    scale = torch.rand(Cout, generator=g) + 0.5
    bias = torch.randn(Cout, generator=g) * 0.1
    xc, wc = x.cuda(), w.cuda()
    y_ref = F.conv2d(xc.float(), wc.float(), stride=s, padding=p) * scale.cuda()[None, :, None, None] \
        + bias.cuda()[None, :, None, None]
    res = torch.randn(y_ref.shape, generator=g).bfloat16().cuda()
    y_ref = F.relu(y_ref + res.float())
    wp = K.pack_conv_weight(wc, torch.bfloat16)
    y = K.conv2d_nhwc(xc.permute(0, 2, 3, 1).contiguous(), wp, s, p, scale=scale.cuda(), bias=bias.cuda(), relu=True,
                      residual=res.permute(0, 2, 3, 1).contiguous())
    err = (y.permute(0, 3, 1, 2).float() - y_ref).abs()
    assert (err <= 1e-2 * y_ref.abs() + 2e-2).all(), err.max().item()


# ---- KINET_F32_X3: f32 operands as three bf16 MFMA passes (torch float32_matmul_precision 'high')
@pytest.fixture
def x3_precision():
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision('high')
    yield
    torch.set_float32_matmul_precision(prev)


def _x3_bound(a64, b64):
    # per-product error <= ~2^-16 |a||b| (hi/lo split of both operands, lo*lo dropped), plus
    # f32 accumulation: bound by 4e-5 * (|A| @ |B|) elementwise
    return 4e-5 * (a64.abs() @ b64.abs()) + 1e-6


@pytest.mark.parametrize('M,N,Kd', [(37, 91, 256), (1000, 1024, 256), (513, 256, 1024), (4200, 384, 2048),
                                    (9001, 288, 1024), (9001, 288, 288), (5000, 200, 64)])
def test_linear_f32_x3_vs_f64(K, x3_precision, M, N, Kd):
    g = torch.Generator().manual_seed(M + N + Kd)
    x = torch.randn(M, Kd, generator=g, dtype=torch.float64)
    w = torch.randn(N, Kd, generator=g, dtype=torch.float64) / Kd ** 0.5
    ref = x @ w.T
    y = K.linear(x.float().cuda(), w.float().cuda())
    torch.cuda.synchronize()
    err = (y.double().cpu() - ref).abs()
    # f32 rounding of the operands themselves is part of the bound (2^-24 each)
    assert (err <= _x3_bound(x, w.T) + 2e-7 * (x.abs() @ w.abs().T)).all(), err.max().item()
    # and it is not the exact-f32 path: that one is ~100x tighter
    torch.set_float32_matmul_precision('highest')
    y2 = K.linear(x.float().cuda(), w.float().cuda())
    torch.set_float32_matmul_precision('high')
    torch.cuda.synchronize()
    assert (y2.double().cpu() - ref).abs().max() < err.max() or err.max() == 0


@pytest.mark.parametrize('ks', [1, 3])
def test_conv_f32_x3_vs_f64(K, x3_precision, ks):
    g = torch.Generator().manual_seed(5 + ks)
    B, H, W, Cin, Cout = 2, 23, 31, 64, 128
    x = torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (9 * Cin) ** 0.5
    ref = F.conv2d(x, w, padding=1)
    bound = 4e-5 * F.conv2d(x.abs(), w.abs(), padding=1) + 1e-6
    xn = x.float().permute(0, 2, 3, 1).contiguous().cuda()
    wp = w.float().permute(0, 2, 3, 1).contiguous().cuda()
    y = K.conv2d_nhwc(xn, wp, 1, 1, ksplit=ks)
    torch.cuda.synchronize()
    err = (y.double().cpu().permute(0, 3, 1, 2) - ref).abs()
    assert (err <= bound).all(), err.max().item()


@pytest.mark.parametrize('Kd,M,N', [(40000, 256, 288), (999, 70, 33)])
def test_gemm_tn_f32_x3_vs_f64(K, x3_precision, Kd, M, N):
    g = torch.Generator().manual_seed(Kd)
    a = torch.randn(Kd, M, generator=g, dtype=torch.float64)
    b = torch.randn(Kd, N, generator=g, dtype=torch.float64)
    ref = a.T @ b
    y = K.gemm_tn(a.float().cuda(), b.float().cuda())
    torch.cuda.synchronize()
    err = (y.double().cpu() - ref).abs()
    assert (err <= _x3_bound(a.T, b)).all(), err.max().item()


@pytest.mark.parametrize('B,H,W', [(2, 200, 334), (3, 37, 45), (1, 8, 32), (1, 5, 7)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_direct_conv3x3_c64_vs_fp32(K, B, H, W, dtype):
    """The direct 3x3 / stride 1 / pad 1, 64 -> 64 conv (csrc/conv3x3.hip: ResNet layer-1 conv2,
    weights resident in VGPRs, halo tiles in LDS) against torch fp32 F.conv2d + folded BN +
    ReLU, at the config-2 layer-1 size and at ragged sizes (partial 8 x 32 tiles, an image
    smaller than one tile); and against the implicit-GEMM path (flag 1024) on the same inputs
    (same products, other summation order: within one output rounding)."""
    from kinet_amd import _native
    g = torch.Generator().manual_seed(H * W + B)
    x = torch.randn(B, 64, H, W, generator=g).to(dtype)
    w = (torch.randn(64, 64, 3, 3, generator=g) * (2.0 / 576) ** 0.5).to(dtype)
    scale = torch.rand(64, generator=g) + 0.5
    bias = torch.randn(64, generator=g) * 0.1
    y_ref = F.relu(F.conv2d(x.float(), w.float(), padding=1) * scale[None, :, None, None] + bias[None, :, None, None])
    xn = x.permute(0, 2, 3, 1).contiguous().cuda()
    wp = K.pack_conv_weight(w.cuda(), dtype)
    y = K.conv2d_nhwc(xn, wp, 1, 1, scale=scale.cuda(), bias=bias.cuda(), relu=True)
    old = _native.lib().kinet_gemm_set_flags(1024)
    try:
        y_gemm = K.conv2d_nhwc(xn, wp, 1, 1, scale=scale.cuda(), bias=bias.cuda(), relu=True)
    finally:
        _native.lib().kinet_gemm_set_flags(old)
    torch.cuda.synchronize()
    err = (y.permute(0, 3, 1, 2).float().cpu() - y_ref).abs()
    ulp = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    assert (err <= 2 * ulp * y_ref.abs() + 1e-3).all(), err.max().item()
    d = (y.float() - y_gemm.float()).abs()
    assert (d <= 2 * ulp * y_gemm.float().abs() + 1e-3).all(), d.max().item()
    # unscaled, no ReLU: negative outputs pass through
    y2 = K.conv2d_nhwc(xn, wp, 1, 1)
    torch.cuda.synchronize()
    r2 = F.conv2d(x.float(), w.float(), padding=1)
    assert ((y2.permute(0, 3, 1, 2).float().cpu() - r2).abs() <= 2 * ulp * r2.abs() + 1e-3).all()


@pytest.mark.parametrize('M', [16384, 40007, 355568])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_ffn_fused_tile_variants_bit_identical(K, M, dtype):
    """The fused FFN's tile variants (kinet_ffn_set_debug: 0 = 8 waves x 32 rows without the
    cross-chunk pipeline, 2 = 4 waves x 32 rows, 8 = 8 waves x 16 rows) sum every output element
    in the same order: bit-identical outputs, incl. a ragged last tile."""
    from kinet_amd import _native
    g = torch.Generator().manual_seed(M)
    lin1, lin2, norm = torch.nn.Linear(256, 1024).cuda(), torch.nn.Linear(1024, 256).cuda(), torch.nn.LayerNorm(256).cuda()
    x = torch.randn(M, 256, generator=g).to(dtype).cuda()
    outs = []
    try:
        for knob in (0, 2, 8):
            _native.lib().kinet_ffn_set_debug(knob)
            outs.append(K.ffn_fused(x, lin1, lin2, norm))
    finally:
        _native.lib().kinet_ffn_set_debug(0)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize('D,B,H,W,DB', [(64, 2, 37, 53, 64), (64, 16, 200, 334, 64), (128, 3, 29, 31, 128),
                                        (128, 16, 100, 167, 128), (256, 2, 25, 42, 256), (256, 16, 50, 84, 256),
                                        (256, 1, 1, 5, 256), (64, 2, 37, 53, 128), (64, 16, 200, 334, 128),
                                        (64, 1, 1, 3, 128)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_bottleneck_pair_vs_fp32(K, D, B, H, W, DB, dtype):
    """kinet_bottleneck_pair (block i's conv3 + BN + residual + ReLU -> block i+1's conv1 + BN +
    ReLU in one launch) against torch fp32 on the same rounded weights (the pack folds the BN
    scales into the weight rows before rounding): y within 2 output ulps of the fp32 result, t
    within 2 ulps of the fp32 conv1 of OUR y; ragged row counts (partial 256-row tiles, 5 rows)
    and the config-2 layer-1..3 sizes; DB = 128 at D = 64 is the stage-1 -> stage-2 pair."""
    if dtype == torch.float16 and B == 16 and D != 64:
        pytest.skip('f16 covered at the layer-1 size and the ragged sizes')
    F_ = 4 * D
    g = torch.Generator().manual_seed(D * 1000 + H)
    dev = 'cuda'
    x = torch.relu(torch.randn(B, H, W, D, generator=g)).to(dtype).to(dev)
    res = torch.randn(B, H, W, F_, generator=g).to(dtype).to(dev)
    w3 = (torch.randn(F_, D, 1, 1, generator=g) * (2.0 / D) ** 0.5).to(dev)
    w1 = (torch.randn(DB, F_, 1, 1, generator=g) * (2.0 / F_) ** 0.5).to(dev)
    s3, b3 = (torch.rand(F_, generator=g) + 0.5).to(dev), (torch.randn(F_, generator=g) * 0.1).to(dev)
    s1, b1 = (torch.rand(DB, generator=g) + 0.5).to(dev), (torch.randn(DB, generator=g) * 0.1).to(dev)
    packed = K.bottleneck_pack(w3, w1, s3, s1, dtype)
    y, t = K.bottleneck_pair(x, res, packed, b3, b1)
    torch.cuda.synchronize()
    w3r = (w3.reshape(F_, D) * s3[:, None]).to(dtype).float()
    w1r = (w1.reshape(DB, F_) * s1[:, None]).to(dtype).float()
    y_ref = torch.relu(x.reshape(-1, D).float() @ w3r.T + b3 + res.reshape(-1, F_).float())
    ulp = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    ey = (y.reshape(-1, F_).float() - y_ref).abs()
    assert (ey <= 2 * ulp * y_ref.abs() + 1e-3).all(), ey.max().item()
    t_ref = torch.relu(y.reshape(-1, F_).float() @ w1r.T + b1)
    et = (t.reshape(-1, DB).float() - t_ref).abs()
    assert (et <= 2 * ulp * t_ref.abs() + 1e-3).all(), et.max().item()


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_backbone_bottleneck_pairs_match_unfused(dtype):
    """ResNet-50 body with the fused bottleneck pairs vs every conv on its own (FUSE_BOTTLENECK_PAIRS
    = False): the pair folds the BN scale into the rounded weights instead of the epilogue, so the
    stage outputs agree to bf16 / f16 accumulation level, not bit for bit."""
    from kinet_amd.models import backbone as BB
    torch.manual_seed(0)
    body = BB.ResNetBody([3, 4, 6, 3]).cuda().eval()
    with torch.no_grad():
        for m in body.modules():
            if isinstance(m, BB.FrozenBatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.normal_(0, 0.1)
                m.running_mean.normal_(0, 0.1)
                m.running_var.uniform_(0.5, 1.5)
    img = torch.randn(2, 3, 160, 224, device='cuda')
    old = BB.FUSE_BOTTLENECK_PAIRS, BB.FUSE_PAIR_WIDTHS
    try:
        BB.FUSE_BOTTLENECK_PAIRS, BB.FUSE_PAIR_WIDTHS = True, (64, 128, 256)
        fused = body.forward_nhwc(img, dtype)
        BB.FUSE_BOTTLENECK_PAIRS = False
        plain = body.forward_nhwc(img, dtype)
    finally:
        BB.FUSE_BOTTLENECK_PAIRS, BB.FUSE_PAIR_WIDTHS = old
    torch.cuda.synchronize()
    for a, b in zip(fused, plain):
        assert a.shape == b.shape
        rel = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert rel < (3e-2 if dtype == torch.bfloat16 else 5e-3), rel


@pytest.mark.parametrize('M', [5, 1000, 1068800])
def test_bottleneck_pair64_kernels_bit_identical(K, M):
    """At D = 64 the LDS-resident wave-independent kernel (default) and the LDS-ring kernel
    (kinet_ffn_set_debug 16) sum every element in the same order: bit-identical y and t."""
    from kinet_amd import _native
    g = torch.Generator().manual_seed(M)
    x = torch.relu(torch.randn(M, 1, 1, 64, generator=g)).bfloat16().cuda()
    res = torch.randn(M, 1, 1, 256, generator=g).bfloat16().cuda()
    w3 = (torch.randn(256, 64, 1, 1, generator=g) * 0.2).cuda()
    w1 = (torch.randn(64, 256, 1, 1, generator=g) * 0.1).cuda()
    s3, b3, s1, b1 = (torch.rand(256) + 0.5).cuda(), torch.randn(256).cuda() * 0.1, (torch.rand(64) + 0.5).cuda(), torch.randn(64).cuda() * 0.1
    packed = K.bottleneck_pack(w3, w1, s3, s1, torch.bfloat16)
    y0, t0 = K.bottleneck_pair(x, res, packed, b3, b1)
    old = _native.lib().kinet_ffn_set_debug(16)
    try:
        y1, t1 = K.bottleneck_pair(x, res, packed, b3, b1)
    finally:
        _native.lib().kinet_ffn_set_debug(old)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(t0, t1)


@pytest.mark.parametrize('D,M', [(128, 5), (128, 32640), (256, 5), (256, 1000), (256, 32640), (256, 117600)])
def test_bottleneck_pair_row_tiles_bit_identical(K, D, M):
    """At D = 128 / 256 the pair runs one or two 16-row tiles per wave (chosen by how well the
    tiles fill rounds of one workgroup per CU; kinet_ffn_set_debug 128 / 256 force either): the
    same sums per element, so bit-identical y and t; the automatic choice runs under
    kinet_set_solo_launch 1 (the only mode that picks the 1-tile grid by itself)."""
    from kinet_amd import _native
    g = torch.Generator().manual_seed(M + D)
    F_ = 4 * D
    x = torch.relu(torch.randn(M, 1, 1, D, generator=g)).bfloat16().cuda()
    res = torch.randn(M, 1, 1, F_, generator=g).bfloat16().cuda()
    w3 = (torch.randn(F_, D, 1, 1, generator=g) * (2.0 / D) ** 0.5).cuda()
    w1 = (torch.randn(D, F_, 1, 1, generator=g) * (2.0 / F_) ** 0.5).cuda()
    s3, b3 = (torch.rand(F_, generator=g) + 0.5).cuda(), (torch.randn(F_, generator=g) * 0.1).cuda()
    s1, b1 = (torch.rand(D, generator=g) + 0.5).cuda(), (torch.randn(D, generator=g) * 0.1).cuda()
    packed = K.bottleneck_pack(w3, w1, s3, s1, torch.bfloat16)
    outs = []
    for knob, solo in ((0, 0), (0, 1), (128, 0), (256, 0)):
        old, old_solo = _native.lib().kinet_ffn_set_debug(knob), _native.lib().kinet_set_solo_launch(solo)
        try:
            outs.append(K.bottleneck_pair(x, res, packed, b3, b1))
        finally:
            _native.lib().kinet_ffn_set_debug(old)
            _native.lib().kinet_set_solo_launch(old_solo)
    torch.cuda.synchronize()
    for y, t in outs[1:]:
        assert torch.equal(outs[0][0], y) and torch.equal(outs[0][1], t)


@pytest.mark.parametrize('B,H,W', [(4, 68, 120), (8, 50, 84)])
def test_conv_partial_round_tiles_bit_identical(K, B, H, W):
    """With one batch in flight (kinet_set_solo_launch 1) a multi-tap conv whose 256x256 tiles
    would fill under 60 % of one round runs 128x256 tiles instead (csrc/gemm.hip): the same K
    order per element, so bit-identical outputs to the default 256x256 round."""
    from kinet_amd import _native
    g = torch.Generator().manual_seed(B * H * W)
    x = torch.randn(B, H, W, 256, generator=g).bfloat16().cuda()
    w = (torch.randn(256, 256, 3, 3, generator=g) * (2.0 / 2304) ** 0.5).bfloat16().cuda()
    scale, bias = (torch.rand(256, generator=g) + 0.5).cuda(), (torch.randn(256, generator=g) * 0.1).cuda()
    wp = K.pack_conv_weight(w, torch.bfloat16)
    y0 = K.conv2d_nhwc(x, wp, 1, 1, scale=scale, bias=bias, relu=True)
    old = _native.lib().kinet_set_solo_launch(1)
    try:
        y1 = K.conv2d_nhwc(x, wp, 1, 1, scale=scale, bias=bias, relu=True)
    finally:
        _native.lib().kinet_set_solo_launch(old)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)


@pytest.mark.parametrize('B,H,W,N', [(16, 200, 334, 512), (2, 67, 81, 256), (1, 64, 64, 512)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_strided_conv1x1_rw_vs_fp32(K, B, H, W, N, dtype):
    """The strided 1x1 conv (ResNet stage-2 downsample, 256 -> 512 at stride 2) on the
    resident-weight conv-row kernel against torch fp32 F.conv2d + folded BN, at the config-2 size
    and ragged sizes (odd H / W, partial row tiles); and against the implicit-GEMM kernel
    (kinet_gemm_set_flags 2048) on the same inputs."""
    from kinet_amd import _native
    g = torch.Generator().manual_seed(H * W + N)
    x = torch.relu(torch.randn(B, 256, H, W, generator=g)).to(dtype)
    w = (torch.randn(N, 256, 1, 1, generator=g) * (1.0 / 256) ** 0.5).to(dtype)
    scale = torch.rand(N, generator=g) + 0.5
    bias = torch.randn(N, generator=g) * 0.1
    xn = x.permute(0, 2, 3, 1).contiguous().cuda()
    wp = K.pack_conv_weight(w.cuda(), dtype)
    y = K.conv2d_nhwc(xn, wp, 2, 0, scale=scale.cuda(), bias=bias.cuda())
    old = _native.lib().kinet_gemm_set_flags(2048)
    try:
        y_gemm = K.conv2d_nhwc(xn, wp, 2, 0, scale=scale.cuda(), bias=bias.cuda())
    finally:
        _native.lib().kinet_gemm_set_flags(old)
    torch.cuda.synchronize()
    ref = (F.conv2d(x.float().cuda(), w.float().cuda(), stride=2) * scale.cuda()[None, :, None, None]
           + bias.cuda()[None, :, None, None])
    ulp = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    err = (y.permute(0, 3, 1, 2).float() - ref).abs()
    assert (err <= 2 * ulp * ref.abs() + 1e-3).all(), err.max().item()
    d = (y.float() - y_gemm.float()).abs()
    assert (d <= 2 * ulp * y_gemm.float().abs() + 1e-3).all(), d.max().item()


@pytest.mark.parametrize('B,H,W', [(2, 50, 66), (1, 37, 41), (2, 800, 1333), (1, 1080, 1920), (1, 9, 7)])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_stem_conv_image_equals_folded_path(K, B, H, W, dtype):
    """kinet_stem_conv_image (folded rows built in LDS from the f32 image) is bit-identical to
    pack_image_kwfold + the folded stem conv (same rounded inputs, same MFMA order), incl. ragged
    tiles and an image smaller than one tile; and both match torch fp32 conv1 + BN + ReLU."""
    g = torch.Generator().manual_seed(H * W + B)
    img = torch.randn(B, 3, H, W, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    scale = torch.rand(64, generator=g) + 0.5
    bias = torch.randn(64, generator=g) * 0.1
    wp = K.pack_stem_weight(w.cuda(), dtype, 24)
    xp = K.pack_image_kwfold(img.cuda(), dtype, 7, 2, 3, 24)
    y0 = K.conv2d_nhwc(xp, wp, (2, 1), (3, 0), scale=scale.cuda(), bias=bias.cuda(), relu=True)
    y1 = K.stem_conv_image(img.cuda(), wp, scale.cuda(), bias.cuda(), dtype)
    torch.cuda.synchronize()
    assert y1.shape == y0.shape
    assert torch.equal(y0, y1)
    if H * W < 10 ** 6:
        ref = F.relu(F.conv2d(img, w, stride=2, padding=3) * scale[None, :, None, None] + bias[None, :, None, None])
        assert _rel(y1.permute(0, 3, 1, 2), ref) < 2e-2

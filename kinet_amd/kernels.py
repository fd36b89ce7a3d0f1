"""Thin torch-tensor front-end over the kinet_amd C-ABI (include/*.h).

Every function launches hand-written HIP kernels from libkinet_amd.so on the current
stream; nothing here falls back to a torch/CPU implementation.  Weights stay torch
Parameters (reference layout, so state_dicts load unchanged); converted copies (dtype
casts, OIHW->OHWI conv packing, folded FrozenBatchNorm) are cached per parameter
version.
"""
import weakref

import torch

from kinet_amd import _native as N

_cache = {}   # id(tensor) -> (weakref(tensor), {tag: ((version, data_ptr), value)})


def _drop(key):
    def cb(ref, _c=_cache):
        ent = _c.get(key) if _c is not None else None
        if ent is not None and ent[0] is ref:   # a newer tensor may have reused the id
            del _c[key]
    return cb


def cached(t, tag, make):
    """Cache make(t) per tensor object (identity-keyed and weakly held, so a freed
    temporary never aliases a new tensor at the same address), invalidated by in-place
    updates (_version)."""
    if t is None:
        return None
    key = id(t)
    ent = _cache.get(key)
    if ent is None or ent[0]() is not t:
        ent = (weakref.ref(t, _drop(key)), {})
        _cache[key] = ent
    slot = ent[1]
    hit = slot.get(tag)
    ver = (t._version, t.data_ptr())
    if hit is not None and hit[0] == ver:
        return hit[1]
    v = make(t)
    slot[tag] = (ver, v)
    return v


def clear_cache():
    _cache.clear()


def cache_values():
    """Strong references to every cached value (HIP-graph recordings keep them allocated)."""
    return [hit[1] for ent in list(_cache.values()) for hit in ent[1].values()]


def cached_multi(tensors, tag, make):
    """Cache make(*tensors) on the first tensor, invalidated if ANY of them changes."""
    t0 = tensors[0]
    key = id(t0)
    ent = _cache.get(key)
    if ent is None or ent[0]() is not t0:
        ent = (weakref.ref(t0, _drop(key)), {})
        _cache[key] = ent
    ver = tuple((t._version, t.data_ptr()) for t in tensors)
    hit = ent[1].get(tag)
    if hit is not None and hit[0] == ver:
        return hit[1]
    v = make(*tensors)
    ent[1][tag] = (ver, v)
    return v


def set_solo_launch(on):
    """Launch-fill policy of the library (include/kinet_gemm.h kinet_set_solo_launch): True when
    the caller keeps ONE batch in flight (latency mode: partial-round shapes run smaller tiles
    that fill the chip alone), False (default) when several streams overlap.  Outputs are the
    same bit for bit either way.  Returns the previous policy."""
    return bool(N.lib().kinet_set_solo_launch(1 if on else 0))


def param_rows(p, start, end):
    """A stable (cached) row-slice view of a parameter, so its dtype cast is cached too."""
    return cached(p, ('rows', start, end), lambda t: t.detach()[start:end])


def param_matrix(p):
    """Conv 1x1 weight (O, I, 1, 1) viewed as a (O, I) GEMM operand (stable object)."""
    return cached(p, 'matrix', lambda t: t.detach().reshape(t.shape[0], -1))


def weight_as(w, dtype):
    return cached(w, ('w', dtype), lambda t: t.detach().to(dtype).contiguous())


def f32(t):
    return None if t is None else cached(t, 'f32', lambda x: x.detach().float().contiguous())


# ----------------------------------------------------------------------------------- GEMM
def _tile(M, N, ln=False, split=False):
    """The gemm_kernel tile launch() in csrc/gemm.hip picks (bm, bn)."""
    if ln:
        return (32 if M <= 8192 else 64), (256 if N <= 256 else 320)
    if split and M <= 4096:
        return 64, 64
    if M <= 4096 and N <= 1024:
        return 32, 64
    if N >= 512 and ((M + 127) // 128) * ((N + 127) // 128) >= 2048:
        return 128, 128
    return (128, 64) if N <= 64 else (64, 128)


def ksplit_for(M, N, K, ln=False):
    """Split-K factor for long-K problems with too few output tiles to fill the CUs twice
    over (the tile choice mirrors launch() in csrc/gemm.hip); 1 = no split."""
    if K < 1024 or M == 0:
        return 1
    bm, bn = _tile(M, N, ln)
    if ((M + bm - 1) // bm) * ((N + bn - 1) // bn) >= 512:
        return 1
    bm, bn = _tile(M, N, ln, split=True)
    tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
    ks = min(4, -(-768 // tiles), K // 256)
    return ks if ks >= 2 else 1


KINET_F32_X3 = 4   # include/kinet_common.h


def mm_code(dt):
    """Input dtype code of a GEMM / convolution: f32 operands follow
    torch.get_float32_matmul_precision() -- 'highest' (torch's default): exact f32 MFMA;
    'high' / 'medium': three bf16 MFMA passes per product (KINET_F32_X3, ~2^-17 relative
    error per product; torch's own 'high' mode is this same bf16x3 split or TF32)."""
    if dt == torch.float32 and torch.get_float32_matmul_precision() != 'highest':
        return KINET_F32_X3
    return N.dtype_code(dt)


def linear(x, weight, bias=None, relu=False, residual=None, row_mask=None, out_dtype=None,
           scale=None, out=None, x_add=None, ln=None):
    """y = LN?(relu?((x [+ x_add]) @ W^T * scale + bias + residual)); rows with row_mask -> 0.
    x (..., K) in bf16/f16/f32; weight (Nout, K) any float dtype (cast+cached);
    ln = (gamma, beta, eps) fuses the post-norm LayerNorm over each output row."""
    N.require_gpu(x)
    K = x.shape[-1]
    lead = x.shape[:-1]
    if x_add is not None and x_add.dim() == x.dim() and x_add.shape != x.shape:
        x_add = x_add.expand(x.shape)   # a frame-shared operand (forward_flat's unpadded pos)
    x2 = x.reshape(-1, K)
    kp = (-K) % 8
    if kp:
        # the GEMM's K must be 8-aligned (16-byte K chunks): zero-pad the inputs (KineT's
        # 4 / 1 / 20 / 5 input features); the padded weight copy is cached
        x2 = torch.nn.functional.pad(x2, (0, kp))
        if x_add is not None:
            x_add = torch.nn.functional.pad(x_add.reshape(-1, K), (0, kp))
        K += kp
    elif x2.stride(-1) != 1 or (x2.stride(0) % 8) or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    a2 = None
    if x_add is not None:
        a2 = x_add.reshape(-1, K)
        if a2.stride() != x2.stride() or a2.data_ptr() % 16:
            x2, a2 = x2.contiguous(), a2.contiguous()
            if a2.stride() != x2.stride():
                raise RuntimeError('linear: x_add must match x layout')
    M = x2.shape[0]
    if kp:
        w = cached(weight, ('w_padk', x.dtype, kp),
                   lambda t: torch.nn.functional.pad(t.detach().to(x.dtype), (0, kp)).contiguous())
    else:
        w = weight_as(weight, x.dtype)
    Nout = w.shape[0]
    odt = out_dtype or x.dtype
    if out is None:
        out = torch.empty((M, Nout), dtype=odt, device=x.device)
        ldc = Nout
    else:
        ldc = out.stride(0)
    r = None
    ldr = 0
    if residual is not None:
        r = residual.reshape(-1, Nout)
        if r.stride(-1) != 1:
            r = r.contiguous()
        if r.dtype != odt:
            r = r.to(odt)
        ldr = r.stride(0)
    mask = None
    if row_mask is not None:
        mask = row_mask.reshape(-1).to(torch.uint8).contiguous()
    e = x.element_size()
    g, b, eps = (f32(ln[0]), f32(ln[1]), float(ln[2])) if ln is not None else (None, None, 0.0)
    work = {'family': 'gemm', 'flops': 2.0 * M * Nout * K, 'shape': (M, Nout, K),
            'bytes': (M * K + Nout * K) * e + M * Nout * out.element_size() * (2 if r is not None else 1)}
    ks = ksplit_for(M, Nout, K, ln is not None) if a2 is None else 1
    if ks > 1:
        ws = torch.empty(ks * M * Nout, dtype=torch.float32, device=x.device)
        N.call('kinet_gemm_splitk', N.ptr(x2), N.ptr(w), N.ptr(out), M, Nout, K, x2.stride(0), K, ldc,
               mm_code(x.dtype), N.ptr(f32(scale)), N.ptr(f32(bias)), N.ptr(r), ldr, int(relu),
               N.ptr(g), N.ptr(b), eps, N.dtype_code(odt), N.ptr(mask), N.ptr(ws), ks, N.stream(x.device),
               work=work)
        return out.view(*lead, Nout) if out.is_contiguous() else out
    N.call('kinet_gemm_ex', N.ptr(x2), N.ptr(a2), N.ptr(w), N.ptr(out), M, Nout, K, x2.stride(0), K, ldc,
           mm_code(x.dtype), N.ptr(f32(scale)), N.ptr(f32(bias)), N.ptr(r), ldr, int(relu),
           N.ptr(g), N.ptr(b), eps, N.dtype_code(odt), N.ptr(mask), N.stream(x.device), work=work)
    return out.view(*lead, Nout) if out.is_contiguous() else out


def ffn_supported(x, linear1, linear2):
    """The fused FFN kernel covers the 16-bit compute modes at d_model 256 / 288."""
    D = x.shape[-1]
    F_ = linear1.weight.shape[0]
    return (x.dtype in (torch.bfloat16, torch.float16) and D in (256, 288) and F_ % 32 == 0
            and linear1.bias is not None and linear2.bias is not None)


def ffn_pack(w1, w2, dtype):
    """kinet_ffn_pack of (W1 (F, D), W2 (D, F)), cached per parameter version."""
    def make(a, b):
        F_, D = a.shape
        a16 = a.detach().to(dtype).contiguous()
        b16 = b.detach().to(dtype).contiguous()
        out = torch.empty(2 * D * F_, dtype=dtype, device=a.device)
        N.call('kinet_ffn_pack', N.ptr(a16), N.ptr(b16), N.ptr(out), D, F_, N.dtype_code(dtype), N.stream(a.device))
        return out
    return cached_multi([w1, w2], ('ffn_pack', dtype), make)


def ffn_fused(x, linear1, linear2, norm=None, out=None):
    """y = norm(x + linear2(relu(linear1(x)))) in one launch (deformable_transformer.py:284-288,
    :361-365); the (M, F) hidden tensor stays on chip.  x (..., D) bf16/f16."""
    N.require_gpu(x)
    D = x.shape[-1]
    F_ = linear1.weight.shape[0]
    x2 = x.reshape(-1, D)
    if x2.stride(-1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    M = x2.shape[0]
    wp = ffn_pack(linear1.weight, linear2.weight, x.dtype)
    if out is None:
        out = torch.empty((M, D), dtype=x.dtype, device=x.device)
    elif out.dtype != x.dtype or out.stride(-1) != 1 or out.numel() != M * D:
        raise RuntimeError('ffn_fused: out must be a unit-stride (M, D) tensor of the input dtype')
    g, b, eps = (f32(norm.weight), f32(norm.bias), float(norm.eps)) if norm is not None else (None, None, 0.0)
    e = x.element_size()
    work = {'family': 'gemm', 'flops': 4.0 * M * D * F_, 'shape': ('ffn', M, D, F_),
            'bytes': (2 * M * D + 2 * D * F_) * e}
    N.call('kinet_ffn_fused', N.ptr(x2), x2.stride(0), N.ptr(wp), N.ptr(f32(linear1.bias)), N.ptr(f32(linear2.bias)),
           N.ptr(g), N.ptr(b), eps, N.ptr(out), D, M, D, F_, N.dtype_code(x.dtype), N.stream(x.device), work=work)
    return out.view(*x.shape[:-1], D)


def value_proj_headmajor(x, weight, bias, head_dim, row_mask=None, out_dtype=None):
    """MSDA value projection written head-major: x (B, S, K) -> (Nout/head_dim, B, S, head_dim),
    padding rows zeroed (ms_deform_attn.py:64-67).  out_dtype: x.dtype, or float16 from bf16
    operands (the sampling kernel's mixed f16 x f32 FMA path)."""
    N.require_gpu(x)
    B, S, K = x.shape
    x2 = x.reshape(B * S, K)
    if x2.stride(-1) != 1 or (x2.stride(0) % 8) or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    w = weight_as(weight, x.dtype)
    Nout = w.shape[0]
    od = out_dtype or x.dtype
    out = torch.empty((Nout // head_dim, B, S, head_dim), dtype=od, device=x.device)
    mask = row_mask.reshape(-1).to(torch.uint8).contiguous() if row_mask is not None else None
    e = x.element_size()
    N.call('kinet_gemm_headmajor', N.ptr(x2), N.ptr(w), N.ptr(out), B * S, Nout, K, x2.stride(0), K,
           N.dtype_code(x.dtype), N.dtype_code(od), N.ptr(f32(bias)), N.ptr(mask), S, head_dim, N.stream(x.device),
           work={'family': 'gemm', 'flops': 2.0 * B * S * Nout * K, 'shape': (B * S, Nout, K),
                 'bytes': (B * S * K + Nout * K + B * S * Nout) * e})
    return out


class SplitValue:
    """A head_dim-36 MSDA value in the two head-major planes of kinet_gemm_headmajor_split:
    main (M, B, S, 32) and tail (M, B, S, 4), views of one buffer."""
    __slots__ = ('main', 'tail')

    def __init__(self, main, tail):
        self.main, self.tail = main, tail

    @property
    def shape(self):
        M_, B, S, _ = self.main.shape
        return (M_, B, S, 36)

    @property
    def dtype(self):
        return self.main.dtype

    @property
    def device(self):
        return self.main.device

    def dim(self):
        return 4

    def merged(self):
        """(M, B, S, 36) head-major copy (tests / the generic kernel)."""
        return torch.cat([self.main, self.tail], -1)


def split_value_weights(weight, bias, heads):
    """value_proj rows reordered [every head's channels 0-31 | every head's channels 32-35] (the
    split GEMM's column order), cached per parameter version."""
    D = weight.shape[0] // heads

    def perm(t):
        t = t.detach().view(heads, D, *t.shape[1:])
        return torch.cat([t[:, :32].reshape(heads * 32, *t.shape[2:]), t[:, 32:].reshape(heads * (D - 32), *t.shape[2:])],
                         0).contiguous()
    return cached(weight, 'split_w', perm), cached(bias, 'split_b', lambda b: perm(b).float().contiguous())


def value_proj_headmajor_split(x, weight_split, bias_split, heads, row_mask=None, out_dtype=None):
    """MSDA value projection of a head_dim-36 layer into the two planes the split encoder
    kernel reads (kinet_gemm_headmajor_split): x (B, S, K), weight/bias from split_value_weights
    -> SplitValue(main (heads, B, S, 32), tail (heads, B, S, 4)); padding rows zeroed
    (ms_deform_attn.py:64-67)."""
    N.require_gpu(x)
    B, S, K = x.shape
    x2 = x.reshape(B * S, K)
    if x2.stride(-1) != 1 or (x2.stride(0) % 8) or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    w = weight_as(weight_split, x.dtype)
    Nout = w.shape[0]
    od = out_dtype or x.dtype
    buf = torch.empty(B * S * Nout, dtype=od, device=x.device)
    main = buf[:heads * B * S * 32].view(heads, B, S, 32)
    tail = buf[heads * B * S * 32:].view(heads, B, S, Nout // heads - 32)
    mask = row_mask.reshape(-1).to(torch.uint8).contiguous() if row_mask is not None else None
    e = x.element_size()
    N.call('kinet_gemm_headmajor_split', N.ptr(x2), N.ptr(w), N.ptr(buf), B * S, Nout, K, x2.stride(0), K,
           N.dtype_code(x.dtype), N.dtype_code(od), N.ptr(f32(bias_split)), N.ptr(mask), S, 32, heads * 32,
           Nout // heads - 32, N.stream(x.device),
           work={'family': 'gemm', 'flops': 2.0 * B * S * Nout * K, 'shape': (B * S, Nout, K),
                 'bytes': (B * S * K + Nout * K + B * S * Nout) * e})
    return SplitValue(main, tail)


# ----------------------------------------------------------------------------------- conv
def pack_conv_weight(w, dtype, cin_pad=None):
    """OIHW -> OHWI (Cin fastest), optional zero channel padding, cast."""
    def make(t):
        o, i, kh, kw = t.shape
        p = t.detach().permute(0, 2, 3, 1)
        if cin_pad and cin_pad > i:
            p = torch.nn.functional.pad(p, (0, cin_pad - i))
        return p.to(dtype).contiguous()
    return cached(w, ('conv', dtype, cin_pad), make)


def pack_stem_weight(w, dtype, cg):
    """OIHW (Cout, 3, KH, KW) -> (Cout, KH, 1, cg) with w'[o][kh][0][kw*3 + c] = w[o][c][kh][kw]:
    the weights of the tap-folded stem convolution over pack_image_kwfold's layout."""
    def make(t):
        o, i, kh, kw = t.shape
        p = t.detach().permute(0, 2, 3, 1).reshape(o, kh, 1, kw * i)
        p = torch.nn.functional.pad(p, (0, cg - kw * i))
        return p.to(dtype).contiguous()
    return cached(w, ('stem', dtype, cg), make)


def conv2d_nhwc(x, w_packed, stride, pad, scale=None, bias=None, relu=False, residual=None, out=None, ksplit=None):
    """x (B, H, W, Cin) NHWC contiguous; w_packed (Cout, KH, KW, Cin); returns (B, Ho, Wo, Cout).
    stride / pad: int or (vertical, horizontal)."""
    B, H, W, Cin = x.shape
    Cout, KH, KW, Cin2 = w_packed.shape
    if Cin2 != Cin:
        raise RuntimeError(f'conv2d: weight Cin {Cin2} != input Cin {Cin}')
    sh, sw = (stride, stride) if isinstance(stride, int) else stride
    ph, pw = (pad, pad) if isinstance(pad, int) else pad
    Ho = (H + 2 * ph - KH) // sh + 1
    Wo = (W + 2 * pw - KW) // sw + 1
    if out is None:
        out = torch.empty((B, Ho, Wo, Cout), dtype=x.dtype, device=x.device)
    ldy = out.stride(2) if out.dim() == 4 else out.stride(-2)
    r = None
    if residual is not None:
        r = residual
    e = x.element_size()
    work = {'family': 'conv', 'flops': 2.0 * B * Ho * Wo * Cout * KH * KW * Cin,
            'shape': (B, H, W, Cin, Cout, KH, sh),
            'bytes': (B * H * W * Cin + Cout * KH * KW * Cin + B * Ho * Wo * Cout * (2 if r is not None else 1)) * e}
    tail = (mm_code(x.dtype), N.ptr(scale), N.ptr(bias), N.ptr(r), Cout if r is not None else 0, int(relu), ldy)
    if sh != sw or ph != pw:
        if ksplit not in (None, 1):
            raise RuntimeError('conv2d: split-K needs equal strides / pads')
        N.call('kinet_conv2d_ex', N.ptr(x), N.ptr(w_packed), N.ptr(out), B, H, W, Cin, Ho, Wo, Cout, KH, KW,
               sh, sw, ph, pw, *tail, N.stream(x.device), work=work)
        return out
    args = (N.ptr(x), N.ptr(w_packed), N.ptr(out), B, H, W, Cin, Ho, Wo, Cout, KH, KW, sh, ph) + tail
    ks = ksplit_for(B * Ho * Wo, Cout, KH * KW * Cin) if ksplit is None else ksplit
    if ks > 1:
        ws = torch.empty(ks * B * Ho * Wo * Cout, dtype=torch.float32, device=x.device)
        N.call('kinet_conv2d_splitk', *args, N.ptr(ws), ks, N.stream(x.device), work=work)
    else:
        N.call('kinet_conv2d', *args, N.stream(x.device), work=work)
    return out


def stem_conv_image(img, w_packed, scale, bias, dtype):
    """ResNet stem (7x7/2 conv + folded BN + ReLU) straight from the f32 NCHW image
    (kinet_stem_conv_image): (B, 3, H, W) -> (B, (H-1)//2+1, (W-1)//2+1, 64) NHWC in dtype.
    w_packed: pack_stem_weight(conv1.weight, dtype, 24)."""
    img = img.float().contiguous()
    N.require_gpu(img)
    B, C, H, W = img.shape
    if C != 3:
        raise RuntimeError('stem_conv_image expects 3-channel images')
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = torch.empty((B, Ho, Wo, 64), dtype=dtype, device=img.device)
    work = {'family': 'conv', 'flops': 2.0 * B * Ho * Wo * 64 * 147, 'shape': ('stem', B, H, W),
            'bytes': B * 3 * H * W * 4 + B * Ho * Wo * 64 * y.element_size()}
    N.call('kinet_stem_conv_image', N.ptr(img), N.ptr(w_packed), N.ptr(f32(scale)), N.ptr(f32(bias)), N.ptr(y),
           B, H, W, N.dtype_code(dtype), N.stream(img.device), work=work)
    return y


def bottleneck_pack(w3, w1, s3, s1, dtype):
    """kinet_bottleneck_pack of conv3 (F, D, 1, 1) and the next block's conv1 (DB, F, 1, 1) with
    their FrozenBN scales folded in, cached per parameter version."""
    def make(a, b, sa, sb):
        F_, D, DB = a.shape[0], a.shape[1], b.shape[0]
        a32 = a.detach().reshape(F_, D).float().contiguous()
        b32 = b.detach().reshape(DB, F_).float().contiguous()
        out = torch.empty((D + DB) * F_, dtype=dtype, device=a.device)
        N.call('kinet_bottleneck_pack', N.ptr(a32), N.ptr(b32), N.ptr(f32(sa)), N.ptr(f32(sb)), N.ptr(out), D, F_, DB,
               N.dtype_code(dtype), N.stream(a.device))
        return out
    return cached_multi([w3, w1, s3, s1], ('bneck_pack', dtype), make)


def bottleneck_pair_supported(dtype, w3, w1):
    """The fused pair covers 16-bit NHWC rows with D = planes in {64, 128, 256}, F = 4 D (conv3
    weight (F, D, 1, 1)) and the next conv1 (DB, F, 1, 1) with DB = D, or DB = 128 at D = 64."""
    F_, D, DB = w3.shape[0], w3.shape[1], w1.shape[0]
    return (dtype in (torch.bfloat16, torch.float16) and D in (64, 128, 256) and F_ == 4 * D
            and (DB == D or (D == 64 and DB == 128))
            and tuple(w3.shape) == (F_, D, 1, 1) and tuple(w1.shape) == (DB, F_, 1, 1))


def bottleneck_pair(x, residual, packed, b3, b1):
    """ResNet bottleneck pair (kinet_bottleneck_pair): x = block i's conv2 output (B, H, W, D)
    NHWC, residual (B, H, W, F) -> (y, t): y = relu(conv3(x) * s3 + b3 + residual) (the block
    output, F = 4 D channels), t = relu(conv1'(y) * s1 + b1) (the next block's conv1 output,
    DB = b1.numel() channels); the BN scales are in `packed` (bottleneck_pack)."""
    N.require_gpu(x)
    B, H, W, D = x.shape
    F_ = 4 * D
    if residual.shape != (B, H, W, F_) or not residual.is_contiguous() or residual.dtype != x.dtype:
        raise RuntimeError('bottleneck_pair: residual must be a contiguous (B, H, W, 4D) tensor of the input dtype')
    M = B * H * W
    DB = b1.numel()
    y = torch.empty((B, H, W, F_), dtype=x.dtype, device=x.device)
    t = torch.empty((B, H, W, DB), dtype=x.dtype, device=x.device)
    e = x.element_size()
    work = {'family': 'conv', 'flops': 2.0 * M * F_ * (D + DB), 'shape': ('bneck', M, D, F_, DB),
            'bytes': (M * D + 2 * M * F_ + M * DB + (D + DB) * F_) * e}
    N.call('kinet_bottleneck_pair', N.ptr(x), D, N.ptr(residual), N.ptr(packed), N.ptr(f32(b3)), N.ptr(f32(b1)),
           N.ptr(y), N.ptr(t), M, D, F_, DB, N.dtype_code(x.dtype), N.stream(x.device), work=work)
    return y, t


def maxpool_3x3s2(x):
    B, H, W, C = x.shape
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = torch.empty((B, Ho, Wo, C), dtype=x.dtype, device=x.device)
    N.call('kinet_maxpool2d_3x3s2', N.ptr(x), N.ptr(y), B, H, W, C, N.dtype_code(x.dtype), N.stream(x.device))
    return y


def pack_image(img, dtype, cpad=8):
    """(B, 3, H, W) f32 NCHW -> (B, H, W, cpad) NHWC dtype."""
    img = img.float().contiguous()
    B, C, H, W = img.shape
    if C != 3:
        raise RuntimeError('pack_image expects 3-channel images')
    y = torch.empty((B, H, W, cpad), dtype=dtype, device=img.device)
    N.call('kinet_pack_image_nhwc', N.ptr(img), N.ptr(y), B, H, W, cpad, N.dtype_code(dtype), N.stream(img.device))
    return y


def pack_image_kwfold(img, dtype, kw, stride, pad, cg):
    """(B, 3, H, W) f32 NCHW -> (B, H, Wo, cg) with the kw horizontal taps of a stride-`stride`
    filter folded into channels (kinet_pack_image_kwfold)."""
    img = img.float().contiguous()
    B, C, H, W = img.shape
    if C != 3:
        raise RuntimeError('pack_image_kwfold expects 3-channel images')
    Wo = (W + 2 * pad - kw) // stride + 1
    y = torch.empty((B, H, Wo, cg), dtype=dtype, device=img.device)
    N.call('kinet_pack_image_kwfold', N.ptr(img), N.ptr(y), B, H, W, kw, stride, pad, cg, N.dtype_code(dtype),
           N.stream(img.device), work={'family': 'kinet_pack_image_kwfold'})
    return y


# ------------------------------------------------------------------------------ norms
def layernorm(x, weight, bias, eps=1e-5, residual=None, out=None):
    d = x.shape[-1]
    x2 = x.contiguous()
    r = residual.contiguous() if residual is not None else None
    y = out if out is not None else torch.empty_like(x2)
    rows = x2.numel() // d
    N.call('kinet_layernorm', N.ptr(x2), N.ptr(r), N.ptr(f32(weight)), N.ptr(f32(bias)), N.ptr(y), rows, d,
           float(eps), N.dtype_code(x.dtype), 0, N.stream(x.device),
           work={'family': 'norm', 'bytes': rows * d * x2.element_size() * (3 if r is not None else 2)})
    return y


def groupnorm_nhwc(x, weight, bias, groups, eps=1e-5, out=None, out_batch_stride=None):
    """x (B, HW, C) contiguous -> out rows at out + b*out_batch_stride (default packed)."""
    B, HW, C = x.shape
    if out is None:
        out = torch.empty_like(x)
        out_batch_stride = HW * C
    nws = N.lib().kinet_groupnorm_workspace(B, HW, C, groups, N.dtype_code(x.dtype))
    stats = torch.empty(max(1, nws), dtype=torch.float32, device=x.device)
    N.call('kinet_groupnorm', N.ptr(x), N.ptr(f32(weight)), N.ptr(f32(bias)), N.ptr(out), B, HW, C, groups,
           int(out_batch_stride), float(eps), N.dtype_code(x.dtype), N.ptr(stats), N.stream(x.device),
           work={'family': 'norm', 'bytes': 2 * x.numel() * x.element_size()})
    return out


def add(a, b, out=None):
    a = a.contiguous()
    b = b.contiguous()
    y = out if out is not None else torch.empty_like(a)
    N.call('kinet_add', N.ptr(a), N.ptr(b), N.ptr(y), a.numel(), N.dtype_code(a.dtype), N.stream(a.device),
           work={'family': 'eltwise', 'bytes': 3 * a.numel() * a.element_size()})
    return y


# ---------------------------------------------------------------- position embedding
def sine_position_embed(mask, dim_t, num_pos_feats, three_d=False, frame=0, frames=1, normalize=True, scale=1.0,
                        level_embed=None, out=None, out_batch_stride=None, out_dtype=torch.float32):
    """Sine embedding of a padding mask (B, H, W) as NHWC rows (kinet_sine_position_embed):
    returns (B, H*W, C) (or writes rows into `out` at out + b*out_batch_stride)."""
    N.require_gpu(mask)
    B, H, W = mask.shape
    C = (3 if three_d else 2) * num_pos_feats
    if out is None:
        out = torch.empty((B, H * W, C), dtype=out_dtype, device=mask.device)
        out_batch_stride = H * W * C
    m = mask.to(torch.uint8).contiguous()
    N.call('kinet_sine_position_embed', N.ptr(m), N.ptr(dim_t), N.ptr(f32(level_embed) if level_embed is not None
                                                                          else None),
           N.ptr(out), B, H, W, num_pos_feats, int(three_d), frame, frames, int(normalize), float(scale),
           int(out_batch_stride), N.dtype_code(out.dtype), N.stream(mask.device),
           work={'family': 'pos_embed', 'bytes': B * H * W * C * out.element_size()})
    return out


def nms(boxes, scores, iou_threshold):
    """torchvision.ops.nms semantics on the GPU: indices of the kept boxes, by descending score
    (ties by index).  boxes (n, 4) xyxy, scores (n)."""
    N.require_gpu(boxes, scores)
    n = boxes.shape[0]
    keep = torch.zeros(n, dtype=torch.uint8, device=boxes.device)
    if n:
        b = boxes.float().contiguous()
        s = scores.float().contiguous()
        N.call('kinet_nms', N.ptr(b), N.ptr(s), N.ptr(keep), n, float(iou_threshold), N.stream(boxes.device))
        idx = keep.nonzero().flatten()
        # descending, ties by index, NaN first: the kernel's own rank order
        return idx[torch.sort(s[idx], descending=True, stable=True)[1]]
    return keep.nonzero().flatten()


# --------------------------------------------------------------------------- attention
_SEED_POOL = {}     # device index -> [seeds tensor, next index, generator state key after the draw]
_SEED_BLOCK = 64


def _gen_key(gen):
    return (gen.initial_seed(), gen.get_offset())


def dropout_seed(device):
    """A device int64 seed for the dropout kernels, drawn from torch's generator of `device`
    (as F.dropout draws its Philox offset from it), without a host sync.  Seeds are drawn 64 at
    a time (one launch instead of one per dropout site); the block is redrawn whenever the
    generator has moved since the draw (torch.manual_seed, other random ops), so a reseeded
    run replays the same seeds."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    gen = torch.cuda.default_generators[idx]
    ent = _SEED_POOL.get(idx)
    if ent is None or ent[1] >= _SEED_BLOCK or ent[2] != _gen_key(gen):
        seeds = torch.randint(0, 2 ** 62, (_SEED_BLOCK,), dtype=torch.int64, device=torch.device('cuda', idx))
        ent = _SEED_POOL[idx] = [seeds, 0, _gen_key(gen)]
    s = ent[0][ent[1]:ent[1] + 1]
    ent[1] += 1
    return s


def dropout_mask(seed, n, p):
    """The keep mask (uint8, n elements) the dropout kernels derive from `seed` at probability p."""
    keep = torch.empty(n, dtype=torch.uint8, device=seed.device)
    N.call('kinet_dropout_mask', N.ptr(seed), n, float(p), N.ptr(keep), N.stream(seed.device))
    return keep


def mha_core(q, k, v, heads, scale, key_mask=None, out=None, dropout_p=0.0, seed=None):
    """q (B, Lq, E) (row stride may exceed E), k/v (B, Lk, E) -> (B, Lq, E).  dropout_p > 0:
    attention-probability dropout with the keep mask of `seed` (kinet_mha_core_dropout)."""
    B, Lq, E = q.shape
    Lk = k.shape[1]
    D = E // heads
    for t in (q, k, v):
        if t.stride(-1) != 1 or t.stride(0) != t.shape[1] * t.stride(1):
            raise RuntimeError('mha_core: rows must be unit-stride with packed batches')
    o = out if out is not None else torch.empty((B, Lq, E), dtype=q.dtype, device=q.device)
    km = key_mask.to(torch.uint8).contiguous() if key_mask is not None else None
    if dropout_p > 0:
        N.call('kinet_mha_core_dropout', N.ptr(q), q.stride(1), N.ptr(k), k.stride(1), N.ptr(v), v.stride(1),
               N.ptr(o), o.stride(1), B, Lq, Lk, heads, D, float(scale), N.dtype_code(q.dtype), N.ptr(km),
               float(dropout_p), N.ptr(seed), N.stream(q.device),
               work={'family': 'attn', 'flops': 4.0 * B * heads * Lq * Lk * D})
        return o
    N.call('kinet_mha_core', N.ptr(q), q.stride(1), N.ptr(k), k.stride(1), N.ptr(v), v.stride(1), N.ptr(o),
           o.stride(1), B, Lq, Lk, heads, D, float(scale), N.dtype_code(q.dtype), N.ptr(km), N.stream(q.device),
           work={'family': 'attn', 'flops': 4.0 * B * heads * Lq * Lk * D})
    return o


def box_refine(tmp, ref, valid_ratios=None, want_input=True, out=None):
    """tmp (B, Q, 4) f32, ref (B, Q, 2|4) f32 -> new_ref (B, Q, 4) [, ref_input (B, Q, L, 4)];
    out: optional contiguous (B, Q, 4) f32 destination of new_ref."""
    B, Q, _ = tmp.shape
    tmp = tmp.float().contiguous()
    ref = ref.float().contiguous()
    nref = out if out is not None else torch.empty((B, Q, 4), dtype=torch.float32, device=tmp.device)
    rin = None
    L = 0
    if want_input:
        vr = valid_ratios.float().contiguous()
        L = vr.shape[1]
        rin = torch.empty((B, Q, L, 4), dtype=torch.float32, device=tmp.device)
    else:
        vr = None
    N.call('kinet_box_refine', N.ptr(tmp), N.ptr(ref), ref.shape[-1], N.ptr(vr), N.ptr(nref), N.ptr(rin), B, Q, L,
           N.stream(tmp.device))
    return nref, rin


# ------------------------------------------------------------------------------ MSDA
_tile_orders = {}


def encoder_tile_order(shapes, device, qt=16):
    """Processing order of the encoder's 16-query tiles for msda_fused: sorted by the
    normalised image row of each tile's first query, so the tiles of all levels that sample
    the same image band run together and share the value rows in L2 (the natural order
    sweeps the image once per level).  Cached per (shapes, device)."""
    key = (tuple(tuple(int(v) for v in s) for s in shapes), str(device), qt)
    o = _tile_orders.get(key)
    if o is None:
        import numpy as np
        hw = np.array([h * w for h, w in key[0]], dtype=np.int64)
        starts = np.concatenate([[0], np.cumsum(hw)[:-1]])
        lq = int(hw.sum())
        q = np.arange((lq + qt - 1) // qt, dtype=np.int64) * qt
        lvl = np.searchsorted(starts, q, side='right') - 1
        H = np.array([h for h, _ in key[0]], dtype=np.float64)[lvl]
        W = np.array([w for _, w in key[0]], dtype=np.int64)[lvl]
        y = ((q - starts[lvl]) // W + 0.5) / H
        o = torch.as_tensor(np.argsort(y, kind='stable').astype(np.int32), device=device)
        _tile_orders[key] = o
    return o


_host_shapes = {}
_enc_plans = {}
# template-argument spelling of the element types in rocprofv3 kernel names
_KT = {torch.bfloat16: 'kinet::bf16_t', torch.float16: 'kinet::f16_t', torch.float32: 'float', torch.float64: 'double'}


def msda_encoder_set_strips(strips):
    """Strips per head map for the encoder sampler on the calling thread (0 = the plan's own
    choice; kinet_msda_encoder_set_strips, A/B tooling).  The cached plans are dropped, so
    msda_encoder_plan reports what the next launch runs.  Returns the previous value."""
    old = N.lib().kinet_msda_encoder_set_strips(int(strips))
    _enc_plans.clear()
    return old


def msda_encoder_plan(shapes, batch, n_heads, Lq, channels=32):
    """kinet_msda_encoder_plan_ex for host level shapes: (levels gathered from HBM, strips per head
    map, LDS map pixels used, workgroups), or None when no strip plan fits the LDS map.  Cached."""
    key = (tuple(tuple(int(v) for v in s) for s in shapes), int(batch), int(n_heads), int(Lq), int(channels))
    if key not in _enc_plans:
        import ctypes
        hs = (ctypes.c_int64 * 8)(*[v for s in key[0] for v in s])
        out = (ctypes.c_int32 * 4)()
        rc = N.lib().kinet_msda_encoder_plan_ex(ctypes.cast(hs, ctypes.c_void_p), key[1], key[2], key[3], key[4],
                                                ctypes.cast(out, ctypes.c_void_p))
        _enc_plans[key] = tuple(out) if rc == 0 else None
    return _enc_plans[key]


# head_dim-36 encoder calls through the split value planes + kinet_msda_encoder_forward_split
# when eligible; False keeps the generic fused kernel on the (M, B, S, 36) value (A/B and tests)
MSDA_SPLIT = [True]


def msda_split_supported(dtype, head_dim, shapes, Lq, n_heads, n_levels, n_points, batch):
    """True when a head_dim-36 encoder call runs on the strip kernel with the split value planes:
    16-bit compute, 4 levels x 4 points, >= 2048 queries per frame, a strip plan for 72-byte
    pixels and a tail plane below 2^28 bytes."""
    if not MSDA_SPLIT[0] or dtype not in (torch.bfloat16, torch.float16) or head_dim != 36:
        return False
    if n_levels != 4 or n_points != 4 or Lq < 2048 or shapes is None or len(shapes) != 4:
        return False
    S = sum(int(h) * int(w) for h, w in shapes)
    if batch * Lq >= (1 << 24) or S * 8 >= (1 << 28):
        return False
    return msda_encoder_plan(shapes, batch, n_heads, Lq, 36) is not None


def msda_encoder_split(value, shapes, offlog_hm, reference_points, n_heads, query_attn_mask=None, out_dtype=None,
                       query_tile_order=None):
    """Head_dim-36 encoder sampling (kinet_msda_encoder_forward_split): value a SplitValue from
    value_proj_headmajor_split, offlog_hm (M, B, Lq, 48) f16, reference_points (B, Lq, 4, 2|4) f32
    -> (B, Lq, M*36)."""
    main, tail = value.main, value.tail
    M_, B, S, _ = main.shape
    D = 36
    Lq = offlog_hm.shape[2]
    key = tuple(tuple(int(v) for v in s) for s in shapes)
    hs = _host_shapes.get(key)
    if hs is None:
        hs = _host_shapes[key] = torch.tensor(key, dtype=torch.int64)
    ref = reference_points.float().contiguous()
    od = out_dtype or torch.bfloat16
    out = torch.empty((B, Lq, M_ * D), dtype=od, device=main.device)
    qm = query_attn_mask.to(torch.uint8).contiguous() if query_attn_mask is not None else None
    if query_tile_order is not None and (query_tile_order.dtype != torch.int32 or
                                         query_tile_order.numel() != (Lq + 15) // 16):
        raise RuntimeError('msda_encoder_split: query_tile_order must be int32 with ceil(Lq/16) entries')
    offlog_hm = offlog_hm.contiguous()
    nsamp = B * Lq * M_ * 16
    plan = msda_encoder_plan(key, B, M_, Lq, 36)
    kname = 'msda_enc_kernel<%s, %d, %d, %s, false, true, 12>' % (_KT[od], plan[0] if plan else -1, ref.shape[-1],
                                                                  'true' if qm is not None else 'false')
    N.call('kinet_msda_encoder_forward_split', N.ptr(main), main.stride(1), main.stride(0), N.ptr(tail),
           tail.stride(1), tail.stride(0), N.ptr(hs), N.ptr(offlog_hm), N.ptr(ref), ref.shape[-1], N.ptr(qm),
           N.ptr(out), B, S, M_, D, 4, Lq, 4, N.dtype_code(od), N.ptr(query_tile_order), N.stream(main.device),
           work={'family': 'msda', 'flops': 10.0 * nsamp * D, 'Lq': Lq, 'S': S, 'kernel': kname,
                 # compulsory bytes: both value planes once, f16 offsets + logits, refs, output once
                 'bytes': B * S * M_ * D * 2 + offlog_hm.numel() * 2 + ref.numel() * 4
                 + out.numel() * out.element_size()})
    return out


def msda_encoder_supported(value, shapes, Lq, n_heads, n_levels, n_points, batch):
    """True when kinet_msda_encoder_forward takes the call: f16 head-major values of head_dim
    32, 4 levels x 4 points, an encoder-sized query set (>= 2048 per frame) and a strip plan
    that fits the LDS map (kinet_msda_encoder_plan)."""
    if value.dim() != 4 or value.dtype != torch.float16 or value.shape[-1] != 32 or value.stride(2) != 32:
        return False
    if n_levels != 4 or n_points != 4 or Lq < 2048 or shapes is None or len(shapes) != 4:
        return False
    if batch * Lq >= (1 << 24) or msda_encoder_plan(shapes, batch, n_heads, Lq) is None:
        return False
    return value.data_ptr() % 16 == 0 and value.stride(1) % 8 == 0 and value.stride(0) % 8 == 0


def _load_add_operand(x2, x_add, B, Lq, K):
    """(x2, a2, a2_rows) for a GEMM over x2 = x.reshape(B*Lq, K) rows with x_add added at load:
    an x_add of ONE frame (1, Lq, K) for a batch of B > 1 frames stays one frame in memory and
    every frame's rows read it (a2_rows = Lq: the unpadded batch's shared position embedding,
    deformable_transformer.py forward_flat) -- else x_add has x's rows and layout."""
    if x_add is None:
        return x2, None, 0
    if x_add.shape[0] == 1 and B > 1 and Lq >= 32:
        if x2.stride(-1) != 1 or x2.stride(0) != K or x2.data_ptr() % 16:
            x2 = x2.contiguous()
        a2 = x_add.reshape(Lq, K)
        if a2.stride() != x2.stride() or a2.data_ptr() % 16:
            a2 = a2.contiguous()
        return x2, a2, Lq
    if x_add.shape[0] != B:
        x_add = x_add.expand(B, Lq, K)
    a2 = x_add.reshape(B * Lq, K)
    if x2.stride(-1) != 1 or (x2.stride(0) % 8) or x2.data_ptr() % 16 or a2.stride() != x2.stride() or \
            a2.data_ptr() % 16:
        x2, a2 = x2.contiguous(), a2.contiguous()
    return x2, a2, 0


def offsets_proj_headmajor(x, weight, bias, heads, x_add=None, out_dtype=torch.float16):
    """The MSDA offsets + logits projection (x [+ x_add]) @ W^T + b stored head-major
    (heads, B, Lq, Nout/heads): W's rows must already be grouped per head
    (MSDeformAttn.packed_offsets_weights_headmajor)."""
    N.require_gpu(x)
    B, Lq, K = x.shape
    x2 = x.reshape(B * Lq, K)
    if x_add is None and (x2.stride(-1) != 1 or (x2.stride(0) % 8) or x2.data_ptr() % 16):
        x2 = x2.contiguous()
    x2, a2, a2_rows = _load_add_operand(x2, x_add, B, Lq, K)
    w = weight_as(weight, x.dtype)
    Nout = w.shape[0]
    rec = Nout // heads
    out = torch.empty((heads, B, Lq, rec), dtype=out_dtype, device=x.device)
    e = x.element_size()
    N.call('kinet_gemm_headmajor_ex', N.ptr(x2), N.ptr(a2), N.ptr(w), N.ptr(out), B * Lq, Nout, K, x2.stride(0), K,
           N.dtype_code(x.dtype), N.dtype_code(out_dtype), N.ptr(f32(bias)), None, Lq, rec, a2_rows,
           N.stream(x.device),
           work={'family': 'gemm', 'flops': 2.0 * B * Lq * Nout * K, 'shape': (B * Lq, Nout, K),
                 'role': 'msda_prep',
                 'bytes': (B * Lq * K + (0 if a2 is None else a2.shape[0] * K) + Nout * K) * e + B * Lq * Nout * 2})
    return out


def msda_encoder(value, shapes, offlog_hm, reference_points, n_heads, query_attn_mask=None, out_dtype=None,
                 query_tile_order=None):
    """Encoder-sized MSDeformAttn sampling (kinet_msda_encoder_forward): value (M, B, S, 32)
    f16 head-major, shapes = host list of (H, W), offlog_hm (M, B, Lq, 48) f16 from
    offsets_proj_headmajor, reference_points (B, Lq, 4, 2|4) f32 -> (B, Lq, M*32)."""
    M_, B, S, D = value.shape
    Lq = offlog_hm.shape[2]
    key = tuple(tuple(int(v) for v in s) for s in shapes)
    hs = _host_shapes.get(key)
    if hs is None:
        hs = _host_shapes[key] = torch.tensor(key, dtype=torch.int64)
    ref = reference_points.float().contiguous()
    od = out_dtype or torch.bfloat16
    out = torch.empty((B, Lq, M_ * D), dtype=od, device=value.device)
    qm = query_attn_mask.to(torch.uint8).contiguous() if query_attn_mask is not None else None
    if query_tile_order is not None and (query_tile_order.dtype != torch.int32 or
                                         query_tile_order.numel() != (Lq + 15) // 16):
        raise RuntimeError('msda_encoder: query_tile_order must be int32 with ceil(Lq/16) entries')
    offlog_hm = offlog_hm.contiguous()
    nsamp = B * Lq * M_ * 16
    plan = msda_encoder_plan(key, B, M_, Lq)
    # the instantiation kinet_msda_encoder_forward launches (as rocprofv3 names it)
    kname = 'msda_enc_kernel<%s, %d, %d, %s>' % (_KT[od], plan[0] if plan else -1, ref.shape[-1],
                                                   'true' if qm is not None else 'false')
    N.call('kinet_msda_encoder_forward', N.ptr(value), value.stride(1), value.stride(0), N.ptr(hs), N.ptr(offlog_hm),
           N.ptr(ref), ref.shape[-1], N.ptr(qm), N.ptr(out), B, S, M_, D, 4, Lq, 4, N.dtype_code(od),
           N.ptr(query_tile_order), N.stream(value.device),
           work={'family': 'msda', 'flops': 10.0 * nsamp * D, 'Lq': Lq, 'S': S, 'kernel': kname,
                 # compulsory bytes: value once, f16 offsets + logits, refs, output once
                 'bytes': B * S * M_ * D * 2 + offlog_hm.numel() * 2 + ref.numel() * 4 + out.numel() * out.element_size()})
    return out


# encoder calls sample through kinet_msda_sample_records + kinet_msda_encoder_forward_records
# (phase 1 in the projection epilogue) when eligible; False keeps the f16 offsets/logits path
# (A/B and tests)
MSDA_RECORDS = [True]


def msda_record_frac_bits(shapes):
    """Fraction bits of the records' fixed-point locations for these level shapes: the most that
    leave an integer part holding every level's H and W (at most 10), or None (< 6: too large)."""
    mx = max(max(int(h), int(w)) for h, w in shapes)
    ib = max(1, (mx - 1).bit_length())
    fb = min(10, 16 - ib)
    return fb if fb >= 6 else None


def msda_records_supported(query, shapes_host, n_heads, n_levels, n_points):
    return (MSDA_RECORDS[0] and query.dtype in (torch.bfloat16, torch.float16) and query.shape[-1] == 256
            and n_heads % 4 == 0 and n_levels == 4 and n_points == 4 and shapes_host is not None
            and len(shapes_host) == 4 and msda_record_frac_bits(shapes_host) is not None)


def msda_sample_records(x, weight, bias, heads, reference_points, shapes_host, x_add=None, query_attn_mask=None):
    """The encoder MSDA projection with softmax / locations / bilinear setup in the GEMM epilogue
    (kinet_msda_sample_records): x (B, Lq, 256) [+ x_add], W rows grouped (head, level, 12)
    (MSDeformAttn.packed_records_weights), reference_points (B, Lq, 4, 2|4) -> (records
    (heads, B, Lq, 24) int32 = 96 bytes each, frac_bits)."""
    N.require_gpu(x)
    B, Lq, K_ = x.shape
    x2 = x.reshape(B * Lq, K_)
    if x_add is None and (x2.stride(-1) != 1 or (x2.stride(0) % 8) or x2.data_ptr() % 16):
        x2 = x2.contiguous()
    x2, a2, a2_rows = _load_add_operand(x2, x_add, B, Lq, K_)
    w = weight_as(weight, x.dtype)
    key = tuple(tuple(int(v) for v in s) for s in shapes_host)
    hs = _host_shapes.get(key)
    if hs is None:
        hs = _host_shapes[key] = torch.tensor(key, dtype=torch.int64)
    fb = msda_record_frac_bits(key)
    ref = reference_points.float().contiguous()
    qm = query_attn_mask.to(torch.uint8).contiguous() if query_attn_mask is not None else None
    rec = torch.empty((heads, B, Lq, 24), dtype=torch.int32, device=x.device)
    e = x.element_size()
    N.call('kinet_msda_sample_records', N.ptr(x2), N.ptr(a2), N.ptr(w), N.ptr(f32(bias)), B * Lq, heads, K_,
           x2.stride(0), N.dtype_code(x.dtype), N.ptr(ref), ref.shape[-1], N.ptr(qm), N.ptr(hs), 4, 4, fb, N.ptr(rec),
           a2_rows, N.stream(x.device),
           work={'family': 'gemm', 'flops': 2.0 * B * Lq * heads * 48 * K_, 'shape': (B * Lq, heads * 48, K_),
                 'role': 'msda_prep',
                 'bytes': (B * Lq * K_ + (0 if a2 is None else a2.shape[0] * K_) + heads * 48 * K_) * e
                 + ref.numel() * 4 + rec.numel() * 4})
    return rec, fb


def msda_encoder_records(value, shapes, records, frac_bits, out_dtype=None, query_tile_order=None):
    """Encoder-sized MSDA sampling from sampling records (kinet_msda_encoder_forward_records):
    value (M, B, S, 32) f16 head-major, records (M, B, Lq, 24) int32 from msda_sample_records
    -> (B, Lq, M*32)."""
    M_, B, S, D = value.shape
    Lq = records.shape[2]
    key = tuple(tuple(int(v) for v in s) for s in shapes)
    hs = _host_shapes.get(key)
    if hs is None:
        hs = _host_shapes[key] = torch.tensor(key, dtype=torch.int64)
    od = out_dtype or torch.bfloat16
    out = torch.empty((B, Lq, M_ * D), dtype=od, device=value.device)
    if query_tile_order is not None and (query_tile_order.dtype != torch.int32 or
                                         query_tile_order.numel() != (Lq + 15) // 16):
        raise RuntimeError('msda_encoder_records: query_tile_order must be int32 with ceil(Lq/16) entries')
    records = records.contiguous()
    nsamp = B * Lq * M_ * 16
    plan = msda_encoder_plan(key, B, M_, Lq)
    kname = 'msda_enc_kernel<%s, %d, 2, false, true>' % (_KT[od], plan[0] if plan else -1)
    N.call('kinet_msda_encoder_forward_records', N.ptr(value), value.stride(1), value.stride(0), N.ptr(hs),
           N.ptr(records), int(frac_bits), N.ptr(out), B, S, M_, D, 4, Lq, 4, N.dtype_code(od),
           N.ptr(query_tile_order), N.stream(value.device),
           work={'family': 'msda', 'flops': 10.0 * nsamp * D, 'Lq': Lq, 'S': S, 'kernel': kname,
                 # compulsory bytes: value once, the 96-byte records, output once
                 'bytes': B * S * M_ * D * 2 + records.numel() * 4 + out.numel() * out.element_size()})
    return out


def msda_fused(value, spatial_shapes, offlog, reference_points, n_heads, n_levels, n_points,
               query_attn_mask=None, want_loc_attw=False, head_major=False, out_dtype=None,
               query_tile_order=None):
    """Sampling of MSDeformAttn.forward (ms_deform_attn.py:69-87) in one kernel.
    value: projected values, either (B, S, d) row-major (column slices allowed) or, with
    head_major=True, (M, B, S, D) as written by value_proj_headmajor;
    offlog (B, Lq, M*L*P*3) f32 (or f16 with 16-bit values) [offsets | logits];
    reference_points (B, Lq, L, 2|4) f32.
    out_dtype: value.dtype, or bfloat16 from float16 values (mixed-precision gather path).
    query_tile_order: optional int32 (ceil(Lq/16),) processing order of the 16-query tiles
    (encoder_tile_order); only the fast 16-bit D=32 kernel uses it, the generic kernel
    ignores it (the output is identical either way).
    Cached weights/geometry are built on the stream current at first use: a caller that
    runs several streams from a cold start synchronises once after the first forward.
    Returns (B, Lq, d) [, loc, attw]."""
    if head_major:
        M_, B, S, D = value.shape
        if M_ != n_heads:
            raise RuntimeError(f'head-major value has {M_} heads, module expects {n_heads}')
        d = M_ * D
        if value.stride(-1) != 1 or value.data_ptr() % 16:
            value = value.contiguous()
        vsb, vss, vsm = value.stride(1), value.stride(2), value.stride(0)
    else:
        B, S, d = value.shape
        D = d // n_heads
        if not (value.stride(-1) == 1 and value.data_ptr() % 16 == 0):
            value = value.contiguous()
        vsb, vss, vsm = value.stride(0), value.stride(1), D
    Lq = offlog.shape[1]
    offlog = offlog.contiguous()
    ref = reference_points.float().contiguous()
    if ref.shape[2] != n_levels:
        raise RuntimeError(f'reference_points has {ref.shape[2]} levels, module expects {n_levels}')
    od = out_dtype or value.dtype
    out = torch.empty((B, Lq, d), dtype=od, device=value.device)
    loc = attw = None
    if want_loc_attw:
        loc = torch.empty((B, Lq, n_heads, n_levels, n_points, 2), dtype=torch.float32, device=value.device)
        attw = torch.empty((B, Lq, n_heads, n_levels, n_points), dtype=torch.float32, device=value.device)
    qm = query_attn_mask.to(torch.uint8).contiguous() if query_attn_mask is not None else None
    if query_tile_order is not None:
        # the kernel reads torder[tile] for every 16-query tile of the grid
        t = query_tile_order
        if (t.dtype != torch.int32 or t.device != value.device or not t.is_contiguous()
                or t.numel() != (Lq + 15) // 16):
            raise RuntimeError(f'msda_fused: query_tile_order must be a contiguous int32 tensor on '
                               f'{value.device} with ceil(Lq/16) = {(Lq + 15) // 16} entries')
    if offlog.dtype not in (torch.float32, torch.float16):
        raise RuntimeError('msda_fused: the offsets/logits projection must be f32 or f16')
    ev = value.element_size()
    nsamp = B * Lq * n_heads * n_levels * n_points
    # the instantiation launch_fused (csrc/msda.hip) picks, as rocprofv3 names it
    if (ev == 2 and D == 32 and n_points == 4 and n_levels in (4, 8) and vss % 8 == 0 and vsb % 8 == 0
            and vsm % 8 == 0):
        kname = 'msda_fused_fast_kernel<%s, %s, %s, %s>' % (_KT[value.dtype], _KT[od], _KT[offlog.dtype],
                                                             '4, 4, 2, 2' if n_levels == 4 else '8, 4')
    else:
        kname = 'msda_fused_kernel<%s, *>' % _KT[value.dtype]
    N.call('kinet_msda_fused_forward', N.ptr(value), vsb, vss, vsm, N.ptr(spatial_shapes), N.ptr(offlog),
           offlog.shape[-1], N.ptr(ref), ref.shape[-1], N.ptr(qm), N.ptr(out), N.ptr(loc), N.ptr(attw), B, S,
           n_heads, D, n_levels, Lq, n_points, N.dtype_code(value.dtype), N.dtype_code(od), N.dtype_code(offlog.dtype),
           N.ptr(query_tile_order), N.stream(value.device),
           work={'family': 'msda', 'flops': 10.0 * nsamp * D,
                 # compulsory bytes: value once, f32 offsets+logits, refs, output once
                 'bytes': B * S * d * ev + nsamp * 3 * offlog.element_size() + ref.numel() * 4
                 + B * Lq * d * out.element_size()
                 + (nsamp * 3 * 4 if want_loc_attw else 0),
                 'Lq': Lq, 'S': S, 'shape': (B, Lq, S), 'kernel': kname})
    if want_loc_attw:
        return out, loc, attw
    return out


# ------------------------------------------------------------------ backward (kinet_grad.h)
def transpose2d(x):
    """(R, C) -> (C, R) contiguous (kinet_transpose)."""
    N.require_gpu(x)
    if x.stride(-1) != 1:
        x = x.contiguous()
    R, C = x.shape
    y = torch.empty((C, R), dtype=x.dtype, device=x.device)
    N.call('kinet_transpose', N.ptr(x), N.ptr(y), R, C, x.stride(0), R, N.dtype_code(x.dtype), N.stream(x.device),
           work={'family': 'grad', 'bytes': 2 * x.numel() * x.element_size()})
    return y


def im2col_nhwc(x, KH, KW, stride, pad):
    """x (B, H, W, C) -> (B*Ho*Wo, KH*KW*C) patch matrix (kinet_im2col_nhwc)."""
    B, H, W, C = x.shape
    sh, sw = (stride, stride) if isinstance(stride, int) else stride
    ph, pw = (pad, pad) if isinstance(pad, int) else pad
    Ho, Wo = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
    cols = torch.empty((B * Ho * Wo, KH * KW * C), dtype=x.dtype, device=x.device)
    N.call('kinet_im2col_nhwc', N.ptr(x.contiguous()), N.ptr(cols), B, H, W, C, Ho, Wo, KH, KW, sh, sw, ph, pw,
           N.dtype_code(x.dtype), N.stream(x.device), work={'family': 'grad', 'bytes': 2 * cols.numel() * x.element_size()})
    return cols


def col2im_nhwc(cols, x_shape, KH, KW, stride, pad):
    """Adjoint of im2col_nhwc: (B*Ho*Wo, KH*KW*C) -> (B, H, W, C)."""
    B, H, W, C = x_shape
    sh, sw = (stride, stride) if isinstance(stride, int) else stride
    ph, pw = (pad, pad) if isinstance(pad, int) else pad
    Ho, Wo = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
    dx = torch.empty((B, H, W, C), dtype=cols.dtype, device=cols.device)
    N.call('kinet_col2im_nhwc', N.ptr(cols.contiguous()), N.ptr(dx), B, H, W, C, Ho, Wo, KH, KW, sh, sw, ph, pw,
           N.dtype_code(cols.dtype), N.stream(cols.device),
           work={'family': 'grad', 'bytes': (cols.numel() + dx.numel()) * cols.element_size()})
    return dx


def gemm_tn(a, b, out=None, accumulate=False):
    """out (M, N) f32 [+]= a^T b for a (K, M), b (K, N) (kinet_gemm_tn): weight gradients."""
    N.require_gpu(a, b)
    if a.stride(-1) != 1:
        a = a.contiguous()
    if b.stride(-1) != 1:
        b = b.contiguous()
    K_, M = a.shape
    K2, Nn = b.shape
    if K2 != K_ or a.dtype != b.dtype:
        raise RuntimeError('gemm_tn: operand mismatch')
    if out is None:
        out = torch.empty((M, Nn), dtype=torch.float32, device=a.device)
    nws = N.lib().kinet_gemm_tn_workspace(M, Nn, K_)
    if accumulate:
        nws = max(nws, M * Nn)
    ws = torch.empty(max(1, nws), dtype=torch.float32, device=a.device) if nws else None
    N.call('kinet_gemm_tn', N.ptr(a), N.ptr(b), N.ptr(out), M, Nn, K_, a.stride(0), b.stride(0), out.stride(0),
           mm_code(a.dtype), int(accumulate), N.ptr(ws), N.stream(a.device),
           work={'family': 'gemm', 'flops': 2.0 * M * Nn * K_, 'shape': ('tn', M, Nn, K_)})
    return out


def colsum(a, out=None, accumulate=False):
    """out[c] (+)= sum_r a[r, c] (f32)."""
    if a.stride(-1) != 1:
        a = a.contiguous()
    R, C = a.shape
    if out is None:
        out = torch.empty(C, dtype=torch.float32, device=a.device)
    ws = torch.empty(max(1, N.lib().kinet_colsum_workspace(R, C)), dtype=torch.float32, device=a.device)
    N.call('kinet_colsum', N.ptr(a), N.ptr(out), R, C, a.stride(0), N.dtype_code(a.dtype), int(accumulate), N.ptr(ws),
           N.stream(a.device), work={'family': 'grad', 'bytes': a.numel() * a.element_size()})
    return out


def layernorm_backward(dy, x, gamma, eps, need_params=True):
    d = x.shape[-1]
    dy2, x2 = dy.reshape(-1, d).contiguous(), x.reshape(-1, d).contiguous()
    rows = x2.shape[0]
    dx = torch.empty_like(x2)
    dg = torch.empty(d, dtype=torch.float32, device=x.device) if need_params else None
    db = torch.empty(d, dtype=torch.float32, device=x.device) if need_params else None
    ws = torch.empty(max(1, N.lib().kinet_layernorm_backward_workspace(rows, d)), dtype=torch.float32, device=x.device)
    N.call('kinet_layernorm_backward', N.ptr(dy2), N.ptr(x2), N.ptr(f32(gamma)), N.ptr(dx), N.ptr(dg), N.ptr(db), rows,
           d, float(eps), N.dtype_code(x.dtype), N.ptr(ws), N.stream(x.device),
           work={'family': 'norm', 'bytes': 3 * x2.numel() * x2.element_size()})
    return dx.view(x.shape), dg, db


def _rows(t, d):
    t = t.reshape(-1, d)
    return t if t.is_contiguous() else t.contiguous()


def dropout_add_layernorm(x, r, weight, bias, eps, p, seed):
    """LayerNorm(x + dropout_p(r)) over the last dim, f32 (kinet_dropout_add_layernorm)."""
    d = x.shape[-1]
    x2, r2 = _rows(x, d), _rows(r, d)
    y = torch.empty_like(x2)
    N.call('kinet_dropout_add_layernorm', N.ptr(x2), N.ptr(r2), N.ptr(f32(weight)), N.ptr(f32(bias)), N.ptr(y),
           x2.shape[0], d, float(eps), float(p), N.ptr(seed), N.stream(x.device),
           work={'family': 'norm', 'bytes': 3 * x2.numel() * 4})
    return y.view(x.shape)


def dropout_add_layernorm_backward(dy, x, r, gamma, eps, p, seed, need_x=True, need_r=True, need_params=True):
    d = x.shape[-1]
    dy2, x2, r2 = _rows(dy, d), _rows(x, d), _rows(r, d)
    rows = x2.shape[0]
    dx = torch.empty_like(x2) if need_x else None
    dr = torch.empty_like(x2) if need_r else None
    dg = torch.empty(d, dtype=torch.float32, device=x.device) if need_params else None
    db = torch.empty(d, dtype=torch.float32, device=x.device) if need_params else None
    ws = torch.empty(max(1, N.lib().kinet_dropout_add_layernorm_backward_workspace(rows, d)) if need_params else 1,
                     dtype=torch.float32, device=x.device)
    N.call('kinet_dropout_add_layernorm_backward', N.ptr(dy2), N.ptr(x2), N.ptr(r2), N.ptr(f32(gamma)), N.ptr(dx),
           N.ptr(dr), N.ptr(dg), N.ptr(db), rows, d, float(eps), float(p), N.ptr(seed), N.ptr(ws), N.stream(x.device),
           work={'family': 'norm', 'bytes': 5 * x2.numel() * 4})
    return (None if dx is None else dx.view(x.shape)), (None if dr is None else dr.view(x.shape)), dg, db


def dropout_act(x, p, seed, relu):
    """dropout_p(relu(x)) (relu optional), f32 (kinet_dropout_act)."""
    x = x.contiguous()
    y = torch.empty_like(x)
    N.call('kinet_dropout_act', N.ptr(x), N.ptr(y), x.numel(), int(relu), float(p), N.ptr(seed), N.stream(x.device),
           work={'family': 'eltwise', 'bytes': 2 * x.numel() * 4})
    return y


def dropout_act_backward(dy, y, p, seed, relu):
    dy = dy.contiguous()
    dx = torch.empty_like(dy)
    N.call('kinet_dropout_act_backward', N.ptr(dy), N.ptr(y), N.ptr(dx), dy.numel(), int(relu), float(p), N.ptr(seed),
           N.stream(dy.device), work={'family': 'eltwise', 'bytes': 3 * dy.numel() * 4})
    return dx


def _packed_rows(t):
    """(N, Lq, C) with unit column stride and packed batches -> its row stride (elements)."""
    if t.stride(-1) != 1 or t.stride(0) != t.shape[1] * t.stride(1):
        t = t.contiguous()
    return t, t.stride(1)


def msda_prep(offlog, refs, shapes, query_mask, heads, levels, points):
    """Sampling locations (N, Lq, M, L, P, 2) and attention weights (N, Lq, M, L, P) from the
    packed [sampling offsets | attention logits] projection (N, Lq, >= M*L*P*3)
    (ms_deform_attn.py:64-82), f32 (kinet_msda_prep)."""
    Nb, Lq = offlog.shape[:2]
    ol, ld = _packed_rows(offlog)
    rf = refs.contiguous()
    loc = torch.empty((Nb, Lq, heads, levels, points, 2), dtype=torch.float32, device=ol.device)
    attw = torch.empty((Nb, Lq, heads, levels, points), dtype=torch.float32, device=ol.device)
    qm = query_mask.to(torch.uint8).contiguous() if query_mask is not None else None
    N.call('kinet_msda_prep', N.ptr(ol), ld, N.ptr(rf), N.ptr(shapes.contiguous()), N.ptr(qm), N.ptr(loc),
           N.ptr(attw), Nb * Lq, heads, levels, points, rf.shape[-1], N.stream(ol.device),
           work={'family': 'msda_glue', 'bytes': 2 * (loc.numel() + attw.numel()) * 4})
    return loc, attw


def msda_prep_backward(grad_loc, grad_attw, attw, offlog, refs, shapes, heads, levels, points,
                       need_offlog=True, need_refs=True):
    """Gradients of msda_prep: w.r.t. the packed offlog (its layout, contiguous) and refs."""
    Nb, Lq = offlog.shape[:2]
    dev = offlog.device
    gl, ga = grad_loc.contiguous(), grad_attw.contiguous()
    ol = offlog.contiguous()      # the gradient takes offlog's (contiguous) layout
    ld = ol.shape[-1]
    rf = refs.contiguous()
    dol = torch.empty(ol.shape, dtype=torch.float32, device=dev) if need_offlog else None
    dref = torch.empty(rf.shape, dtype=torch.float32, device=dev) if need_refs else None
    N.call('kinet_msda_prep_backward', N.ptr(gl), N.ptr(ga), N.ptr(attw), N.ptr(ol), ld, N.ptr(rf),
           N.ptr(shapes.contiguous()), N.ptr(dol), N.ptr(dref), Nb * Lq, heads, levels, points, rf.shape[-1],
           N.stream(dev), work={'family': 'msda_glue', 'bytes': 3 * (gl.numel() + ga.numel()) * 4})
    return dol, dref


def inverse_sigmoid(x, eps=1e-5):
    x = x.contiguous()
    y = torch.empty_like(x)
    N.call('kinet_inverse_sigmoid', N.ptr(x), N.ptr(y), x.numel(), float(eps), N.stream(x.device),
           work={'family': 'eltwise', 'bytes': 2 * x.numel() * 4})
    return y


def inverse_sigmoid_backward(dy, x, eps=1e-5):
    dy = dy.contiguous()
    dx = torch.empty_like(dy)
    N.call('kinet_inverse_sigmoid_backward', N.ptr(dy), N.ptr(x), N.ptr(dx), dy.numel(), float(eps),
           N.stream(dy.device), work={'family': 'eltwise', 'bytes': 3 * dy.numel() * 4})
    return dx


def groupnorm_backward(dy, x, gamma, groups, eps, need_params=True):
    """x, dy (B, HW, C) NHWC."""
    B, HW, C = x.shape
    dy, x = dy.contiguous(), x.contiguous()
    dx = torch.empty_like(x)
    dg = torch.empty(C, dtype=torch.float32, device=x.device) if need_params else None
    db = torch.empty(C, dtype=torch.float32, device=x.device) if need_params else None
    ws = torch.empty(max(1, N.lib().kinet_groupnorm_backward_workspace(B, HW, C, groups)), dtype=torch.float32,
                     device=x.device)
    N.call('kinet_groupnorm_backward', N.ptr(dy), N.ptr(x), N.ptr(f32(gamma)), N.ptr(dx), N.ptr(dg), N.ptr(db), B, HW,
           C, groups, float(eps), N.dtype_code(x.dtype), N.ptr(ws), N.stream(x.device),
           work={'family': 'norm', 'bytes': 4 * x.numel() * x.element_size()})
    return dx, dg, db


def mha_backward_qk(qk, v, do, heads, scale, key_mask=None, dropout_p=0.0, seed=None):
    """Backward of mha_core on the packed [q | k] projection qk (B, L, 2E) (self-attention,
    q = k input): returns dqk (B, L, 2E, the same packing -- the input gradient of ONE q|k
    projection GEMM) and dv."""
    B, L, E2 = qk.shape
    E = E2 // 2
    qk, v, do = qk.contiguous(), v.contiguous(), do.contiguous()
    for t in (qk, v, do):
        if t.dtype != torch.float32:
            raise RuntimeError('mha_backward_qk: f32 operands')
    dqk = torch.empty((B, L, E2), dtype=torch.float32, device=qk.device)
    dv = torch.empty((B, L, E), dtype=torch.float32, device=qk.device)
    ws = torch.empty(max(1, N.lib().kinet_mha_backward_workspace(B, L, L, heads)), dtype=torch.float32,
                     device=qk.device)
    km = key_mask.to(torch.uint8).contiguous() if key_mask is not None else None
    N.call('kinet_mha_backward', N.ptr(qk), E2, N.ptr(qk[..., E:]), E2, N.ptr(v), E, N.ptr(do), E, N.ptr(dqk),
           N.ptr(dqk[..., E:]), N.ptr(dv), B, L, L, heads, E // heads, float(scale), N.ptr(km), N.ptr(ws),
           float(dropout_p), N.ptr(seed) if dropout_p > 0 else None, N.stream(qk.device),
           work={'family': 'attn', 'flops': 8.0 * B * heads * L * L * (E // heads)})
    return dqk, dv


def mha_backward(q, k, v, do, heads, scale, key_mask=None, dropout_p=0.0, seed=None):
    """Backward of mha_core (f32): returns dq, dk, dv with the layouts of q, k, v."""
    B, Lq, E = q.shape
    Lk = k.shape[1]
    for t in (q, k, v, do):
        if t.dtype != torch.float32 or t.stride(-1) != 1 or t.stride(0) != t.shape[1] * t.stride(1):
            raise RuntimeError('mha_backward: f32 rows, unit stride, packed batches')
    dq = torch.empty((B, Lq, E), dtype=torch.float32, device=q.device)
    dk = torch.empty((B, Lk, E), dtype=torch.float32, device=q.device)
    dv = torch.empty((B, Lk, E), dtype=torch.float32, device=q.device)
    ws = torch.empty(max(1, N.lib().kinet_mha_backward_workspace(B, Lq, Lk, heads)), dtype=torch.float32,
                     device=q.device)
    km = key_mask.to(torch.uint8).contiguous() if key_mask is not None else None
    # dq/dk/dv are written with q/k/v's row strides: give them packed copies of the layouts
    if q.stride(1) != E or k.stride(1) != E or v.stride(1) != E:
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
    N.call('kinet_mha_backward', N.ptr(q), E, N.ptr(k), E, N.ptr(v), E, N.ptr(do.contiguous()), E, N.ptr(dq),
           N.ptr(dk), N.ptr(dv), B, Lq, Lk, heads, E // heads, float(scale), N.ptr(km), N.ptr(ws), float(dropout_p),
           N.ptr(seed) if dropout_p > 0 else None, N.stream(q.device),
           work={'family': 'attn', 'flops': 8.0 * B * heads * Lq * Lk * (E // heads)})
    return dq, dk, dv

"""Training-path operators on kinet_amd kernels: torch.autograd.Functions whose forward AND
backward run the hand-written HIP kernels (include/kinet_gemm.h, kinet_ops.h, kinet_grad.h).

The reference trains the detector with `losses.backward()` (src/trackformer/engine.py:
145-149) through torch's Conv2d / Linear / LayerNorm / GroupNorm / MultiheadAttention
(cuDNN / cuBLAS); kinet_amd's autograd path (DeformableDETR._forward_reference and the
transformer / backbone modules under autograd) calls these functions instead, so a
training step runs no vendor GEMM / convolution library kernel.  Compute dtype is f32, as
the reference trains (no AMP anywhere in src/).  The transformer's elementwise glue runs on
kinet kernels too (csrc/train_ops.hip): residual dropout + LayerNorm, dropout(relu) of the
FFN hidden, the MSDA softmax / sampling-location preparation and inverse_sigmoid, one kernel
each way; what stays in torch is autograd's own gradient accumulation, the loss and the
sigmoid / masked_fill glue of the heads.

    linear(x, weight, bias)                 nn.Linear
    layer_norm(x, weight, bias, eps)        nn.LayerNorm over the last dim
    group_norm_nhwc(x, groups, w, b, eps)   nn.GroupNorm on (B, HW, C)
    conv_nhwc(x, weight, ...)               nn.Conv2d (+ FrozenBatchNorm2d, residual, ReLU) on NHWC
    mha_core(q, k, v, heads, key_mask)      the softmax(QK^T / sqrt(d)) V core of nn.MultiheadAttention
    dropout_add_layer_norm(x, r, ln, drop)  ln(x + drop(r)), the post-norm residual sub-layer
    dropout_act(x, drop)                    drop(relu(x)), the FFN hidden
    msda_prep(off, logits, refs, ...)       MSDeformAttn sampling locations + softmaxed weights
    inverse_sigmoid(x)                      util/misc.py:609-613

Weight gradients are reductions over the row (pixel / token) dimension (kinet_gemm_tn,
split-K with a fixed-order finalize), input gradients are GEMMs against the transposed
weight (kinet_gemm_ex) -- for convolutions against the patch matrix, scattered back by
the deterministic kinet_col2im_nhwc gather.
"""
import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from kinet_amd import _native as N
from kinet_amd import kernels as K


def _f32(t):
    if t.dtype != torch.float32:
        raise RuntimeError(f'kinet_amd training path computes in f32 (got {t.dtype})')
    return t


# ----------------------------------------------------------------------------- Linear
class _Linear(Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        N.require_gpu(x)
        _f32(x)
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        if x2.stride(-1) != 1 or x2.stride(0) != x2.shape[1]:
            x2 = x2.contiguous()
        # the output is allocated in its final shape (not a view of a 2-D result), so callers
        # may modify it in place as they would an nn.Linear output (deformable_transformer.py:420)
        y = torch.empty(*lead, weight.shape[0], dtype=x.dtype, device=x.device)
        K.linear(x2, weight.detach(), None if bias is None else bias.detach(), out=y.view(-1, weight.shape[0]))
        ctx.save_for_backward(x2, weight)
        ctx.has_bias = bias is not None
        ctx.lead = lead
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous().float()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wt = K.transpose2d(weight.detach().float())                 # (in, out)
            n_out = dy2.shape[1]
            if n_out % 8:   # the GEMM's K (= out features, e.g. 20 class logits) must be 8-aligned
                pad = 8 - n_out % 8
                dy_p, wt = torch.nn.functional.pad(dy2, (0, pad)), torch.nn.functional.pad(wt, (0, pad))
            else:
                dy_p = dy2
            dx = K.linear(dy_p, wt).view(*ctx.lead, x2.shape[1])        # dy @ W
        if ctx.needs_input_grad[1]:
            dw = K.gemm_tn(dy2, x2)                                     # dy^T x
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = K.colsum(dy2)
        return dx, dw, db


def linear(x, weight, bias=None):
    """F.linear(x, weight, bias) on kinet kernels (forward and backward)."""
    return _Linear.apply(x, weight, bias)


def linear_module(x, mod):
    return _Linear.apply(x, mod.weight, mod.bias)


# ---------------------------------------------------------------------------- LayerNorm
class _LayerNorm(Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        _f32(x)
        xc = x.contiguous()
        y = K.layernorm(xc, weight.detach(), bias.detach(), eps)
        ctx.save_for_backward(xc, weight)
        ctx.eps = eps
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        need_p = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        dx, dg, db = K.layernorm_backward(dy.contiguous().float(), x, weight, ctx.eps, need_params=need_p)
        return (dx if ctx.needs_input_grad[0] else None, dg if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None, None)


def layer_norm(x, ln):
    """nn.LayerNorm `ln` applied to x (last dim)."""
    return _LayerNorm.apply(x, ln.weight, ln.bias, float(ln.eps))


# ---------------------------------------------------------------------------- GroupNorm
class _GroupNormNHWC(Function):
    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps):
        _f32(x)
        xc = x.contiguous()
        y = K.groupnorm_nhwc(xc, weight.detach(), bias.detach(), groups, eps)
        ctx.save_for_backward(xc, weight)
        ctx.groups, ctx.eps = groups, eps
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        need_p = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        dx, dg, db = K.groupnorm_backward(dy.contiguous().float(), x, weight, ctx.groups, ctx.eps, need_params=need_p)
        return (dx if ctx.needs_input_grad[0] else None, dg if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None, None, None)


def group_norm_nhwc(x, gn):
    """nn.GroupNorm `gn` on x (B, HW, C)."""
    return _GroupNormNHWC.apply(x, gn.weight, gn.bias, gn.num_groups, float(gn.eps))


# ------------------------------------------------------------------------------ Conv2d
class _ConvNHWC(Function):
    """y = relu?(conv(x, W) * scale + shift + residual), NHWC; scale/shift: a folded
    FrozenBatchNorm2d (constants) or (None, conv bias)."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, stride, pad, scale, shift, relu):
        _f32(x)
        x = x.contiguous()
        wp = K.pack_conv_weight(weight, torch.float32)                       # (O, KH, KW, I)
        sh = shift if bias is None else bias.detach().float().contiguous()
        y = K.conv2d_nhwc(x, wp, stride, pad, scale=scale, bias=sh, relu=relu,
                          residual=None if residual is None else residual.contiguous())
        ctx.save_for_backward(x, weight, y if relu else None)
        ctx.conf = (stride, pad, scale, relu, bias is not None, residual is not None)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        stride, pad, scale, relu, has_bias, has_res = ctx.conf
        dz = dy.contiguous().float()
        if relu:
            dz = dz.masked_fill(y <= 0, 0.0)
        d_res = dz if has_res and ctx.needs_input_grad[3] else None
        dzs = dz * scale if scale is not None else dz                       # through the folded BN scale
        O, I, KH, KW = weight.shape
        B, H, W, _ = x.shape
        Ho, Wo = dz.shape[1], dz.shape[2]
        dz2 = dzs.reshape(B * Ho * Wo, O)
        s = (stride, stride) if isinstance(stride, int) else stride
        p = (pad, pad) if isinstance(pad, int) else pad
        pointwise = KH == 1 and KW == 1 and s == (1, 1) and p == (0, 0)
        dx = dw = db = None
        if ctx.needs_input_grad[1]:
            cols = x.reshape(B * H * W, I) if pointwise else K.im2col_nhwc(x, KH, KW, s, p)
            g = K.gemm_tn(dz2, cols)
            # a 1x1 kernel's (O, I) rows already are the OIHW layout: viewed, not permuted, so the
            # gradient carries the parameter's own strides (I, 1, 1, 1) -- a permuted view keeps
            # (I, 1, I, I), which DDP's bucket views reject with a copy per step
            dw = g.view(O, I, 1, 1) if KH == 1 and KW == 1 else g.view(O, KH, KW, I).permute(0, 3, 1, 2).contiguous()
        if ctx.needs_input_grad[0]:
            wpt = K.transpose2d(K.pack_conv_weight(weight, torch.float32).reshape(O, KH * KW * I))   # (KH*KW*I, O)
            dcols = K.linear(dz2, wpt)                                                            # (P, KH*KW*I)
            dx = dcols.view(B, H, W, I) if pointwise else K.col2im_nhwc(dcols, (B, H, W, I), KH, KW, s, p)
        if has_bias and ctx.needs_input_grad[2]:
            db = K.colsum(dz2)
        return dx, dw, db, d_res, None, None, None, None, None


def conv_nhwc(x, weight, bias=None, stride=1, pad=0, scale=None, shift=None, relu=False, residual=None):
    """Convolution of NHWC x with an OIHW weight (+ bias or folded-BN scale/shift, residual,
    ReLU) on kinet kernels, differentiable w.r.t. x, weight, bias and residual."""
    return _ConvNHWC.apply(x, weight, bias, residual, stride, pad, scale, shift, relu)


# ---------------------------------------------------------------------------- attention
class _MHACore(Function):
    @staticmethod
    def forward(ctx, q, k, v, heads, scale, key_mask, dropout_p, seed):
        _f32(q)
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o = K.mha_core(q, k, v, heads, scale, key_mask=key_mask, dropout_p=dropout_p, seed=seed)
        ctx.save_for_backward(q, k, v)
        ctx.conf = (heads, scale, key_mask, dropout_p, seed)
        return o

    @staticmethod
    @once_differentiable
    def backward(ctx, do):
        q, k, v = ctx.saved_tensors
        heads, scale, key_mask, dropout_p, seed = ctx.conf
        dq, dk, dv = K.mha_backward(q, k, v, do.contiguous().float(), heads, scale, key_mask, dropout_p, seed)
        return dq, dk, dv, None, None, None, None, None


def mha_core(q, k, v, heads, scale, key_mask=None, dropout_p=0.0, seed=None):
    """softmax(q k^T * scale, -inf at masked keys) v per head; q (B, Lq, E), k/v (B, Lk, E).
    dropout_p > 0: the probabilities are dropped (and the survivors scaled by 1/(1-p)) with
    the keep mask of the device int64 `seed` (kernels.dropout_seed when None), regenerated
    by the backward."""
    if dropout_p > 0 and seed is None:
        seed = K.dropout_seed(q.device)
    return _MHACore.apply(q, k, v, heads, scale, key_mask, float(dropout_p), seed)


class _MHACoreQK(Function):
    """mha_core with q and k the two halves of one packed projection qk (B, L, 2E): the
    backward returns the packed gradient (one q|k input-gradient GEMM, no add of two)."""

    @staticmethod
    def forward(ctx, qk, v, heads, scale, key_mask, dropout_p, seed):
        _f32(qk)
        qk, v = qk.contiguous(), v.contiguous()
        E = qk.shape[-1] // 2
        o = K.mha_core(qk[..., :E], qk[..., E:], v, heads, scale, key_mask=key_mask, dropout_p=dropout_p, seed=seed)
        ctx.save_for_backward(qk, v)
        ctx.conf = (heads, scale, key_mask, dropout_p, seed)
        return o

    @staticmethod
    @once_differentiable
    def backward(ctx, do):
        qk, v = ctx.saved_tensors
        heads, scale, key_mask, dropout_p, seed = ctx.conf
        dqk, dv = K.mha_backward_qk(qk, v, do.float(), heads, scale, key_mask, dropout_p, seed)
        return dqk, dv, None, None, None, None, None


def multihead_attention(mod, query, key, value, key_padding_mask=None):
    """nn.MultiheadAttention(query, key, value, key_padding_mask)[0] for batch-first inputs
    (the decoder self-attention, deformable_transformer.py:371, transposes to (L, B, E) and
    back around the call): in_proj split q|k|v (torch's packed in_proj_weight layout),
    attention core, out_proj.  In training mode the attention probabilities are dropped with
    the module's `dropout` probability (nn.MultiheadAttention(d, heads, dropout=p),
    deformable_transformer.py:345), in the HIP core; the mask comes from torch's CUDA
    generator state through a device seed, so it is not torch's own mask (parity by mask
    statistics and by gradients under a fixed mask, tests/test_autograd_gpu.py)."""
    E = mod.embed_dim
    w, b = mod.in_proj_weight, mod.in_proj_bias
    p = mod.dropout if mod.training else 0.0
    if query is key:
        # self-attention with q = k inputs (deformable_transformer.py:370): ONE GEMM for the
        # packed q|k projection, its gradient packed the same way
        qk = linear(query, w[:2 * E], b[:2 * E])
        v = linear(value, w[2 * E:], b[2 * E:])
        seed = K.dropout_seed(qk.device) if p > 0 else None
        o = _MHACoreQK.apply(qk, v, mod.num_heads, mod.head_dim ** -0.5, key_padding_mask, float(p), seed)
        return linear(o, mod.out_proj.weight, mod.out_proj.bias)
    q = linear(query, w[:E], b[:E])
    k = linear(key, w[E:2 * E], b[E:2 * E])
    v = linear(value, w[2 * E:], b[2 * E:])
    o = mha_core(q, k, v, mod.num_heads, mod.head_dim ** -0.5, key_padding_mask, dropout_p=p)
    return linear(o, mod.out_proj.weight, mod.out_proj.bias)


# ------------------------------------------------------- training glue (csrc/train_ops.hip)
_ZERO_SEED = {}


def _seed(device, p):
    """A fresh device seed when dropout is active, else a cached zero seed (p = 0 keeps all)."""
    if p > 0:
        return K.dropout_seed(device)
    s = _ZERO_SEED.get(device)
    if s is None:
        s = _ZERO_SEED[device] = torch.zeros(1, dtype=torch.int64, device=device)
    return s


def _drop_p(drop):
    return float(drop.p) if drop is not None and drop.training else 0.0


class _DropoutAddLayerNorm(Function):
    @staticmethod
    def forward(ctx, x, r, weight, bias, eps, p, seed):
        _f32(x)
        _f32(r)
        y = K.dropout_add_layernorm(x, r, weight.detach(), bias.detach(), eps, p, seed)
        ctx.save_for_backward(x, r, weight, seed)
        ctx.conf = (eps, p)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x, r, weight, seed = ctx.saved_tensors
        eps, p = ctx.conf
        ng = ctx.needs_input_grad
        dx, dr, dg, db = K.dropout_add_layernorm_backward(dy.float(), x, r, weight, eps, p, seed, need_x=ng[0],
                                                          need_r=ng[1], need_params=ng[2] or ng[3])
        return dx, dr, dg if ng[2] else None, db if ng[3] else None, None, None, None


def dropout_add_layer_norm(x, r, ln, drop):
    """ln(x + drop(r)) -- the post-norm residual sub-layer (deformable_transformer.py:100,108,
    186,196,199) as one kernel forward and one backward; `drop` an nn.Dropout (its p applies in
    training mode), the keep mask from a device seed drawn from torch's CUDA generator."""
    p = _drop_p(drop)
    return _DropoutAddLayerNorm.apply(x, r, ln.weight, ln.bias, float(ln.eps), p, _seed(x.device, p))


class _DropoutAct(Function):
    @staticmethod
    def forward(ctx, x, p, seed, relu):
        _f32(x)
        y = K.dropout_act(x, p, seed, relu)
        ctx.save_for_backward(y if relu else None, seed)
        ctx.conf = (p, relu)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        y, seed = ctx.saved_tensors
        p, relu = ctx.conf
        return K.dropout_act_backward(dy.float(), y, p, seed, relu), None, None, None


def dropout_act(x, drop, relu=True):
    """drop(relu(x)) (the FFN hidden, deformable_transformer.py:99,185) in one kernel each way."""
    p = _drop_p(drop)
    return _DropoutAct.apply(x, p, _seed(x.device, p), relu)


class _MSDAPrep(Function):
    @staticmethod
    def forward(ctx, offlog, refs, shapes, query_mask, heads, levels, points):
        _f32(offlog)
        loc, attw = K.msda_prep(offlog, refs.float(), shapes, query_mask, heads, levels, points)
        ctx.save_for_backward(attw, offlog, refs, shapes)
        ctx.conf = (heads, levels, points)
        return loc, attw

    @staticmethod
    @once_differentiable
    def backward(ctx, dloc, dattw):
        attw, offlog, refs, shapes = ctx.saved_tensors
        heads, levels, points = ctx.conf
        ng = ctx.needs_input_grad
        dloc = torch.zeros(attw.shape + (2,), dtype=torch.float32, device=attw.device) if dloc is None else dloc.float()
        dattw = torch.zeros_like(attw) if dattw is None else dattw.float()
        dol, dref = K.msda_prep_backward(dloc, dattw, attw, offlog, refs.float(), shapes, heads, levels, points,
                                         need_offlog=ng[0], need_refs=ng[1])
        if dref is not None and dref.dtype != refs.dtype:
            dref = dref.to(refs.dtype)
        return dol, dref, None, None, None, None, None


def msda_prep(offlog, refs, shapes, query_mask, heads, levels, points):
    """(sampling_locations, attention_weights) of MSDeformAttn (ms_deform_attn.py:64-82) from the
    packed projection offlog (N, Lq, M*L*P*2 offsets | M*L*P logits) and refs (N, Lq, L, 2|4):
    loc (N, Lq, M, L, P, 2), attw (N, Lq, M, L, P) (softmax over L*P, 0 at masked queries);
    differentiable w.r.t. offlog and refs, one kernel each way."""
    return _MSDAPrep.apply(offlog, refs, shapes, query_mask, heads, levels, points)


class _InverseSigmoid(Function):
    @staticmethod
    def forward(ctx, x, eps):
        xc = x.contiguous()
        ctx.save_for_backward(xc)
        ctx.eps = eps
        return K.inverse_sigmoid(xc, eps)

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        return K.inverse_sigmoid_backward(dy.float(), x, ctx.eps), None


def inverse_sigmoid(x, eps=1e-5):
    """util/misc.py:609-613 on f32 device tensors, one kernel each way."""
    return _InverseSigmoid.apply(x, float(eps))

"""ORACLE / TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
and there only as the checker / the timed CPU baseline -- never by kinet_amd.

Two CPU restatements of the reference MSDeformAttn sampling operator:

* `core_pytorch(value, shapes, loc, attw)` -- restates
  `ms_deform_attn_core_pytorch` (src/trackformer/models/ops/functions/ms_deform_attn_func.py:34-54):
  per-level `F.grid_sample(bilinear, zeros, align_corners=False)` on (N*M, D, H, W)
  with grid = 2*loc - 1, weighted sum over L*P.  This is "the reference CPU path"
  that BASELINE.json names; it is also what bench.py times as cpu_baseline.
* `fwd(...)` / `bwd(...)` -- ctypes front-end of oracle/msda_oracle.c, the loop-nest
  restatement of the CUDA kernels (ms_deform_im2col_cuda.cuh:165-378), including
  the backward the reference only has on CUDA.

Both are pinned against tests/golden/msda_*.npz (produced from the reference itself
by tests/golden/make_golden.py) in tests/test_oracle_golden.py.
"""
import ctypes
import os
import subprocess

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_SRC = os.path.join(_HERE, "msda_oracle.c")
_LIB = os.path.join(_HERE, "_build", "libmsda_oracle.so")


def build():
    """Compile the C restatement (gcc, no reference sources involved)."""
    os.makedirs(os.path.dirname(_LIB), exist_ok=True)
    if os.path.exists(_LIB) and os.path.getmtime(_LIB) >= os.path.getmtime(_SRC):
        return _LIB
    subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", _LIB, _SRC, "-lm"])
    return _LIB


_lib = None


def _load():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        for suf in ("f32", "f64"):
            getattr(_lib, f"msda_oracle_fwd_{suf}").restype = ctypes.c_int
            getattr(_lib, f"msda_oracle_bwd_{suf}").restype = ctypes.c_int
    return _lib


def level_start_index(shapes):
    shapes = np.asarray(shapes, dtype=np.int64).reshape(-1, 2)
    areas = shapes[:, 0] * shapes[:, 1]
    return np.concatenate([[0], np.cumsum(areas)[:-1]]).astype(np.int64)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _dims(value, loc):
    N, S, M, D = value.shape
    _, Lq, M2, L, P, two = loc.shape
    assert M2 == M and two == 2
    return N, S, M, D, L, Lq, P


def fwd(value, shapes, loc, attw):
    """numpy in/out; dtype float32 or float64 -> (N, Lq, M*D)."""
    value = np.ascontiguousarray(value)
    dt = value.dtype
    suf = {np.dtype(np.float32): "f32", np.dtype(np.float64): "f64"}[dt]
    loc = np.ascontiguousarray(loc, dtype=dt)
    attw = np.ascontiguousarray(attw, dtype=dt)
    shapes = np.ascontiguousarray(shapes, dtype=np.int64).reshape(-1, 2)
    ls = level_start_index(shapes)
    N, S, M, D, L, Lq, P = _dims(value, loc)
    out = np.zeros((N, Lq, M * D), dtype=dt)
    rc = getattr(_load(), f"msda_oracle_fwd_{suf}")(
        _ptr(value), _ptr(shapes), _ptr(ls), _ptr(loc), _ptr(attw), _ptr(out),
        N, S, M, D, L, Lq, P)
    assert rc == 0
    return out


def bwd(value, shapes, loc, attw, grad_out):
    """-> (grad_value, grad_loc, grad_attw), same dtype as value."""
    value = np.ascontiguousarray(value)
    dt = value.dtype
    suf = {np.dtype(np.float32): "f32", np.dtype(np.float64): "f64"}[dt]
    loc = np.ascontiguousarray(loc, dtype=dt)
    attw = np.ascontiguousarray(attw, dtype=dt)
    grad_out = np.ascontiguousarray(grad_out, dtype=dt)
    shapes = np.ascontiguousarray(shapes, dtype=np.int64).reshape(-1, 2)
    ls = level_start_index(shapes)
    N, S, M, D, L, Lq, P = _dims(value, loc)
    gv = np.zeros_like(value)
    gl = np.zeros_like(loc)
    ga = np.zeros_like(attw)
    rc = getattr(_load(), f"msda_oracle_bwd_{suf}")(
        _ptr(value), _ptr(shapes), _ptr(ls), _ptr(loc), _ptr(attw), _ptr(grad_out),
        _ptr(gv), _ptr(gl), _ptr(ga), N, S, M, D, L, Lq, P)
    assert rc == 0
    return gv, gl, ga


def core_pytorch(value, value_spatial_shapes, sampling_locations, attention_weights):
    """Restatement of ms_deform_attn_core_pytorch (ms_deform_attn_func.py:34-54); torch CPU tensors."""
    N_, S_, M_, D_ = value.shape
    _, Lq_, M_, L_, P_, _ = sampling_locations.shape
    hw = [(int(h), int(w)) for h, w in value_spatial_shapes]
    value_list = value.split([h * w for h, w in hw], dim=1)
    grids = 2 * sampling_locations - 1
    sampled = []
    for lid, (H_, W_) in enumerate(hw):
        v = value_list[lid].flatten(2).transpose(1, 2).reshape(N_ * M_, D_, H_, W_)
        g = grids[:, :, :, lid].transpose(1, 2).flatten(0, 1)
        sampled.append(F.grid_sample(v, g, mode='bilinear', padding_mode='zeros', align_corners=False))
    aw = attention_weights.transpose(1, 2).reshape(N_ * M_, 1, Lq_, L_ * P_)
    out = (torch.stack(sampled, dim=-2).flatten(-2) * aw).sum(-1).view(N_, M_ * D_, Lq_)
    return out.transpose(1, 2).contiguous()


# --------------------------------------------------------------------------- sampling records
# The encoder path's "sampling records" (kinet_msda_sample_records, include/kinet_msda.h): the
# reference's MSDA preparation (ms_deform_attn.py:68-82) followed by the bilinear setup of
# ms_deform_im2col_cuda.cuh:227-233, stored per (head, query, level, point) as a fixed-point
# top-left corner + fraction and an attention weight with the out-of-level corners folded in.

def prep(offlog, ref, shapes, qmask, M, L, P):
    """ms_deform_attn.py:68-82 op for op (torch CPU, the dtype of offlog): offlog (B, Lq,
    M*L*P*3) = [sampling_offsets (M, L, P, 2) | attention logits (M, L*P)] -> (loc (B, Lq, M, L,
    P, 2), attw (B, Lq, M, L, P))."""
    B, Lq = offlog.shape[:2]
    so = offlog[..., :M * L * P * 2].reshape(B, Lq, M, L, P, 2)
    aw = F.softmax(offlog[..., M * L * P * 2:].reshape(B, Lq, M, L * P), -1).reshape(B, Lq, M, L, P)
    if qmask is not None:
        aw = aw.masked_fill(qmask[..., None, None, None], 0.0)
    sh = torch.as_tensor(shapes, dtype=offlog.dtype)
    if ref.shape[-1] == 2:
        # the reference divides (x, y) by (H, W) -- spatial_shapes unswapped (:77-79)
        loc = ref[:, :, None, :, None, :] + so / sh[None, None, None, :, None, :]
    else:
        loc = ref[:, :, None, :, None, :2] + so / P * ref[:, :, None, :, None, 2:] * 0.5
    return loc, aw


def sample_records(loc, attw, ref, shapes, fb):
    """(loc, attw) as above + the (B, Lq, L, 2|4) reference points -> records (M, B, Lq, 24)
    int32 (96 bytes: [4 levels x 4 u32 locations | 4 levels x 4 f16 weights]), the encoding
    include/kinet_msda.h states: per sample h = y*H - 0.5, w = x*W - 0.5 (cuh:227-228); outside
    (-1, H) x (-1, W) (cuh:229) weight 0; a top row -1 becomes row 0 with the weight times lh and
    lh = 0, a bottom row H-1 keeps the weight times (1 - lh) and lh = 0, the same for columns;
    the location is the coordinate clamped into the level, rounded to fb fraction bits (a carry
    moves the corner) -- exactly the folded corner + fraction above; a sample outside the level
    has weight 0 at the query's own pixel."""
    loc = loc.double()
    a = attw.double().clone()
    B, Lq, M, L, P, _ = loc.shape
    H = torch.tensor([int(h) for h, _ in shapes], dtype=torch.float64)[None, None, None, :, None]
    W = torch.tensor([int(w) for _, w in shapes], dtype=torch.float64)[None, None, None, :, None]
    h = loc[..., 1] * H - 0.5
    w = loc[..., 0] * W - 0.5
    valid = (h > -1) & (w > -1) & (h < H) & (w < W)
    hl, wl = torch.floor(h), torch.floor(w)
    lh, lw = h - hl, w - wl
    top = hl < 0
    a = torch.where(top, a * lh, a)
    bot = ~top & (hl >= H - 1)
    a = torch.where(bot, a * (1 - lh), a)
    hl = torch.where(top, torch.zeros_like(hl), torch.where(bot, H - 1 + 0 * hl, hl))
    lh = torch.where(top | bot, torch.zeros_like(lh), lh)
    left = wl < 0
    a = torch.where(left, a * lw, a)
    right = ~left & (wl >= W - 1)
    a = torch.where(right, a * (1 - lw), a)
    wl = torch.where(left, torch.zeros_like(wl), torch.where(right, W - 1 + 0 * wl, wl))
    lw = torch.where(left | right, torch.zeros_like(lw), lw)
    s = float(1 << fb)
    a = torch.where(valid, a, torch.zeros_like(a))
    # fixed point of the clamped coordinate (= the folded corner + rounded fraction in the level)
    ph = torch.floor(torch.minimum(torch.clamp(h, min=0.0), H - 1) * s + 0.5)
    pw = torch.floor(torch.minimum(torch.clamp(w, min=0.0), W - 1) * s + 0.5)
    # outside the level: the query's own pixel, weight 0
    r = ref.double()[:, :, None, :, None, :]
    hr = torch.clamp(torch.floor(r[..., 1] * H), torch.zeros_like(H), H - 1).expand_as(ph)
    wr = torch.clamp(torch.floor(r[..., 0] * W), torch.zeros_like(W), W - 1).expand_as(pw)
    ph = torch.where(valid, ph, hr * s)
    pw = torch.where(valid, pw, wr * s)
    word = (ph.long() << 16) | pw.long()   # (B, Lq, M, L, P)
    word = word.to(torch.int64) & 0xffffffff
    locw = torch.where(word >= 2 ** 31, word - 2 ** 32, word).to(torch.int32)
    a16 = (a.to(torch.float16).view(torch.int16).to(torch.int32) & 0xffff).reshape(B, Lq, M, L * P)
    aw_words = a16[..., 0::2] | (a16[..., 1::2] << 16)                                          # (B, Lq, M, L*P/2)
    rec = torch.cat([locw.reshape(B, Lq, M, L * P), aw_words], -1)        # (B, Lq, M, 24) for L = P = 4
    return rec.permute(2, 0, 1, 3).contiguous()


def decode_records(rec, shapes, fb):
    """records (M, B, Lq, 1.5 L P) int32 (24 for L = P = 4) -> (loc (B, Lq, M, L, P, 2), attw (B, Lq, M, L, P)) float64
    whose reference sampling (cuh:165-237, `fwd`) is exactly what a record asks for: the corner
    (hl, wl) + fractions become the location ((wl + lw + 0.5) / W, (hl + lh + 0.5) / H)."""
    rec = rec.long() & 0xffffffff
    M, B, Lq, n = rec.shape
    L = len(shapes)
    P = (2 * n) // (3 * L)          # n = L*P locations + L*P/2 weight words
    locw = rec[..., :L * P].reshape(M, B, Lq, L, P)
    aww = rec[..., L * P:]
    hl = locw >> (16 + fb)
    qh = (locw >> 16) & ((1 << fb) - 1)
    wl = (locw >> fb) & ((1 << (16 - fb)) - 1)
    qw = locw & ((1 << fb) - 1)
    s = float(1 << fb)
    H = torch.tensor([int(h) for h, _ in shapes], dtype=torch.float64)[None, None, None, :, None]
    W = torch.tensor([int(w) for _, w in shapes], dtype=torch.float64)[None, None, None, :, None]
    y = (hl.double() + qh.double() / s + 0.5) / H
    x = (wl.double() + qw.double() / s + 0.5) / W
    lo = (aww & 0xffff).to(torch.int16)
    hi = ((aww >> 16) & 0xffff).to(torch.int16)
    a = torch.stack([lo, hi], -1).reshape(M, B, Lq, L, P).view(torch.float16).double()   # pairs of (l, p)
    loc = torch.stack([x, y], -1).permute(1, 2, 0, 3, 4, 5).contiguous()
    return loc, a.permute(1, 2, 0, 3, 4).contiguous()

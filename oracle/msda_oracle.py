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

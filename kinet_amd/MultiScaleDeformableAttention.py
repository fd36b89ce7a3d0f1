"""Drop-in for the reference extension module `MultiScaleDeformableAttention`
(pybind11 surface at src/trackformer/models/ops/src/vision.cpp:4-7), backed by
libkinet_amd.so (include/kinet_msda.h).

    ms_deform_attn_forward(value, spatial_shapes, sampling_loc, attn_weight, im2col_step)
        -> Tensor (N, Lq, M*D)                               [ms_deform_attn_cuda.cu:19-86]
    ms_deform_attn_backward(value, spatial_shapes, sampling_loc, attn_weight, grad_output, im2col_step)
        -> [grad_value, grad_sampling_loc, grad_attn_weight]  [ms_deform_attn_cuda.cu:89-168]

Same argument meaning, shapes and dtypes; validation errors are RuntimeError like the
reference's AT_ASSERTM.  Additionally accepts bf16/fp16 `value` with fp32 locations and
weights (perf mode).  Put kinet_amd/ on sys.path (or import kinet_amd, which registers
this module under its bare name) to satisfy `import MultiScaleDeformableAttention`
in ms_deform_attn_func.py:11.
"""
import torch

from kinet_amd import _native as _n


def _dims(value, spatial_shapes, sampling_loc, attn_weight):
    if value.dim() != 4:
        raise RuntimeError(f'value must be (N, S, M, D), got {tuple(value.shape)}')
    N, S, M, D = value.shape
    if sampling_loc.dim() != 6 or sampling_loc.shape[-1] != 2:
        raise RuntimeError(f'sampling_loc must be (N, Lq, M, L, P, 2), got {tuple(sampling_loc.shape)}')
    _, Lq, M2, L, P, _ = sampling_loc.shape
    if sampling_loc.shape[0] != N or M2 != M:
        raise RuntimeError('sampling_loc batch/heads do not match value')
    if tuple(attn_weight.shape) != (N, Lq, M, L, P):
        raise RuntimeError(f'attn_weight must be {(N, Lq, M, L, P)}, got {tuple(attn_weight.shape)}')
    if tuple(spatial_shapes.shape) != (L, 2) or spatial_shapes.dtype != torch.int64:
        raise RuntimeError('spatial_shapes must be an int64 (L, 2) tensor')
    return N, S, M, D, L, Lq, P


def _loc_dtype_ok(value, t):
    if value.dtype in (torch.float32, torch.float64):
        return t.dtype == value.dtype
    return t.dtype == torch.float32


def _prep(value, spatial_shapes, sampling_loc, attn_weight):
    _n.require_gpu(value, spatial_shapes, sampling_loc, attn_weight)
    if not value.is_contiguous():
        raise RuntimeError('value tensor has to be contiguous')   # ms_deform_attn_cuda.cu:29
    if not (_loc_dtype_ok(value, sampling_loc) and _loc_dtype_ok(value, attn_weight)):
        raise RuntimeError(f'unsupported dtypes value={value.dtype} loc={sampling_loc.dtype} '
                           f'attw={attn_weight.dtype}')
    return (spatial_shapes.contiguous(), sampling_loc.contiguous(), attn_weight.contiguous())


def ms_deform_attn_forward(value, spatial_shapes, sampling_loc, attn_weight, im2col_step):
    N, S, M, D, L, Lq, P = _dims(value, spatial_shapes, sampling_loc, attn_weight)
    spatial_shapes, sampling_loc, attn_weight = _prep(value, spatial_shapes, sampling_loc, attn_weight)
    out = torch.empty((N, Lq, M * D), dtype=value.dtype, device=value.device)
    _n.call('kinet_msda_forward', _n.ptr(value), _n.ptr(spatial_shapes), _n.ptr(sampling_loc),
            _n.ptr(attn_weight), _n.ptr(out), N, S, M, D, L, Lq, P, int(im2col_step),
            _n.dtype_code(value.dtype), _n.dtype_code(sampling_loc.dtype), _n.stream(value.device))
    return out


def ms_deform_attn_backward(value, spatial_shapes, sampling_loc, attn_weight, grad_output, im2col_step):
    N, S, M, D, L, Lq, P = _dims(value, spatial_shapes, sampling_loc, attn_weight)
    spatial_shapes, sampling_loc, attn_weight = _prep(value, spatial_shapes, sampling_loc, attn_weight)
    _n.require_gpu(grad_output)
    grad_output = grad_output.to(value.dtype).contiguous()
    if grad_output.numel() != N * Lq * M * D:
        raise RuntimeError('grad_output must have N*Lq*M*D elements')
    grad_value = torch.empty_like(value)
    grad_loc = torch.empty_like(sampling_loc)
    grad_attw = torch.empty_like(attn_weight)
    ws_bytes = _n.lib().kinet_msda_backward_workspace_bytes(N, S, M, D, _n.dtype_code(value.dtype))
    ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=value.device) if ws_bytes else None
    work = {'family': 'msda_bwd', 'Lq': Lq, 'S': S,
            # SURVEY 8(d) B_bwd: value + grad_out + loc/attw + f32 grad_value + grad loc/attw
            'bytes': (N * S * M * D * value.element_size() + N * Lq * M * D * grad_output.element_size()
                      + 12 * N * Lq * M * L * P + 4 * N * S * M * D + 12 * N * Lq * M * L * P)}
    _n.call('kinet_msda_backward', _n.ptr(value), _n.ptr(spatial_shapes), _n.ptr(sampling_loc),
            _n.ptr(attn_weight), _n.ptr(grad_output), _n.ptr(grad_value), _n.ptr(grad_loc),
            _n.ptr(grad_attw), _n.ptr(ws), N, S, M, D, L, Lq, P, int(im2col_step),
            _n.dtype_code(value.dtype), _n.dtype_code(sampling_loc.dtype), _n.stream(value.device), work=work)
    # the launcher's own choice (csrc/msda.hip): the list kernel sums grad_value rows on chip
    work['kernel'] = {1: 'msda_bwd_list_kernel', 0: 'msda_bwd_kernel'}.get(
        _n.lib().kinet_msda_backward_last_kernel(), 'none')
    return [grad_value, grad_loc, grad_attw]

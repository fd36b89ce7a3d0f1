"""ctypes binding of the kinet_amd C-ABI (include/*.h) -> kinet_amd/_lib/libkinet_amd.so.

There is deliberately NO fallback: if the library is missing or fails to load, every
op raises.  (The reference behaves the same way -- MultiScaleDeformableAttention is
imported at module import time, ms_deform_attn_func.py:11, and its CPU branch is an
AT_ERROR, ms_deform_attn.h:27.)
"""
import ctypes
import os

import torch

# KINET_AMD_LIB: an alternative build of the same sources (A/B tooling only)
_LIB_PATH = os.environ.get('KINET_AMD_LIB') or os.path.join(os.path.dirname(os.path.abspath(__file__)), '_lib', 'libkinet_amd.so')

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
F = ctypes.c_float

# symbol -> argtypes (restype int unless listed in _RESTYPES)
_SIGS = {
    'kinet_msda_forward': [P, P, P, P, P] + [I] * 10 + [P],
    'kinet_msda_backward': [P] * 9 + [I] * 10 + [P],
    'kinet_msda_backward_workspace_bytes': [I] * 5,
    'kinet_msda_backward_tune': [I] * 5,
    'kinet_msda_backward_debug': [I],
    'kinet_msda_backward_last_kernel': [],
    'kinet_msda_encoder_forward': [P, I64, I64, P, P, P, I, P, P] + [I] * 8 + [P, P],
    'kinet_msda_encoder_plan': [P, I, I, I, P],
    'kinet_msda_encoder_set_strips': [I],
    'kinet_msda_encoder_plan_ex': [P, I, I, I, I, P],
    'kinet_msda_encoder_forward_split': [P, I64, I64, P, I64, I64, P, P, P, I, P, P] + [I] * 8 + [P, P],
    'kinet_msda_sample_records': [P, P, P, P, I, I, I, I, I, P, I, P, P, I, I, I, P, I, P],
    'kinet_msda_encoder_forward_records': [P, I64, I64, P, P, I, P] + [I] * 8 + [P, P],
    'kinet_msda_fused_forward': [P, I64, I64, I64, P, P, I, P, I, P, P, P, P] + [I] * 10 + [P, P],
    'kinet_gemm_set_flags': [I],
    'kinet_set_solo_launch': [I],
    'kinet_gemm_force_tile': [I, I],
    'kinet_gemm_headmajor': [P, P, P] + [I] * 7 + [P, P, I, I, P],
    'kinet_gemm_headmajor_ex': [P, P, P, P] + [I] * 7 + [P, P, I, I, I, P],
    'kinet_gemm_headmajor_split': [P, P, P] + [I] * 7 + [P, P, I, I, I, I, P],
    'kinet_gemm': [P, P, P] + [I] * 7 + [P, P, P, I, I, I, P, I, P],
    'kinet_gemm_ex': [P, P, P, P] + [I] * 7 + [P, P, P, I, I, P, P, F, I, P, P],
    'kinet_conv2d': [P, P, P] + [I] * 12 + [P, P, P, I, I, I, P],
    'kinet_conv2d_ex': [P, P, P] + [I] * 14 + [P, P, P, I, I, I, P],
    'kinet_conv2d_splitk': [P, P, P] + [I] * 12 + [P, P, P, I, I, I, P, I, P],
    'kinet_gemm_splitk': [P, P, P] + [I] * 7 + [P, P, P, I, I, P, P, F, I, P, P, I, P],
    'kinet_ffn_pack': [P, P, P, I, I, I, P],
    'kinet_ffn_set_debug': [I],
    'kinet_ffn_fused': [P, I, P, P, P, P, P, F, P, I, I, I, I, I, P],
    'kinet_stem_conv_image': [P, P, P, P, P, I, I, I, I, P],
    'kinet_bottleneck_pack': [P, P, P, P, P, I, I, I, I, P],
    'kinet_bottleneck_pair': [P, I, P, P, P, P, P, P, I, I, I, I, I, P],
    'kinet_layernorm': [P] * 5 + [I, I, F, I, I, P],
    'kinet_groupnorm': [P] * 4 + [I] * 5 + [F, I, P, P],
    'kinet_groupnorm_workspace': [I] * 5,
    'kinet_maxpool2d_3x3s2': [P, P] + [I] * 5 + [P],
    'kinet_pack_image_nhwc': [P, P] + [I] * 5 + [P],
    'kinet_pack_image_kwfold': [P, P] + [I] * 8 + [P],
    'kinet_mha_set_mfma': [I],
    'kinet_mha_core': [P, I, P, I, P, I, P, I] + [I] * 5 + [F, I, P, P],
    'kinet_add': [P, P, P, I64, I, P],
    'kinet_box_refine': [P, P, I, P, P, P, I, I, I, P],
    'kinet_nms': [P, P, P, I, F, P],
    'kinet_sine_position_embed': [P, P, P, P] + [I] * 8 + [F, I64, I, P],
    'kinet_transpose': [P, P, I, I, I64, I64, I, P],
    'kinet_im2col_nhwc': [P, P] + [I] * 13 + [P],
    'kinet_col2im_nhwc': [P, P] + [I] * 13 + [P],
    'kinet_gemm_tn_workspace': [I, I, I],
    'kinet_gemm_tn': [P, P, P, I, I, I, I64, I64, I64, I, I, P, P],
    'kinet_colsum_workspace': [I, I],
    'kinet_colsum': [P, P, I, I, I64, I, I, P, P],
    'kinet_layernorm_backward_workspace': [I, I],
    'kinet_layernorm_backward': [P, P, P, P, P, P, I, I, F, I, P, P],
    'kinet_groupnorm_backward_workspace': [I, I, I, I],
    'kinet_groupnorm_backward': [P, P, P, P, P, P, I, I, I, I, F, I, P, P],
    'kinet_mha_backward_workspace': [I, I, I, I],
    'kinet_mha_backward': [P, I, P, I, P, I, P, I, P, P, P, I, I, I, I, I, F, P, P, F, P, P],
    'kinet_mha_core_dropout': [P, I, P, I, P, I, P, I] + [I] * 5 + [F, I, P, F, P, P],
    'kinet_dropout_mask': [P, I64, F, P, P],
    'kinet_dropout_add_layernorm': [P] * 5 + [I, I, F, F, P, P],
    'kinet_dropout_add_layernorm_backward_workspace': [I, I],
    'kinet_dropout_add_layernorm_backward': [P] * 8 + [I, I, F, F, P, P, P],
    'kinet_dropout_act': [P, P, I64, I, F, P, P],
    'kinet_dropout_act_backward': [P, P, P, I64, I, F, P, P],
    'kinet_msda_prep': [P, I64] + [P] * 5 + [I64, I, I, I, I, P],
    'kinet_msda_prep_backward': [P] * 4 + [I64] + [P] * 4 + [I64, I, I, I, I, P],
    'kinet_inverse_sigmoid': [P, P, I64, F, P],
    'kinet_inverse_sigmoid_backward': [P, P, P, I64, F, P],
    'kinet_last_error': [],
    'kinet_version': [],
}
_RESTYPES = {'kinet_last_error': ctypes.c_char_p, 'kinet_version': ctypes.c_char_p,
             'kinet_msda_backward_workspace_bytes': ctypes.c_int64, 'kinet_msda_backward_tune': None,
             'kinet_groupnorm_workspace': ctypes.c_long,
             'kinet_gemm_tn_workspace': ctypes.c_int64, 'kinet_colsum_workspace': ctypes.c_int64,
             'kinet_layernorm_backward_workspace': ctypes.c_int64,
             'kinet_dropout_add_layernorm_backward_workspace': ctypes.c_int64,
             'kinet_groupnorm_backward_workspace': ctypes.c_int64,
             'kinet_mha_backward_workspace': ctypes.c_int64}

DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3}

_lib = None
_load_error = None


def lib():
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise RuntimeError(f'kinet_amd native library not built: {_LIB_PATH} missing '
                           f'(run `python -m kinet_amd.build`)')
    try:
        L = ctypes.CDLL(_LIB_PATH)
    except OSError as e:   # pragma: no cover
        _load_error = e
        raise RuntimeError(f'failed to load {_LIB_PATH}: {e}') from e
    for name, args in _SIGS.items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    _lib = L
    return L


def exported(name):
    return hasattr(lib(), name)


_trace = None   # list of (name, work dict, start event, end event) while tracing


def trace_begin():
    """Record a HIP event pair around every subsequent launch (bench.py roofline pass)."""
    global _trace
    _trace = []


def trace_end():
    global _trace
    t, _trace = _trace, None
    return t


_fns = {}


def call(name, *args, work=None):
    """Invoke a C-ABI entry point and raise RuntimeError on a non-zero status.
    `work` ({'flops': .., 'bytes': ..}) annotates the launch for the tracer."""
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(lib(), name)
    if _trace is not None:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = fn(*args)
        e.record()
        _trace.append((name, work or {}, s, e))
    else:
        rc = fn(*args)
    if rc != 0:
        msg = lib().kinet_last_error().decode(errors='replace')
        raise RuntimeError(f'{name}: {msg}')
    return rc


def ptr(t):
    # c_void_p argtypes take plain ints: no ctypes object per pointer argument
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, '_cuda_getCurrentRawStream', None)


def stream(device=None):
    """The current HIP stream of `device` as an int handle (the caller's stream, as
    at::cuda::getCurrentCUDAStream() in the reference)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        else:
            idx = device.index if isinstance(device, torch.device) else int(device)
            if idx is None:
                idx = torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(dt):
    try:
        return DT[dt]
    except KeyError:
        raise RuntimeError(f'kinet_amd: unsupported dtype {dt}') from None


def require_gpu(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            # reference: AT_ASSERTM(value.type().is_cuda(), ...) (ms_deform_attn_cuda.cu:31-34)
            raise RuntimeError('kinet_amd ops run on the GPU only: got a CPU tensor '
                               '(the reference CPU branch is AT_ERROR too, ms_deform_attn.h:27)')

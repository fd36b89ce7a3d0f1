"""Operator + module surface of multi-scale deformable attention, mirroring
src/trackformer/models/ops/functions/ms_deform_attn_func.py and
src/trackformer/models/ops/modules/ms_deform_attn.py.

`MSDeformAttnFunction.apply(value, value_spatial_shapes, sampling_locations,
attention_weights, im2col_step)` is the reference operator boundary
(ms_deform_attn_func.py:14-31); `MSDeformAttn` keeps the reference parameter names
(sampling_offsets / attention_weights / value_proj / output_proj, ms_deform_attn.py:27-30)
so reference state_dicts load unchanged.
"""
import torch
from torch import nn
from torch.autograd import Function
from torch.autograd.function import once_differentiable
from torch.nn.init import constant_, xavier_uniform_

from kinet_amd import MultiScaleDeformableAttention as MSDA
from kinet_amd import autograd as A
from kinet_amd import kernels as K


def value_dtype_for(compute_dtype):
    """Storage dtype of projected MSDA values: f16 under bf16 compute (see project_value)."""
    return torch.float16 if compute_dtype == torch.bfloat16 else compute_dtype


class MSDeformAttnFunction(Function):
    """ms_deform_attn_func.py:14-31 -- same forward/backward contract."""

    @staticmethod
    def forward(ctx, value, value_spatial_shapes, sampling_locations, attention_weights, im2col_step):
        ctx.im2col_step = im2col_step
        output = MSDA.ms_deform_attn_forward(value, value_spatial_shapes, sampling_locations,
                                             attention_weights, ctx.im2col_step)
        ctx.save_for_backward(value, value_spatial_shapes, sampling_locations, attention_weights)
        return output

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        value, value_spatial_shapes, sampling_locations, attention_weights = ctx.saved_tensors
        grad_value, grad_sampling_loc, grad_attn_weight = MSDA.ms_deform_attn_backward(
            value, value_spatial_shapes, sampling_locations, attention_weights, grad_output, ctx.im2col_step)
        return grad_value, None, grad_sampling_loc, grad_attn_weight, None


class MSDeformAttn(nn.Module):
    """ms_deform_attn.py:15-89.  Inference runs the fused HIP path (one GEMM for
    value_proj with the padding mask in its epilogue, one GEMM for the concatenated
    sampling_offsets | attention_weights projection, the fused softmax/location/sampling
    kernel, and output_proj); with autograd enabled it runs the unfused reference
    sequence through MSDeformAttnFunction so gradients flow exactly as upstream."""

    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4, im2col_step=64):
        super().__init__()
        if d_model % n_heads != 0:
            raise ValueError('d_model must be divisible by n_heads, but got {} and {}'.format(d_model, n_heads))
        self.im2col_step = im2col_step
        self.d_model = d_model
        self.n_levels = n_levels
        self.n_heads = n_heads
        self.n_points = n_points
        self.sampling_offsets = nn.Linear(d_model, n_heads * n_levels * n_points * 2)
        self.attention_weights = nn.Linear(d_model, n_heads * n_levels * n_points)
        self.value_proj = nn.Linear(d_model, d_model)
        self.output_proj = nn.Linear(d_model, d_model)
        self._reset_parameters()
        self._packed = None

    def _reset_parameters(self):
        # ms_deform_attn.py:34-47
        constant_(self.sampling_offsets.weight.data, 0.)
        # the reference's fixed 8-direction table (ms_deform_attn.py:36-37; n_heads must be 8)
        grid_init = torch.tensor([-1, -1, -1, 0, -1, 1, 0, -1, 0, 1, 1, -1, 1, 0, 1, 1], dtype=torch.float32) \
            .view(self.n_heads, 1, 1, 2).repeat(1, self.n_levels, self.n_points, 1)
        for i in range(self.n_points):
            grid_init[:, :, i, :] *= i + 1
        with torch.no_grad():
            self.sampling_offsets.bias = nn.Parameter(grid_init.view(-1))
        constant_(self.attention_weights.weight.data, 0.)
        constant_(self.attention_weights.bias.data, 0.)
        xavier_uniform_(self.value_proj.weight.data)
        constant_(self.value_proj.bias.data, 0.)
        xavier_uniform_(self.output_proj.weight.data)
        constant_(self.output_proj.bias.data, 0.)

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes,
                input_padding_mask=None, query_attn_mask=None):
        N, Len_q, _ = query.shape
        N, Len_in, _ = input_flatten.shape
        # autograd whenever grad mode is on (frozen parameters still need input gradients,
        # as upstream's module is differentiable w.r.t. query / input_flatten / refs)
        if torch.is_grad_enabled():
            return self._forward_autograd(query, reference_points, input_flatten, input_spatial_shapes,
                                          input_padding_mask, query_attn_mask)
        value = self.project_value(input_flatten, input_padding_mask)
        out = self.sample(query, reference_points, value, input_spatial_shapes, query_attn_mask)
        return K.linear(out, self.output_proj.weight, self.output_proj.bias)

    def project_value(self, input_flatten, input_padding_mask=None, encoder_shapes=None):
        """value_proj + padding masked_fill (ms_deform_attn.py:64-66), written head-major
        (M, N, S, D) for the gather kernel; bf16 compute stores the values as f16 (more
        mantissa, and the sampling kernel's mixed f16 x f32 FMA reads them directly).
        encoder_shapes (host level shapes of an encoder call, Lq = S): a head_dim-36 layer then
        writes the two planes of the split strip kernel (K.SplitValue)."""
        D = self.d_model // self.n_heads
        if encoder_shapes is not None and K.msda_split_supported(
                input_flatten.dtype, D, encoder_shapes, input_flatten.shape[1], self.n_heads, self.n_levels,
                self.n_points, input_flatten.shape[0]):
            w, b = K.split_value_weights(self.value_proj.weight, self.value_proj.bias, self.n_heads)
            return K.value_proj_headmajor_split(input_flatten, w, b, self.n_heads, row_mask=input_padding_mask,
                                                out_dtype=value_dtype_for(input_flatten.dtype))
        return K.value_proj_headmajor(input_flatten, self.value_proj.weight, self.value_proj.bias,
                                      self.d_model // self.n_heads, row_mask=input_padding_mask,
                                      out_dtype=value_dtype_for(input_flatten.dtype))

    # -- pieces used by the fused transformer layers ------------------------------------
    def packed_offsets_weights(self):
        """[sampling_offsets ; attention_weights] stacked into one (M*L*P*3, d) GEMM."""
        so, aw = self.sampling_offsets, self.attention_weights
        w = K.cached_multi([so.weight, aw.weight], 'packed_w',
                           lambda a, b: torch.cat([a.detach(), b.detach()], 0).contiguous())
        b = K.cached_multi([so.bias, aw.bias], 'packed_b',
                           lambda a, b: torch.cat([a.detach(), b.detach()], 0).float().contiguous())
        return w, b

    def packed_offsets_weights_headmajor(self):
        """The same projection with its rows grouped per head -- head m's L*P*2 offset rows,
        then its L*P logit rows -- so a head-major store of the GEMM output is the
        (M, N, Lq, L*P*3) layout kinet_msda_encoder_forward reads."""
        so, aw = self.sampling_offsets, self.attention_weights
        M, LP = self.n_heads, self.n_levels * self.n_points

        def interleave(a, b):
            return torch.cat([a.detach().view(M, 2 * LP, *a.shape[1:]), b.detach().view(M, LP, *b.shape[1:])],
                             1).reshape(M * 3 * LP, *a.shape[1:])
        w = K.cached_multi([so.weight, aw.weight], 'packed_w_hm', lambda a, b: interleave(a, b).contiguous())
        b = K.cached_multi([so.bias, aw.bias], 'packed_b_hm', lambda a, b: interleave(a, b).float().contiguous())
        return w, b

    def packed_records_weights(self):
        """The same projection with its rows grouped per (head, level) -- the level's 4 points'
        (x, y) offset rows, then its 4 logit rows (12 rows) -- the layout whose GEMM epilogue
        writes the sampling records (kinet_msda_sample_records)."""
        so, aw = self.sampling_offsets, self.attention_weights
        M, L, P = self.n_heads, self.n_levels, self.n_points

        def group(a, b):
            return torch.cat([a.detach().view(M, L, 2 * P, *a.shape[1:]), b.detach().view(M, L, P, *b.shape[1:])],
                             2).reshape(M * L * 3 * P, *a.shape[1:])
        w = K.cached_multi([so.weight, aw.weight], 'packed_w_rec', lambda a, b: group(a, b).contiguous())
        b = K.cached_multi([so.bias, aw.bias], 'packed_b_rec', lambda a, b: group(a, b).float().contiguous())
        return w, b

    def sample(self, query, reference_points, value, input_spatial_shapes, query_attn_mask=None, query_add=None,
               query_order=None, shapes_host=None):
        """value already projected: head-major (M, N, S, D) from project_value (or a
        row-major (N, S, d) tensor); the offsets/weights projection input is query
        (+ query_add, e.g. the position embedding, added at GEMM load time); returns the
        pre-output_proj (N, Lq, d).  shapes_host: the level shapes as a host list (lets an
        encoder-sized call take kinet_msda_encoder_forward)."""
        N_, Lq = query.shape[:2]
        if isinstance(value, K.SplitValue):
            # head_dim 36 on the strip kernel (value planes from project_value(encoder_shapes=...))
            w, b = self.packed_offsets_weights_headmajor()
            offlog = K.offsets_proj_headmajor(query, w, b, self.n_heads, x_add=query_add)
            return K.msda_encoder_split(value, shapes_host, offlog, reference_points, self.n_heads, query_attn_mask,
                                        out_dtype=query.dtype, query_tile_order=query_order)
        if (query.dtype in (torch.bfloat16, torch.float16) and
                K.msda_encoder_supported(value, shapes_host, Lq, self.n_heads, self.n_levels, self.n_points, N_)):
            if K.msda_records_supported(query, shapes_host, self.n_heads, self.n_levels, self.n_points):
                # phase 1 (softmax, locations, bilinear setup) in the projection's epilogue
                w, b = self.packed_records_weights()
                rec, fb = K.msda_sample_records(query, w, b, self.n_heads, reference_points, shapes_host,
                                                x_add=query_add, query_attn_mask=query_attn_mask)
                return K.msda_encoder_records(value, shapes_host, rec, fb, out_dtype=query.dtype,
                                              query_tile_order=query_order)
            w, b = self.packed_offsets_weights_headmajor()
            offlog = K.offsets_proj_headmajor(query, w, b, self.n_heads, x_add=query_add)
            return K.msda_encoder(value, shapes_host, offlog, reference_points, self.n_heads, query_attn_mask,
                                  out_dtype=query.dtype, query_tile_order=query_order)
        w, b = self.packed_offsets_weights()
        # bf16 compute: offsets/logits in f16 (half the bytes of f32 through HBM twice; f16
        # keeps 11 mantissa bits for the pixel offsets); parity mode stays f32.  The f16 offsets
        # and the bf16-from-f16 output are the head_dim-32 fast kernel's; other head dims (36)
        # run the generic kernel on f32 offsets with the values' own output dtype
        fast = self.d_model // self.n_heads == 32
        od = torch.float16 if query.dtype == torch.bfloat16 and fast else torch.float32
        offlog = K.linear(query, w, b, out_dtype=od, x_add=query_add)
        out = K.msda_fused(value, input_spatial_shapes, offlog, reference_points,
                           self.n_heads, self.n_levels, self.n_points, query_attn_mask,
                           head_major=(value.dim() == 4), out_dtype=query.dtype if fast else value.dtype,
                           query_tile_order=query_order)
        return out if out.dtype == query.dtype else out.to(query.dtype)

    def _forward_autograd(self, query, reference_points, input_flatten, input_spatial_shapes,
                          input_padding_mask, query_attn_mask):
        # ms_deform_attn.py:64-88
        N, Len_q, _ = query.shape
        N, Len_in, _ = input_flatten.shape
        value = A.linear_module(input_flatten, self.value_proj)
        if input_padding_mask is not None:
            value = value.masked_fill(input_padding_mask[..., None], float(0))
        value = value.view(N, Len_in, self.n_heads, self.d_model // self.n_heads)
        if reference_points.shape[-1] not in (2, 4):
            raise ValueError('Last dim of reference_points must be 2 or 4, but get {} instead.'
                             .format(reference_points.shape[-1]))
        # :67-82 (softmax over L*P, query mask, locations from the reference points) in one
        # kernel each way (kinet_msda_prep)
        # ONE projection GEMM over [sampling_offsets ; attention_weights] (one input-gradient GEMM
        # in the backward instead of two plus the add of their results)
        so, aw = self.sampling_offsets, self.attention_weights
        offlog = A.linear(query, torch.cat([so.weight, aw.weight], 0), torch.cat([so.bias, aw.bias], 0))
        sampling_locations, attention_weights = A.msda_prep(
            offlog, reference_points, input_spatial_shapes, query_attn_mask, self.n_heads, self.n_levels,
            self.n_points)
        output = MSDeformAttnFunction.apply(value, input_spatial_shapes, sampling_locations,
                                            attention_weights, self.im2col_step)
        return A.linear_module(output, self.output_proj)

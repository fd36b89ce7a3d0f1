"""Deformable-DETR encoder/decoder on the kinet_amd kernels.

Mirrors src/trackformer/models/deformable_transformer.py (DeformableTransformer :21-257,
encoder layer :260-299, encoder :302-330, decoder layer :333-386, decoder :389-434,
build_deforamble_transformer :437-457) with the same module/parameter names.

Two execution paths with identical arithmetic:
  * inference (autograd disabled) -- every op is a HIP kernel: value_proj GEMM with the
    padding mask in its epilogue, ONE GEMM for the concatenated sampling_offsets |
    attention_weights projection (f32 out), the fused softmax/location/sampling MSDA
    kernel, output_proj GEMM with the residual add in its epilogue, LayerNorm kernel,
    FFN as two GEMMs (ReLU / residual fused), decoder self-attention as in_proj GEMMs +
    the MHA kernel, and box refinement as one small kernel.  Activations stay in the
    compute dtype (bf16 perf mode, f32 parity mode) in (batch, tokens, channels) layout.
  * training (autograd enabled) -- the reference's op sequence, op for op, on kinet_amd
    autograd Functions (kinet_amd/autograd.py: Linear, LayerNorm, attention core with its
    probability dropout, ...; forward and backward HIP kernels) with MSDeformAttnFunction
    (HIP forward / backward) at the operator boundary; torch supplies only glue (dropout
    masks outside attention, adds, reshapes).
Reference quirks kept on purpose: 2-d sampling offsets divided by
(H, W) applied to (x, y); multi-frame memory concatenated [current, prev] while shapes,
masks and valid ratios stay [prev, current].
"""
import copy

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.init import constant_, normal_, xavier_uniform_

from kinet_amd import autograd as A
from kinet_amd import kernels as K
from kinet_amd.models.misc import host_to_device, inverse_sigmoid
from kinet_amd.msda import MSDeformAttn, value_dtype_for


def _get_clones(module, N):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def _get_activation_fn(activation):
    if activation == "relu":
        return F.relu
    if activation == "gelu":
        return F.gelu
    if activation == "glu":
        return F.glu
    raise RuntimeError(F"activation should be relu/gelu, not {activation}.")


_FORCE_REFERENCE = [0]


def _active_dropout(module):
    return module.training and any(isinstance(m, (nn.Dropout, nn.MultiheadAttention)) and
                                   getattr(m, 'p', getattr(m, 'dropout', 0.0)) > 0 for m in module.modules())


def fast_path(module=None):
    """HIP inference path: no autograd, not inside reference_path(), and -- when `module`
    is given -- no dropout that train mode would apply (a train-mode module under no_grad
    must still drop activations as the reference does)."""
    if torch.is_grad_enabled() or _FORCE_REFERENCE[0]:
        return False
    return module is None or not _active_dropout(module)


class reference_path:
    """Run the op-for-op module path even without grad (e.g. the no-grad previous-frame
    pass of training, which the reference runs in train mode -- with dropout)."""

    def __enter__(self):
        _FORCE_REFERENCE[0] += 1

    def __exit__(self, *exc):
        _FORCE_REFERENCE[0] -= 1


class DeformableTransformerEncoderLayer(nn.Module):
    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        if activation != 'relu':
            raise NotImplementedError('only relu FFNs are on the configured hot path')
        self.self_attn = MSDeformAttn(d_model, n_levels, n_heads, n_points)
        self.dropout1 = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.linear1 = nn.Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation)
        self.dropout2 = nn.Dropout(dropout)
        self.linear2 = nn.Linear(d_ffn, d_model)
        self.dropout3 = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(d_model)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, src):
        # linear2(dropout2(relu(linear1(src)))), norm2(src + dropout3(src2)): the dropout / relu /
        # residual / LayerNorm glue in one kernel each way (csrc/train_ops.hip)
        src2 = A.linear_module(A.dropout_act(A.linear_module(src, self.linear1), self.dropout2), self.linear2)
        return A.dropout_add_layer_norm(src, src2, self.norm2, self.dropout3)

    def forward(self, src, pos, reference_points, spatial_shapes, padding_mask=None, query_order=None,
                shapes_host=None):
        if fast_path(self):
            return self.forward_fast(src, pos, reference_points, spatial_shapes, padding_mask, query_order,
                                     shapes_host)
        src2 = self.self_attn(self.with_pos_embed(src, pos), reference_points, src, spatial_shapes, padding_mask)
        src = A.dropout_add_layer_norm(src, src2, self.norm1, self.dropout1)
        return self.forward_ffn(src)

    def forward_fast(self, src, pos, reference_points, spatial_shapes, padding_mask=None, query_order=None,
                     shapes_host=None):
        # deformable_transformer.py:290-299, one kernel per step
        a = self.self_attn
        value = a.project_value(src, padding_mask, encoder_shapes=shapes_host)         # head-major
        samp = a.sample(src, reference_points, value, spatial_shapes, query_add=pos,   # (src+pos) @ W
                        query_order=query_order, shapes_host=shapes_host)
        n1, n2 = self.norm1, self.norm2
        src = K.linear(samp, a.output_proj.weight, a.output_proj.bias, residual=src, ln=(n1.weight, n1.bias, n1.eps))
        if K.ffn_supported(src, self.linear1, self.linear2):
            return K.ffn_fused(src, self.linear1, self.linear2, n2)
        h = K.linear(src, self.linear1.weight, self.linear1.bias, relu=True)
        return K.linear(h, self.linear2.weight, self.linear2.bias, residual=src, ln=(n2.weight, n2.bias, n2.eps))


class DeformableTransformerEncoder(nn.Module):
    def __init__(self, encoder_layer, num_layers):
        super().__init__()
        self.layers = _get_clones(encoder_layer, num_layers)
        self.num_layers = num_layers

    @staticmethod
    def get_reference_points(spatial_shapes, valid_ratios, device):
        """deformable_transformer.py:309-321: pixel centres normalised by the valid extent."""
        reference_points_list = []
        for lvl, (H_, W_) in enumerate(spatial_shapes):
            H_, W_ = int(H_), int(W_)
            ref_y, ref_x = torch.meshgrid(torch.linspace(0.5, H_ - 0.5, H_, dtype=torch.float32, device=device),
                                          torch.linspace(0.5, W_ - 0.5, W_, dtype=torch.float32, device=device),
                                          indexing='ij')
            ref_y = ref_y.reshape(-1)[None] / (valid_ratios[:, None, lvl, 1] * H_)
            ref_x = ref_x.reshape(-1)[None] / (valid_ratios[:, None, lvl, 0] * W_)
            reference_points_list.append(torch.stack((ref_x, ref_y), -1))
        reference_points = torch.cat(reference_points_list, 1)
        return reference_points[:, :, None] * valid_ratios[:, None]

    def forward(self, src, spatial_shapes, valid_ratios, pos=None, padding_mask=None, reference_points=None,
                query_order=None, shapes_host=None):
        output = src
        if reference_points is None:
            shapes = spatial_shapes.tolist() if torch.is_tensor(spatial_shapes) else spatial_shapes
            shapes_host = shapes_host or [tuple(int(v) for v in s) for s in shapes]
            reference_points = self.get_reference_points(shapes, valid_ratios, device=src.device)
        if not torch.is_tensor(spatial_shapes):
            spatial_shapes = host_to_device(spatial_shapes, torch.long, src.device)
        for layer in self.layers:
            output = layer(output, pos, reference_points, spatial_shapes, padding_mask, query_order=query_order,
                           shapes_host=shapes_host)
        return output


class DeformableTransformerDecoderLayer(nn.Module):
    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        if activation != 'relu':
            raise NotImplementedError('only relu FFNs are on the configured hot path')
        self.cross_attn = MSDeformAttn(d_model, n_levels, n_heads, n_points)
        self.dropout1 = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.self_attn = nn.MultiheadAttention(d_model, n_heads, dropout=dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(d_model)
        self.linear1 = nn.Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation)
        self.dropout3 = nn.Dropout(dropout)
        self.linear2 = nn.Linear(d_ffn, d_model)
        self.dropout4 = nn.Dropout(dropout)
        self.norm3 = nn.LayerNorm(d_model)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, tgt):
        tgt2 = A.linear_module(A.dropout_act(A.linear_module(tgt, self.linear1), self.dropout3), self.linear2)
        return A.dropout_add_layer_norm(tgt, tgt2, self.norm3, self.dropout4)

    def forward(self, tgt, query_pos, reference_points, src, src_spatial_shapes, src_padding_mask=None,
                query_attn_mask=None, value=None, out=None):
        if fast_path(self):
            return self.forward_fast(tgt, query_pos, reference_points, src, src_spatial_shapes, src_padding_mask,
                                     query_attn_mask, value, out)
        q = k = self.with_pos_embed(tgt, query_pos)
        # nn.MultiheadAttention on (L, B, E) transposes (:371) == the batch-first kinet path
        tgt2 = A.multihead_attention(self.self_attn, q, k, tgt, key_padding_mask=query_attn_mask)
        tgt = A.dropout_add_layer_norm(tgt, tgt2, self.norm2, self.dropout2)
        tgt2 = self.cross_attn(self.with_pos_embed(tgt, query_pos), reference_points, src, src_spatial_shapes,
                               src_padding_mask, query_attn_mask)
        tgt = A.dropout_add_layer_norm(tgt, tgt2, self.norm1, self.dropout1)
        return self.forward_ffn(tgt)

    def forward_fast(self, tgt, query_pos, reference_points, src, src_spatial_shapes, src_padding_mask=None,
                     query_attn_mask=None, value=None, out=None):
        # deformable_transformer.py:367-386
        d = tgt.shape[-1]
        sa = self.self_attn
        n1, n2, n3 = self.norm1, self.norm2, self.norm3
        qk = K.linear(tgt, K.param_rows(sa.in_proj_weight, 0, 2 * d), K.param_rows(sa.in_proj_bias, 0, 2 * d),
                      x_add=query_pos)                                            # q = k = tgt + query_pos
        v = K.linear(tgt, K.param_rows(sa.in_proj_weight, 2 * d, 3 * d), K.param_rows(sa.in_proj_bias, 2 * d, 3 * d))
        attn = K.mha_core(qk[..., :d], qk[..., d:], v, sa.num_heads, sa.head_dim ** -0.5, key_mask=query_attn_mask)
        tgt = K.linear(attn, sa.out_proj.weight, sa.out_proj.bias, residual=tgt, ln=(n2.weight, n2.bias, n2.eps))
        ca = self.cross_attn
        if value is None:
            value = ca.project_value(src, src_padding_mask)
        samp = ca.sample(tgt, reference_points, value, src_spatial_shapes, query_attn_mask, query_add=query_pos)
        tgt = K.linear(samp, ca.output_proj.weight, ca.output_proj.bias, residual=tgt, ln=(n1.weight, n1.bias, n1.eps))
        out2 = None if out is None else out.view(-1, out.shape[-1])
        if K.ffn_supported(tgt, self.linear1, self.linear2):
            y = K.ffn_fused(tgt, self.linear1, self.linear2, n3, out=out2)
        else:
            h = K.linear(tgt, self.linear1.weight, self.linear1.bias, relu=True)
            y = K.linear(h, self.linear2.weight, self.linear2.bias, residual=tgt, ln=(n3.weight, n3.bias, n3.eps),
                         out=out2)
        return y if out is None else out


def mlp_fast(mlp, x, out_dtype=torch.float32):
    """detr.py:937-951 MLP (ReLU between layers) as chained GEMMs; last layer in out_dtype."""
    n = len(mlp.layers)
    for i, layer in enumerate(mlp.layers):
        last = i == n - 1
        x = K.linear(x, layer.weight, layer.bias, relu=not last, out_dtype=out_dtype if last else None)
    return x


class DeformableTransformerDecoder(nn.Module):
    def __init__(self, decoder_layer, num_layers, return_intermediate=False):
        super().__init__()
        self.layers = _get_clones(decoder_layer, num_layers)
        self.num_layers = num_layers
        self.return_intermediate = return_intermediate
        self.bbox_embed = None
        self.class_embed = None

    def forward(self, tgt, reference_points, src, src_spatial_shapes, src_valid_ratios,
                query_pos=None, src_padding_mask=None, query_attn_mask=None):
        if fast_path(self):
            return self.forward_fast(tgt, reference_points, src, src_spatial_shapes, src_valid_ratios,
                                     query_pos, src_padding_mask, query_attn_mask)
        output = tgt
        intermediate, intermediate_reference_points = [], []
        for lid, layer in enumerate(self.layers):
            if reference_points.shape[-1] == 4:
                reference_points_input = reference_points[:, :, None] \
                    * torch.cat([src_valid_ratios, src_valid_ratios], -1)[:, None]
            else:
                assert reference_points.shape[-1] == 2
                reference_points_input = reference_points[:, :, None] * src_valid_ratios[:, None]
            output = layer(output, query_pos, reference_points_input, src, src_spatial_shapes, src_padding_mask,
                           query_attn_mask)
            if self.bbox_embed is not None:
                tmp = self.bbox_embed[lid](output)
                if reference_points.shape[-1] == 4:
                    new_reference_points = (tmp + inverse_sigmoid(reference_points)).sigmoid()
                else:
                    new_reference_points = tmp
                    new_reference_points[..., :2] = tmp[..., :2] + inverse_sigmoid(reference_points)
                    new_reference_points = new_reference_points.sigmoid()
                reference_points = new_reference_points.detach()
            if self.return_intermediate:
                intermediate.append(output)
                intermediate_reference_points.append(reference_points)
        if self.return_intermediate:
            return torch.stack(intermediate), torch.stack(intermediate_reference_points)
        return output, reference_points

    def forward_fast(self, tgt, reference_points, src, src_spatial_shapes, src_valid_ratios,
                     query_pos=None, src_padding_mask=None, query_attn_mask=None):
        output = tgt
        reference_points = reference_points.float()
        vr = src_valid_ratios.float()
        if reference_points.shape[-1] == 4:
            ref_in = reference_points[:, :, None] * torch.cat([vr, vr], -1)[:, None]
        else:
            ref_in = reference_points[:, :, None] * vr[:, None]
        # every layer's cross-attention value_proj reads the same memory: run them as ONE
        # GEMM (S x d x n_layers*d) and hand each layer its column slice (read in place)
        d = tgt.shape[-1]
        nl = len(self.layers)
        vw = K.cached_multi([l.cross_attn.value_proj.weight for l in self.layers], 'dec_value_w',
                            lambda *ws: torch.cat([w.detach() for w in ws], 0).contiguous())
        vb = K.cached_multi([l.cross_attn.value_proj.bias for l in self.layers], 'dec_value_b',
                            lambda *bs: torch.cat([b.detach() for b in bs], 0).float().contiguous())
        ca0 = self.layers[0].cross_attn
        nh = ca0.n_heads
        values = K.value_proj_headmajor(src, vw, vb, d // nh, row_mask=src_padding_mask,
                                        out_dtype=value_dtype_for(src.dtype))                # (nl*M, B, S, D)
        # every layer writes its output / refined boxes straight into the stacked result
        # (the reference stacks the intermediates afterwards, :427-432)
        B, Q = tgt.shape[:2]
        hs_buf = torch.empty((nl, B, Q, d), dtype=tgt.dtype, device=tgt.device) if self.return_intermediate else None
        ref_buf = None
        if self.return_intermediate and self.bbox_embed is not None:
            ref_buf = torch.empty((nl, B, Q, 4), dtype=torch.float32, device=tgt.device)
        intermediate_reference_points = []
        for lid, layer in enumerate(self.layers):
            output = layer(output, query_pos, ref_in, src, src_spatial_shapes, src_padding_mask, query_attn_mask,
                           value=values[lid * nh:(lid + 1) * nh], out=None if hs_buf is None else hs_buf[lid])
            last = lid == nl - 1
            if self.bbox_embed is not None:
                tmp = mlp_fast(self.bbox_embed[lid], output)
                reference_points, nxt = K.box_refine(tmp, reference_points, vr, want_input=not last,
                                                     out=None if ref_buf is None else ref_buf[lid])
                if not last:
                    ref_in = nxt
            if self.return_intermediate:
                intermediate_reference_points.append(reference_points)
        if self.return_intermediate:
            refs = ref_buf if ref_buf is not None else torch.stack(intermediate_reference_points)
            return hs_buf, refs
        return output, reference_points


class DeformableTransformer(nn.Module):
    def __init__(self, d_model=256, nhead=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=1024,
                 dropout=0.1, activation="relu", return_intermediate_dec=False, num_feature_levels=4,
                 dec_n_points=4, enc_n_points=4, two_stage=False, two_stage_num_proposals=300,
                 multi_frame_attention_separate_encoder=False):
        super().__init__()
        if two_stage:
            raise NotImplementedError('two-stage Deformable DETR is not on the configured hot path '
                                      '(two_stage: false in every BASELINE config)')
        self.d_model = d_model
        self.nhead = nhead
        self.two_stage = two_stage
        self.two_stage_num_proposals = two_stage_num_proposals
        self.num_feature_levels = num_feature_levels
        self.multi_frame_attention_separate_encoder = multi_frame_attention_separate_encoder
        enc_levels = num_feature_levels // 2 if multi_frame_attention_separate_encoder else num_feature_levels
        encoder_layer = DeformableTransformerEncoderLayer(d_model, dim_feedforward, dropout, activation,
                                                          enc_levels, nhead, enc_n_points)
        self.encoder = DeformableTransformerEncoder(encoder_layer, num_encoder_layers)
        decoder_layer = DeformableTransformerDecoderLayer(d_model, dim_feedforward, dropout, activation,
                                                          num_feature_levels, nhead, dec_n_points)
        self.decoder = DeformableTransformerDecoder(decoder_layer, num_decoder_layers, return_intermediate_dec)
        self.level_embed = nn.Parameter(torch.Tensor(num_feature_levels, d_model))
        self.reference_points = nn.Linear(d_model, 2)
        self._reset_parameters()

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)
        for m in self.modules():
            if isinstance(m, MSDeformAttn):
                m._reset_parameters()
        xavier_uniform_(self.reference_points.weight.data, gain=1.0)
        constant_(self.reference_points.bias.data, 0.)
        normal_(self.level_embed)

    @staticmethod
    def get_valid_ratio(mask):
        """deformable_transformer.py:124-131."""
        _, H, W = mask.shape
        valid_H = torch.sum(~mask[:, :, 0], 1)
        valid_W = torch.sum(~mask[:, 0, :], 1)
        return torch.stack([valid_W.float() / W, valid_H.float() / H], -1)

    # ---------------------------------------------------------------------------------
    def prepare_inputs(self, srcs, masks, pos_embeds):
        """deformable_transformer.py:136-157 for NCHW inputs (reference call signature)."""
        src_flatten, mask_flatten, lvl_pos_embed_flatten, spatial_shapes = [], [], [], []
        for lvl, (src, mask, pos_embed) in enumerate(zip(srcs, masks, pos_embeds)):
            bs, c, h, w = src.shape
            spatial_shapes.append((h, w))
            src_flatten.append(src.flatten(2).transpose(1, 2))
            mask_flatten.append(mask.flatten(1))
            lvl_pos_embed_flatten.append(pos_embed.flatten(2).transpose(1, 2) + self.level_embed[lvl].view(1, 1, -1))
        src_flatten = torch.cat(src_flatten, 1)
        mask_flatten = torch.cat(mask_flatten, 1)
        lvl_pos_embed_flatten = torch.cat(lvl_pos_embed_flatten, 1)
        valid_ratios = torch.stack([self.get_valid_ratio(m) for m in masks], 1)
        return src_flatten, mask_flatten, lvl_pos_embed_flatten, spatial_shapes, valid_ratios

    def forward(self, srcs, masks, pos_embeds, query_embed=None, targets=None, padded=None):
        src_flatten, mask_flatten, lvl_pos, shapes, valid_ratios = self.prepare_inputs(srcs, masks, pos_embeds)
        if fast_path(self):
            dt = srcs[0].dtype
            src_flatten = src_flatten.to(dt).contiguous()
            lvl_pos = lvl_pos.to(dt).contiguous()
        geo = self.geometry(shapes, valid_ratios, mask_flatten, src_flatten.device, padded)
        return self.forward_flat(src_flatten, lvl_pos, geo, query_embed, targets)

    def geometry(self, shapes, valid_ratios, mask_flatten, device, padded=None):
        """Everything that depends only on the level shapes and padding masks.  padded: whether
        any frame is padded when the caller knows it from the host-side image sizes (None: ask
        the mask, one device -> host sync)."""
        L = len(shapes)
        geo = {'shapes': [tuple(int(v) for v in s) for s in shapes], 'valid_ratios': valid_ratios}
        geo['spatial_shapes'] = host_to_device(geo['shapes'], torch.long, device)
        geo['mask_flatten'] = mask_flatten
        if mask_flatten is None or padded is False:
            geo['pad_mask'] = None
        elif padded:
            geo['pad_mask'] = mask_flatten
        else:
            geo['pad_mask'] = mask_flatten if bool(mask_flatten.any()) else None
        if self.multi_frame_attention_separate_encoder:
            half = L // 2
            s_half = sum(h * w for h, w in geo['shapes'][:half])
            geo['enc'] = []
            for sl_lv, sl_tok in ((slice(0, half), slice(0, s_half)), (slice(half, L), slice(s_half, None))):
                sh = geo['shapes'][sl_lv]
                vr = valid_ratios[:, sl_lv]
                geo['enc'].append(dict(shapes=sh, spatial_shapes=geo['spatial_shapes'][sl_lv].contiguous(),
                                       valid_ratios=vr, tok=sl_tok, order=K.encoder_tile_order(sh, device),
                                       ref=DeformableTransformerEncoder.get_reference_points(sh, vr, device)))
        else:
            geo['enc'] = [dict(shapes=geo['shapes'], spatial_shapes=geo['spatial_shapes'], valid_ratios=valid_ratios,
                               tok=slice(0, None), order=K.encoder_tile_order(geo['shapes'], device),
                               ref=DeformableTransformerEncoder.get_reference_points(geo['shapes'], valid_ratios,
                                                                                     device))]
        return geo

    def _query_inputs(self, query_embed, bs, dt):
        """(query_pos, tgt, reference_points) for `bs` frames without track queries, cached per
        parameter version (deformable_transformer.py:198-202)."""
        rp = self.reference_points
        c = self.d_model

        def make(qe, w, b):
            q, t = torch.split(qe.detach(), c, dim=1)
            ref = K.linear(q.float().contiguous(), w, b).sigmoid()
            return (q.to(dt).unsqueeze(0).expand(bs, -1, -1).contiguous(),
                    t.to(dt).unsqueeze(0).expand(bs, -1, -1).contiguous(),
                    ref.unsqueeze(0).expand(bs, -1, -1).contiguous())
        return K.cached_multi([query_embed, rp.weight, rp.bias], ('query_inputs', bs, dt), make)

    share_frame_pos = True   # forward_flat: unpadded frames read one shared position embedding (A/B, tests)

    def forward_flat(self, src_flatten, lvl_pos_embed_flatten, geo, query_embed=None, targets=None):
        """deformable_transformer.py:159-257 on flattened inputs."""
        assert query_embed is not None
        pad = geo['pad_mask']
        # no frame padded: every frame's position embedding is the same function of the level
        # shapes, so the encoder's projections read frame 0's rows for all frames (x_add of one
        # frame, kernels._load_add_operand) -- the same values, 1/B of the bytes
        pos_shared = self.share_frame_pos and fast_path(self) and pad is None and src_flatten.shape[0] > 1
        encs = []
        for e in geo['enc']:
            tok = e['tok']
            pm = pad[:, tok] if pad is not None else None
            src = src_flatten[:, tok]
            pos = lvl_pos_embed_flatten[:1, tok] if pos_shared else lvl_pos_embed_flatten[:, tok]
            if fast_path(self):
                src, pos = src.contiguous(), pos.contiguous()
                pm = pm.contiguous() if pm is not None else None
            encs.append(self.encoder(src, e['spatial_shapes'], e['valid_ratios'], pos, pm, reference_points=e['ref'],
                                     query_order=e.get('order'), shapes_host=e['shapes']))
        if len(encs) == 2:
            prev_memory, memory = encs
            memory = torch.cat([memory, prev_memory], 1)   # [current, prev] -- reference order (:173)
        else:
            memory = encs[0]

        bs, _, c = memory.shape
        query_attn_mask = None
        tracking = targets is not None and 'track_query_hs_embeds' in targets[0]
        if fast_path(self) and not tracking:
            # inference without track queries: the object queries, their positional half and
            # the initial reference points depend only on parameters -> cached per parameter
            # version, dtype and batch size (no per-forward casts / copies / GEMM)
            query_embed_, tgt, reference_points = self._query_inputs(query_embed, bs, memory.dtype)
        else:
            query_embed_, tgt = torch.split(query_embed, c, dim=1)
            query_embed_ = query_embed_.unsqueeze(0).expand(bs, -1, -1)
            tgt = tgt.unsqueeze(0).expand(bs, -1, -1)
            rp = self.reference_points
            if fast_path(self):
                reference_points = K.linear(query_embed_[0].float(), rp.weight, rp.bias).sigmoid()
                reference_points = reference_points.unsqueeze(0).expand(bs, -1, -1)
            else:
                reference_points = A.linear_module(query_embed_, rp).sigmoid()
        if tracking:
            prev_hs_embed = torch.stack([t['track_query_hs_embeds'] for t in targets])
            prev_boxes = torch.stack([t['track_query_boxes'] for t in targets])
            prev_query_embed = torch.zeros_like(prev_hs_embed)
            query_embed_ = torch.cat([prev_query_embed.to(query_embed_.dtype), query_embed_], dim=1)
            tgt = torch.cat([prev_hs_embed.to(tgt.dtype), tgt], dim=1)
            reference_points = torch.cat([prev_boxes[..., :2].to(reference_points.dtype), reference_points], dim=1)
        init_reference_out = reference_points
        if fast_path(self) and tracking:
            dt = memory.dtype
            tgt = tgt.to(dt).contiguous()
            query_embed_ = query_embed_.to(dt).contiguous()
        hs, inter_references = self.decoder(tgt, reference_points, memory, geo['spatial_shapes'],
                                            geo['valid_ratios'], query_embed_, pad, query_attn_mask)
        return hs, memory, init_reference_out, inter_references, None, None


def build_deforamble_transformer(args):
    num_feature_levels = args.num_feature_levels
    if args.multi_frame_attention:
        num_feature_levels *= 2
    return DeformableTransformer(
        d_model=args.hidden_dim, nhead=args.nheads, num_encoder_layers=args.enc_layers,
        num_decoder_layers=args.dec_layers, dim_feedforward=args.dim_feedforward, dropout=args.dropout,
        activation="relu", return_intermediate_dec=True, num_feature_levels=num_feature_levels,
        dec_n_points=args.dec_n_points, enc_n_points=args.enc_n_points, two_stage=args.two_stage,
        two_stage_num_proposals=args.num_queries,
        multi_frame_attention_separate_encoder=args.multi_frame_attention and args.multi_frame_attention_separate_encoder)

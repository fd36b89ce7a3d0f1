"""KineT kinematic tracker model on kinet_amd kernels.

The fork's own model: no image, no CNN, no MSDeformAttn -- it reads the detections of a frame
(boxes (B, n, 4) + a confidence channel (B, n, 1), padding-masked) and the trails of the
active tracks, and predicts boxes / classes for `num_queries` object queries plus one query per
tracklet.  Reference: detr.py:288-425 (`KinematicDetectorTransformer`), transformer.py:85-185
(`KinematicTransformer`, `DualKinematicTransformer`, `IntertwinedBranch` :477-492, the post-norm
encoder / decoder layers :283-461), backbone.py:111-167 + 197-216 (`LayerBackboneFC`,
`Kinet_Backbone`, the kine branch of `build_backbone`), position_encoding.py:151-180
(`PositionEmbeddingSineDetections`), detr_tracking.py:524-883 (`KinetTracking`),
models/__init__.py:72-107.  Module names and parameter shapes equal the reference's, so its
state_dicts load unchanged (tests/test_kinet.py pins the key list).

Compute: every Linear (with its ReLU / residual / post-norm LayerNorm fused into the GEMM
epilogue), every LayerNorm and the attention core run kinet kernels (`kernels.linear`,
`kernels.layernorm`, `kernels.mha_core`); the two IntertwinedBranch projections write their
halves of the concatenation in place (strided GEMM outputs).  With autograd on (or in train
mode with dropout) the same graph runs the `kinet_amd.autograd` Functions with the reference's
dropouts.  Batch-first (B, L, d) throughout; the reference's (L, B, d) is a layout detail.
The detection position embedding (a cumsum + sin/cos over a (B, n) mask) is cached per mask.

Reference defects (SURVEY.md Appendix A style -- visible, not silent):
  * cfgs/train_kinet.yaml asks for `position_embedding: sine`, with which the reference calls
    PositionEmbeddingSineDetections(n, normalize=True) -> TypeError (position_encoding.py:193
    vs :151); 'sine' and 'sine_detection' both build the detection embedding here.
  * with tracklet queries (K > 0) the reference builds the metadata queries from the already
    track-extended detection queries (detr.py:397-399: 2K+Q metadata vs K+Q detection queries)
    and IntertwinedBranch's concat raises; here they are built from `query_embed_metadata` (the
    evident intent).  The K > 0 fixture is the reference DualKinematicTransformer + heads run on
    those inputs (tests/golden/make_golden.py gen_kinet).
  * the training sampler (`add_track_queries_to_targets2`, detr_tracking.py:806-862) always
    yields K > 0 when a frame has objects, so reference KineT training only runs with
    ratio_add_tracklets = 0; that case (empty tracklets) is supported, K > 0 training raises.
"""
import math

import torch
import torch.nn.functional as F
from torch import nn

from kinet_amd import autograd as A
from kinet_amd import kernels as K
from kinet_amd.models.deformable_detr import MLP
from kinet_amd.models.misc import NestedTensor, NestedTensorKinet


# ----------------------------------------------------------------------------- op helpers
def _linear(x, mod, fast, relu=False, residual=None, ln=None, x_add=None, drop=None):
    """ln?(residual + drop(relu?(mod(x [+ x_add])))) -- one GEMM with a fused epilogue on the
    fast path; kinet autograd Functions + the reference's dropout otherwise."""
    if fast:
        return K.linear(x, mod.weight, mod.bias, relu=relu, residual=residual, x_add=x_add,
                        ln=None if ln is None else (ln.weight, ln.bias, ln.eps))
    y = A.linear_module(x if x_add is None else x + x_add, mod)
    if relu:
        y = F.relu(y)
    if drop is not None:
        y = drop(y)
    if residual is not None:
        y = residual + y
    return y if ln is None else A.layer_norm(y, ln)


def _attention(mod, query, key, value, fast, q_add=None, k_add=None, key_padding_mask=None):
    """nn.MultiheadAttention(query [+ q_add], key [+ k_add], value, key_padding_mask)[0]
    BEFORE its out_proj (the caller fuses out_proj with residual + LayerNorm); batch-first.
    In training the attention probabilities are dropped with the module's `dropout` (as
    kinet_amd.autograd.multihead_attention)."""
    E = mod.embed_dim
    w, b = mod.in_proj_weight, mod.in_proj_bias
    scale = mod.head_dim ** -0.5
    if fast:
        if query is key and q_add is k_add:       # q = k = x + pos: one GEMM for both
            qk = K.linear(query, K.param_rows(w, 0, 2 * E), K.param_rows(b, 0, 2 * E), x_add=q_add)
            q, k = qk[..., :E], qk[..., E:]
        else:
            q = K.linear(query, K.param_rows(w, 0, E), K.param_rows(b, 0, E), x_add=q_add)
            k = K.linear(key, K.param_rows(w, E, 2 * E), K.param_rows(b, E, 2 * E), x_add=k_add)
        v = K.linear(value, K.param_rows(w, 2 * E, 3 * E), K.param_rows(b, 2 * E, 3 * E))
        return K.mha_core(q, k, v, mod.num_heads, scale, key_mask=key_padding_mask)
    q = A.linear(query if q_add is None else query + q_add, w[:E], b[:E])
    k = A.linear(key if k_add is None else key + k_add, w[E:2 * E], b[E:2 * E])
    v = A.linear(value, w[2 * E:], b[2 * E:])
    return A.mha_core(q, k, v, mod.num_heads, scale, key_padding_mask,
                      dropout_p=mod.dropout if mod.training else 0.0)


def _layer_norm(x, ln, fast, residual=None):
    if fast:
        return K.layernorm(x, ln.weight, ln.bias, ln.eps, residual=residual)
    return A.layer_norm(x if residual is None else x + residual, ln)


def _mlp(mlp, x, fast):
    """detr.py:937-951 MLP (ReLU between layers)."""
    n = len(mlp.layers)
    for i, layer in enumerate(mlp.layers):
        x = _linear(x, layer, fast, relu=i < n - 1)
    return x


# ----------------------------------------------------------------------------- backbone
class LayerBackboneFC(nn.Module):
    """backbone.py:111-125: norm(linear3(drop(relu(linear2(drop(linear1(x)))))))."""

    def __init__(self, input_dim, hidden_dim, activation='relu', dropout=0.1):
        super().__init__()
        if activation != 'relu':
            raise NotImplementedError(activation)
        self.linear1 = nn.Linear(input_dim, hidden_dim)
        self.linear2 = nn.Linear(hidden_dim, hidden_dim)
        self.linear3 = nn.Linear(hidden_dim, hidden_dim)
        self.dropout = nn.Dropout(dropout)
        self.norm = nn.LayerNorm(hidden_dim)

    def run(self, x, fast):
        h = _linear(x, self.linear1, fast, drop=self.dropout)
        h = _linear(h, self.linear2, fast, relu=True, drop=self.dropout)
        return _linear(h, self.linear3, fast, ln=self.norm)


class KinetBackbone(nn.Module):
    """backbone.py:128-167 (`Kinet_Backbone`): one LayerBackboneFC to hidden_dims[-1]."""

    def __init__(self, input_dim, hidden_dims, activation='relu', return_interm_layers=False):
        super().__init__()
        self.return_interm_layers = return_interm_layers
        self.num_channels = hidden_dims
        self.layers = nn.ModuleList([LayerBackboneFC(input_dim, hidden_dims[-1], activation)])

    def run(self, tensor_list, fast):
        x, mask = tensor_list.tensors, tensor_list.mask
        for layer in self.layers:
            x = layer.run(x, fast)
        return [NestedTensor(x, mask)]


class PositionEmbeddingSineDetections(nn.Module):
    """position_encoding.py:151-180: per detection slot, (cumsum(~mask) % max_det - 0.5) /
    max_det * 2pi, sin / cos interleaved over temperature ** (k / num_pos_feats)."""

    def __init__(self, num_pos_feats=64, temperature=10000, scale=None, max_detections=60):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.scale = 2 * math.pi if scale is None else scale
        self.max_detections = max_detections

    def embed(self, mask):
        def make(m):
            y = (~m).cumsum(1, dtype=torch.float32) % self.max_detections
            y = (y - 0.5) / self.max_detections * self.scale
            dim_t = torch.arange(self.num_pos_feats, dtype=torch.float32, device=m.device)
            dim_t = self.temperature ** (dim_t / self.num_pos_feats)
            p = y[:, :, None] / dim_t
            return torch.stack((p.sin(), p.cos()), dim=3).flatten(2)
        return K.cached(mask, ('kinet_pos', self.num_pos_feats, self.max_detections), make)

    def forward(self, tensor_list):
        return self.embed(tensor_list.mask)


class Joiner(nn.Sequential):
    """backbone.py:180-194 for the kinematic backbones: [0] = KinetBackbone, [1] = embedding."""

    def __init__(self, backbone, position_embedding):
        super().__init__(backbone, position_embedding)
        self.num_channels = backbone.num_channels

    def run(self, tensor_list, fast):
        xs = self[0].run(tensor_list, fast)
        return xs, [self[1].embed(x.mask).to(x.tensors.dtype) for x in xs]


# -------------------------------------------------------------------------- transformer
class TransformerEncoderLayer(nn.Module):
    """transformer.py:283-345 (post-norm)."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation='relu', normalize_before=False):
        super().__init__()
        if normalize_before or activation != 'relu':
            raise NotImplementedError('pre-norm / non-ReLU kinematic layers (false in every config)')
        self.self_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)

    def run(self, src, pos, key_padding_mask, fast):
        sa = self.self_attn
        o = _attention(sa, src, src, src, fast, q_add=pos, k_add=pos, key_padding_mask=key_padding_mask)
        src = _linear(o, sa.out_proj, fast, residual=src, ln=self.norm1, drop=self.dropout1)
        h = _linear(src, self.linear1, fast, relu=True, drop=self.dropout)
        return _linear(h, self.linear2, fast, residual=src, ln=self.norm2, drop=self.dropout2)


class TransformerDecoderLayer(nn.Module):
    """transformer.py:348-410 (post-norm)."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation='relu', normalize_before=False):
        super().__init__()
        if normalize_before or activation != 'relu':
            raise NotImplementedError('pre-norm / non-ReLU kinematic layers (false in every config)')
        self.self_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout)
        self.multihead_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.norm3 = nn.LayerNorm(d_model)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.dropout3 = nn.Dropout(dropout)

    def run(self, tgt, memory, pos, query_pos, memory_key_padding_mask, fast):
        sa, ca = self.self_attn, self.multihead_attn
        o = _attention(sa, tgt, tgt, tgt, fast, q_add=query_pos, k_add=query_pos)
        tgt = _linear(o, sa.out_proj, fast, residual=tgt, ln=self.norm1, drop=self.dropout1)
        o = _attention(ca, tgt, memory, memory, fast, q_add=query_pos, k_add=pos,
                       key_padding_mask=memory_key_padding_mask)
        tgt = _linear(o, ca.out_proj, fast, residual=tgt, ln=self.norm2, drop=self.dropout2)
        h = _linear(tgt, self.linear1, fast, relu=True, drop=self.dropout)
        return _linear(h, self.linear2, fast, residual=tgt, ln=self.norm3, drop=self.dropout3)


class TransformerEncoder(nn.Module):
    """transformer.py:236-256 (no final norm when post-norm)."""

    def __init__(self, layer, num_layers):
        super().__init__()
        self.layers = nn.ModuleList(_clone(layer) for _ in range(num_layers))
        self.num_layers = num_layers

    def run(self, src, pos, mask, fast):
        for layer in self.layers:
            src = layer.run(src, pos, mask, fast)
        return src


class TransformerDecoder(nn.Module):
    """transformer.py:259-280: every layer's output stacked, the decoder norm over the stack."""

    def __init__(self, layer, num_layers, d_model, return_intermediate=True):
        super().__init__()
        self.layers = nn.ModuleList(_clone(layer) for _ in range(num_layers))
        self.num_layers = num_layers
        self.norm = nn.LayerNorm(d_model)
        self.return_intermediate = return_intermediate

    def run(self, tgt, memory, pos, query_pos, mask, fast):
        outs = []
        for layer in self.layers:
            tgt = layer.run(tgt, memory, pos, query_pos, mask, fast)
            outs.append(tgt)
        stack = torch.stack(outs) if self.return_intermediate else tgt[None]
        return _layer_norm(stack, self.norm, fast), stack


def _clone(m):
    import copy
    return copy.deepcopy(m)


class KinematicTransformer(nn.Module):
    """transformer.py:85-142: encoder over the detection slots, decoder over the queries."""

    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=2048,
                 dropout=0.1, activation='relu', normalize_before=False, return_intermediate_dec=False,
                 track_attention=False):
        super().__init__()
        if track_attention:
            raise NotImplementedError('track_attention (false in every config)')
        self.d_model, self.nhead = d_model, nhead
        enc = TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation, normalize_before)
        dec = TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation, normalize_before)
        self.encoder = TransformerEncoder(enc, num_encoder_layers)
        self.decoder = TransformerDecoder(dec, num_decoder_layers, d_model, return_intermediate_dec)
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def run(self, src, mask, query_embed, tgt, pos, fast):
        """src (B, n, d), mask (B, n), query_embed / tgt (B, Q, d), pos (B, n, d) ->
        hs (L, B, Q, d) normed, hs without norm, memory (B, n, d)."""
        if tgt is None:
            tgt = torch.zeros_like(query_embed)
        memory = self.encoder.run(src, pos, mask, fast)
        hs, hs_without_norm = self.decoder.run(tgt, memory, pos, query_embed, mask, fast)
        return hs, hs_without_norm, memory


class IntertwinedBranch(nn.Module):
    """transformer.py:477-492: norm(drop(relu([lin1(src1) | lin2(src2)])) + src1);
    `linear2` exists in the reference but is never applied (kept for the state_dict)."""

    def __init__(self, d_model=256, dropout=0.1, activation='relu', dim_concat=3):
        super().__init__()
        self.linear_input1 = nn.Linear(d_model, d_model // 2)
        self.linear_input2 = nn.Linear(d_model, d_model // 2)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(d_model // 2, d_model)
        self.norm = nn.LayerNorm(d_model)
        self.dim_concat = dim_concat

    def run(self, src1, src2, fast):
        h = self.linear_input1.out_features
        if fast:
            lead = src1.shape[:-1]
            x = torch.empty(*lead, 2 * h, dtype=src1.dtype, device=src1.device)
            x2 = x.view(-1, 2 * h)
            K.linear(src1, self.linear_input1.weight, self.linear_input1.bias, relu=True, out=x2[:, :h])
            K.linear(src2, self.linear_input2.weight, self.linear_input2.bias, relu=True, out=x2[:, h:])
            return K.layernorm(x, self.norm.weight, self.norm.bias, self.norm.eps, residual=src1)
        x = torch.cat([A.linear_module(src1, self.linear_input1), A.linear_module(src2, self.linear_input2)], -1)
        return A.layer_norm(self.dropout(F.relu(x)) + src1, self.norm)


class DualKinematicTransformer(nn.Module):
    """transformer.py:145-185: a KinematicTransformer per stream (boxes, metadata), then the
    detection branch mixes in the metadata and the metadata branch the mixed detections."""

    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=2048,
                 dropout=0.1, activation='relu', normalize_before=False, return_intermediate_dec=False,
                 track_attention=False):
        super().__init__()
        self.d_model = d_model
        kw = (d_model, nhead, num_encoder_layers, num_decoder_layers, dim_feedforward, dropout, activation,
              normalize_before, return_intermediate_dec, track_attention)
        self.transformer_det = KinematicTransformer(*kw)
        self.transformer_metadata = KinematicTransformer(*kw)
        self.detection_branch = IntertwinedBranch(d_model, dropout, activation)
        self.metadata_branch = IntertwinedBranch(d_model, dropout, activation)

    def run(self, src_boxes, src_metadata, mask, query_embed_bbox, query_embed_metadata, tgt_bboxes, tgt_metadata,
            pos_boxes, pos_metadata, fast):
        hs_det, hs_without_norm_det, memory_det = self.transformer_det.run(src_boxes, mask, query_embed_bbox,
                                                                           tgt_bboxes, pos_boxes, fast)
        hs_meta, _, _ = self.transformer_metadata.run(src_metadata, mask, query_embed_metadata, tgt_metadata,
                                                      pos_metadata, fast)
        hs_det = self.detection_branch.run(hs_det, hs_meta, fast)
        hs_meta = self.metadata_branch.run(hs_meta, hs_det, fast)
        return hs_det, hs_meta, hs_without_norm_det, memory_det


# ------------------------------------------------------------------------------- model
class KinematicDetectorTransformer(nn.Module):
    """detr.py:288-425."""

    def __init__(self, backbone, transformer, num_classes, num_queries, aux_loss=False, overflow_boxes=False,
                 dim_tracklets_det=128, dim_tracklets_metadata=8):
        super().__init__()
        self.num_queries = num_queries
        self.transformer = transformer
        self.overflow_boxes = overflow_boxes
        d = self.hidden_dim
        self.class_embed = nn.Linear(d, num_classes + 1)
        self.bbox_embed = MLP(d, d, 4, 3)
        self.query_embed_det = nn.Embedding(num_queries, d)
        self.query_embed_metadata = nn.Embedding(num_queries, d)
        self.input_proj_tracklets_det = MLP(dim_tracklets_det, d, d, 3)
        self.input_proj_tracklets_metadata = MLP(dim_tracklets_metadata, d // 2, d, 3)
        self.backbone_det = backbone[0]
        self.backbone_metadata = backbone[1]
        self.aux_loss = aux_loss
        self._compute_dtype = torch.float32

    @property
    def hidden_dim(self):
        return self.transformer.d_model

    def set_compute_dtype(self, dtype):
        """bf16 / f16 / f32 for the inference path (the autograd path computes in f32)."""
        self._compute_dtype = dtype
        return self

    def _fast(self):
        if torch.is_grad_enabled():
            return False
        return not (self.training and any(isinstance(m, nn.Dropout) and m.p > 0 for m in self.modules()))

    def forward(self, samples, targets: list = None):
        fast = self._fast()
        dt = self._compute_dtype if fast else torch.float32
        dets, meta = samples.detections, samples.metadata
        dets = NestedTensor(dets.tensors.to(dt), dets.mask)
        meta = NestedTensor(meta.tensors.to(dt), meta.mask)
        features_det, pos_det = self.backbone_det.run(dets, fast)
        features_metadata, pos_metadata = self.backbone_metadata.run(meta, fast)
        src_det, mask = features_det[-1].decompose()
        src_metadata, _ = features_metadata[-1].decompose()
        B, d = src_det.shape[0], self.hidden_dim
        qd = self.query_embed_det.weight.to(dt)[None].expand(B, -1, -1)
        qm = self.query_embed_metadata.weight.to(dt)[None].expand(B, -1, -1)
        tgt_det = tgt_meta = None
        if targets is not None and len(targets[0]['track_query_hs_embeds_det']) > 0:
            # detr.py:376-404 (metadata queries from query_embed_metadata: see the module docstring)
            trk_det = torch.stack([t['track_query_hs_embeds_det'] for t in targets]).to(dt)
            trk_meta = torch.stack([t['track_query_hs_embeds_meta'] for t in targets]).to(dt)
            Kq = trk_det.shape[1]
            zeros = torch.zeros(B, Kq, d, dtype=dt, device=src_det.device)
            qd, qm = torch.cat([zeros, qd], 1), torch.cat([zeros, qm], 1)
            tgt_det = torch.cat([_mlp(self.input_proj_tracklets_det, trk_det, fast),
                                 torch.zeros_like(qd[:, Kq:])], 1)
            tgt_meta = torch.cat([_mlp(self.input_proj_tracklets_metadata, trk_meta, fast),
                                  torch.zeros_like(qm[:, Kq:])], 1)
        else:
            qd, qm = qd.contiguous(), qm.contiguous()
        hs_det, hs_meta, _, _ = self.transformer.run(src_det, src_metadata, mask, qd, qm, tgt_det, tgt_meta,
                                                     pos_det[0], pos_metadata[0], fast)
        if fast:
            outputs_class = K.linear(hs_meta, self.class_embed.weight, self.class_embed.bias, out_dtype=torch.float32)
            h = hs_det
            for i, layer in enumerate(self.bbox_embed.layers):
                last = i == len(self.bbox_embed.layers) - 1
                h = K.linear(h, layer.weight, layer.bias, relu=not last, out_dtype=torch.float32 if last else None)
            outputs_coord = h.sigmoid()
        else:
            outputs_class = A.linear_module(hs_meta, self.class_embed)
            outputs_coord = self.bbox_embed(hs_det).sigmoid()
        out = {'pred_logits': outputs_class[-1], 'pred_boxes': outputs_coord[-1]}
        if self.aux_loss:
            out['aux_outputs'] = [{'pred_logits': a, 'pred_boxes': b}
                                  for a, b in zip(outputs_class[:-1], outputs_coord[:-1])]
        return out, targets, features_det, src_det, hs_det


class KinetTracking(KinematicDetectorTransformer):
    """detr_tracking.py:524-883 (`KinetTracking` = KinetTrackingBase2 + the detector): tracking
    mode, tracklet-query dimensions, the empty-tracklet targets of training."""

    def __init__(self, tracking_kwargs, detr_kwargs):
        super().__init__(**detr_kwargs)
        tk = dict(track_query_false_positive_prob=0.0, track_query_false_negative_prob=0.0, matcher=None,
                  backprop_prev_frame=False, ratio_add_detections=0.5, frame_range=5, use_encoding=True,
                  num_pos_feats=32, ratio_add_tracklets=1.0, dim_metadata=1)
        tk.update(tracking_kwargs)
        self._matcher = tk['matcher']
        self._track_query_false_positive_prob = tk['track_query_false_positive_prob']
        self._track_query_false_negative_prob = tk['track_query_false_negative_prob']
        self._backprop_prev_frame = tk['backprop_prev_frame']
        self._frame_range = tk['frame_range']
        self._ratio_add_tracklets = tk['ratio_add_tracklets']
        self.dim_metadata = tk['dim_metadata']
        n = tk['num_pos_feats'] if tk['use_encoding'] else 1
        self.dim_tracklets_det = 4 * n * self._frame_range
        self.dim_tracklets_meta = self.dim_metadata * n * self._frame_range
        self._tracking = False

    def train(self, mode: bool = True):
        self._tracking = False
        return super().train(mode)

    def tracking(self):
        self.eval()
        self._tracking = True

    def generate_empty_tracklets(self, targets):
        """detr_tracking.py:627-638."""
        for t in targets:
            dev = t['boxes'].device
            t['track_query_hs_embeds_det'] = torch.zeros([0, self.dim_tracklets_det], device=dev)
            t['track_query_hs_embeds_meta'] = torch.zeros([0, self.dim_tracklets_meta], device=dev)
            t['track_queries_mask'] = torch.zeros(self.num_queries, dtype=torch.bool, device=dev)
            t['track_queries_fal_pos_mask'] = torch.zeros(self.num_queries, dtype=torch.bool, device=dev)
            t['track_query_match_ids'] = torch.zeros(0, dtype=torch.long, device=dev)

    def forward(self, samples, targets: list = None):
        if targets is not None and not self._tracking:
            if int(self._ratio_add_tracklets * max(len(t['labels']) for t in targets)) > 0:
                raise NotImplementedError(
                    'KineT training with tracklet queries: the reference forward raises for K > 0 '
                    '(detr.py:397-399, see kinet_amd/models/kinet.py); train with ratio_add_tracklets = 0')
            self.generate_empty_tracklets(targets)
        return super().forward(samples, targets)


def graph_kinet_forward(model, samples, targets=None, warmup=3):
    """A HIP-graph replay (kinet_amd/graph.py) of the no-grad inference forward of `model` for
    the signature of (samples, targets): batch, detection slots, tracklet-query count, dtypes.
    Returns call(samples, targets) -> the forward's output dict (graph-owned buffers,
    overwritten by the next call).  The batch-1 tracking forward is launch-bound eager
    (~1 ms host for ~0.1 ms of kernels); replay removes the per-kernel host cost."""
    from kinet_amd.graph import GraphedCall
    B = samples.detections.tensors.shape[0]
    has_trk = targets is not None and len(targets[0]['track_query_hs_embeds_det']) > 0

    def flat(smp, tgs):
        ts = [smp.detections.tensors, smp.detections.mask, smp.metadata.tensors, smp.metadata.mask]
        if has_trk:
            ts += [torch.stack([t['track_query_hs_embeds_det'] for t in tgs]),
                   torch.stack([t['track_query_hs_embeds_meta'] for t in tgs])]
        return ts

    def fn(d, dm, m, mm, *trk):
        smp = NestedTensorKinet(NestedTensor(d, dm), NestedTensor(m, mm))
        tgs = None
        if has_trk:
            tgs = [{'track_query_hs_embeds_det': trk[0][i], 'track_query_hs_embeds_meta': trk[1][i]}
                   for i in range(B)]
        return model(smp, tgs)[0]

    gc = GraphedCall(fn, flat(samples, targets), warmup,
                     params=list(model.parameters()) + list(model.buffers()),
                     state_fn=lambda: (model._compute_dtype, model.training))

    def call(smp, tgs=None):
        if (tgs is not None and len(tgs[0]['track_query_hs_embeds_det']) > 0) != has_trk:
            raise ValueError('graph_kinet_forward: tracklet queries present / absent unlike the recording')
        return gc(*flat(smp, tgs))
    return call


def build_kinet(args, num_classes, matcher=None):
    """models/__init__.py:72-107 + backbone.py:197-216 + transformer.py:508-531 (kine branch)."""
    if getattr(args, 'use_encoder_only', False):
        raise NotImplementedError('the encoder-only KineT variant (KinetTracking2) is not built')
    if not args.tracking:
        raise NotImplementedError('Kine model only implemented as tracking model (models/__init__.py:110)')
    if args.position_embedding not in ('sine', 'sine_detection'):
        raise ValueError(f'not supported {args.position_embedding}')
    input_dim_det = args.encoding_dim_detections * 4 if args.use_encoding_dets else 4
    input_dim_meta = 2 if args.use_class else 1
    interm = getattr(args, 'masks', False) or args.num_feature_levels > 1
    pos = PositionEmbeddingSineDetections(args.hidden_dim // 2, max_detections=args.max_number_detection)
    backbone_det = KinetBackbone(input_dim_det, [256, 512, args.hidden_dim], args.activation, interm)
    backbone_meta = KinetBackbone(input_dim_meta, [16, 64, args.hidden_dim], args.activation, interm)
    backbones = [Joiner(backbone_det, pos), Joiner(backbone_meta, pos)]
    meta = 2 if args.use_class else 1
    if args.use_encoding_tracklets:
        dim_det = 4 * args.encoding_dim_tracklets * args.track_prev_frame_range
        dim_meta = meta * args.encoding_dim_tracklets * args.track_prev_frame_range
    else:
        dim_det = 4 * args.track_prev_frame_range
        dim_meta = meta * args.track_prev_frame_range
    transformer = DualKinematicTransformer(d_model=args.hidden_dim, nhead=args.nheads,
                                           num_encoder_layers=args.enc_layers, num_decoder_layers=args.dec_layers,
                                           dim_feedforward=args.dim_feedforward, dropout=args.dropout,
                                           activation=args.activation, normalize_before=args.pre_norm,
                                           return_intermediate_dec=True, track_attention=args.track_attention)
    detr_kwargs = dict(backbone=backbones, transformer=transformer,
                       num_classes=num_classes - 1 if args.focal_loss else num_classes,
                       num_queries=args.num_queries, aux_loss=args.aux_loss, overflow_boxes=args.overflow_boxes,
                       dim_tracklets_det=dim_det, dim_tracklets_metadata=dim_meta)
    tracking_kwargs = dict(track_query_false_positive_prob=args.track_query_false_positive_prob,
                           track_query_false_negative_prob=args.track_query_false_negative_prob,
                           backprop_prev_frame=args.track_backprop_prev_frame, matcher=matcher,
                           use_encoding=args.use_encoding_tracklets, frame_range=args.track_prev_frame_range,
                           num_pos_feats=args.encoding_dim_tracklets, ratio_add_tracklets=args.ratio_add_tracklets)
    return KinetTracking(tracking_kwargs, detr_kwargs)

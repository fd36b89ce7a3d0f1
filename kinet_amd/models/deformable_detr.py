"""DeformableDETR detector on the kinet_amd kernels.

Mirrors src/trackformer/models/deformable_detr.py (DeformableDETR :29-283,
DeformablePostProcess :286-334) and the DETR base pieces it uses (models/detr.py: DETR
attributes :17-60, MLP :937-951) with identical module/parameter names, forward
signature `model(samples, targets=None, prev_features=None) -> (out, targets, features,
memory, hs)` and output dict keys (`pred_logits`, `pred_boxes`, `hs_embed`,
`aux_outputs`).

Inference path (autograd disabled): backbone convs, input projections (1x1 conv = GEMM,
3x3/2 conv = implicit GEMM, GroupNorm written straight into the flattened multi-level
source buffer), the transformer and the heads all run HIP kernels in `compute_dtype`
(torch.bfloat16 perf mode, torch.float32 parity mode).  Everything that depends only on
the frame geometry (padding masks per level, valid ratios, encoder reference points,
sine position embeddings + level embeddings) is computed once per geometry and cached.
With box refinement the per-layer boxes are exactly the decoder's refined references
(the head recomputes bbox_embed[l](hs[l]) + inverse_sigmoid(ref_l), deformable_detr.py:
236-244, which IS the decoder's refinement of layer l, deformable_transformer.py:416-424),
so the head reuses them instead of running the box MLPs twice.
"""
import copy
import math

import torch
import torch.nn.functional as F
from torch import nn

from kinet_amd import autograd as A
from kinet_amd import kernels as K
from kinet_amd.models.backbone import interp_mask, nchw_to_nhwc, nhwc_as_nchw
from kinet_amd.models.deformable_transformer import fast_path, mlp_fast
from kinet_amd.models.misc import (NestedTensor, box_cxcywh_to_xyxy, inverse_sigmoid,
                                   nested_tensor_from_tensor_list)


def _get_clones(module, N):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


class MLP(nn.Module):
    """detr.py:937-951."""

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(nn.Linear(n, k) for n, k in zip([input_dim] + h, h + [output_dim]))

    def forward(self, x):   # autograd path (kinet Linear Functions)
        for i, layer in enumerate(self.layers):
            x = F.relu(A.linear_module(x, layer)) if i < self.num_layers - 1 else A.linear_module(x, layer)
        return x


class DeformableDETR(nn.Module):
    def __init__(self, backbone, transformer, num_classes, num_queries, num_feature_levels,
                 aux_loss=True, with_box_refine=False, two_stage=False, overflow_boxes=False,
                 multi_frame_attention=False, multi_frame_encoding=False, merge_frame_features=False):
        super().__init__()
        if two_stage:
            raise NotImplementedError('two_stage is not on the configured hot path')
        if merge_frame_features:
            raise NotImplementedError('merge_frame_features is false in every configured path')
        # DETR base attributes (detr.py:34-53), same registration order
        self.num_queries = num_queries
        self.transformer = transformer
        self.overflow_boxes = overflow_boxes
        hidden_dim = transformer.d_model
        self.class_embed = nn.Linear(hidden_dim, num_classes + 1)
        self.bbox_embed = MLP(hidden_dim, hidden_dim, 4, 3)
        self.query_embed = nn.Embedding(num_queries, hidden_dim * 2)
        self.backbone = backbone
        self.aux_loss = aux_loss
        # DeformableDETR (deformable_detr.py:48-117)
        self.merge_frame_features = merge_frame_features
        self.multi_frame_attention = multi_frame_attention
        self.multi_frame_encoding = multi_frame_encoding
        self.num_feature_levels = num_feature_levels
        num_channels = backbone.num_channels[-3:]
        if num_feature_levels > 1:
            num_backbone_outs = len(backbone.strides) - 1
            input_proj_list = []
            for i in range(num_backbone_outs):
                input_proj_list.append(nn.Sequential(nn.Conv2d(num_channels[i], hidden_dim, kernel_size=1),
                                                     nn.GroupNorm(32, hidden_dim)))
            in_channels = num_channels[num_backbone_outs - 1]
            for _ in range(num_feature_levels - num_backbone_outs):
                input_proj_list.append(nn.Sequential(
                    nn.Conv2d(in_channels, hidden_dim, kernel_size=3, stride=2, padding=1),
                    nn.GroupNorm(32, hidden_dim)))
                in_channels = hidden_dim
            self.input_proj = nn.ModuleList(input_proj_list)
        else:
            self.input_proj = nn.ModuleList([nn.Sequential(nn.Conv2d(num_channels[0], hidden_dim, kernel_size=1),
                                                           nn.GroupNorm(32, hidden_dim))])
        self.with_box_refine = with_box_refine
        self.two_stage = two_stage
        prior_prob = 0.01
        bias_value = -math.log((1 - prior_prob) / prior_prob)
        self.class_embed.bias.data = torch.ones_like(self.class_embed.bias) * bias_value
        nn.init.constant_(self.bbox_embed.layers[-1].weight.data, 0)
        nn.init.constant_(self.bbox_embed.layers[-1].bias.data, 0)
        for proj in self.input_proj:
            nn.init.xavier_uniform_(proj[0].weight, gain=1)
            nn.init.constant_(proj[0].bias, 0)
        num_pred = transformer.decoder.num_layers
        if with_box_refine:
            self.class_embed = _get_clones(self.class_embed, num_pred)
            self.bbox_embed = _get_clones(self.bbox_embed, num_pred)
            nn.init.constant_(self.bbox_embed[0].layers[-1].bias.data[2:], -2.0)
            self.transformer.decoder.bbox_embed = self.bbox_embed
        else:
            nn.init.constant_(self.bbox_embed.layers[-1].bias.data[2:], -2.0)
            self.class_embed = nn.ModuleList([self.class_embed for _ in range(num_pred)])
            self.bbox_embed = nn.ModuleList([self.bbox_embed for _ in range(num_pred)])
            self.transformer.decoder.bbox_embed = None
        self.compute_dtype = torch.float32
        self._geo_cache = {}

    @property
    def hidden_dim(self):
        return self.transformer.d_model

    def set_compute_dtype(self, dtype):
        """torch.bfloat16 (perf) or torch.float32 (parity) for the HIP inference path."""
        if dtype not in (torch.float32, torch.bfloat16, torch.float16):
            raise ValueError(f'unsupported compute dtype {dtype}')
        self.compute_dtype = dtype
        self._geo_cache.clear()
        return self

    # ------------------------------------------------------------------ geometry cache
    def _geometry(self, cur_masks, prev_masks, shapes_by_frame, key, device):
        """Masks / valid ratios / refs / position+level embeddings for one frame geometry.
        cur_masks: the 3 backbone-level masks of the current frame; prev_masks the same for
        the previous frame (multi-frame) or None.  Mirrors deformable_detr.py:161-221 and
        deformable_transformer.py:136-157."""
        ent = self._geo_cache.get(key) if key is not None else None
        lvl_embed = self.transformer.level_embed
        ver = (lvl_embed._version, lvl_embed.data_ptr(), self.compute_dtype)
        if ent is not None and ent[0] == ver:
            return ent[1]
        frames = [prev_masks, cur_masks] if self.multi_frame_attention else [cur_masks]
        three_d = self.multi_frame_attention and self.multi_frame_encoding
        pe = self.backbone[1]
        # (mask the embedding is computed from, frame index of the 3-d embedding) per level, in
        # level order; the backbone levels use the CURRENT frame's masks (:141, :167)
        masks, pos_src = [], []
        for frame, fmasks in enumerate(frames):
            for l, m in enumerate(fmasks):
                masks.append(m)
                pos_src.append((cur_masks[l], frame if three_d else 0))
            hw_extra = shapes_by_frame[frame][len(fmasks):]
            for (h, w) in hw_extra:
                m = interp_mask(fmasks[0], (h, w))     # :212-213 (from the first level's mask)
                masks.append(m)
                pos_src.append((m, frame if three_d else 0))
        shapes = [s for fs in shapes_by_frame for s in fs]
        B = masks[0].shape[0]
        S = sum(h * w for h, w in shapes)
        d = self.hidden_dim
        # sine embedding + level embedding written straight into the flattened (B, S, d) rows
        # (deformable_transformer.py:141-157) in the compute dtype, one kernel per level
        lvl_pos = torch.empty((B, S, d), dtype=self.compute_dtype, device=device)
        off = 0
        for lvl, ((m, f), (h, w)) in enumerate(zip(pos_src, shapes)):
            pe.rows(m, f, level_embed=lvl_embed[lvl].detach(), out=lvl_pos[:, off:off + h * w], out_batch_stride=S * d)
            off += h * w
        mask_flatten = torch.cat([m.flatten(1) for m in masks], 1)
        valid_ratios = torch.stack([self.transformer.get_valid_ratio(m) for m in masks], 1)
        geo = self.transformer.geometry(shapes, valid_ratios, mask_flatten, device)
        geo.update(lvl_pos=lvl_pos, masks=masks, S=sum(h * w for h, w in shapes))
        if key is not None:
            if len(self._geo_cache) > 16:
                self._geo_cache.clear()
            self._geo_cache[key] = (ver, geo)
        return geo

    # ------------------------------------------------------------------ input projection
    def _project_frame(self, feats_nhwc, src, offsets):
        """input_proj (deformable_detr.py:175-221) for one frame; writes each level's
        GroupNorm output into src[:, off:off+h*w] (the flattened transformer input)."""
        B = feats_nhwc[0].shape[0]
        S = src.shape[1]
        d = self.hidden_dim
        nb = len(feats_nhwc)
        last = None
        for l in range(self.num_feature_levels):   # per frame (deformable_detr.py:194)
            conv, gn = self.input_proj[l][0], self.input_proj[l][1]
            if l < nb:
                x = feats_nhwc[l]
                Bx, h, w, C = x.shape
                y = K.linear(x.view(Bx * h * w, C), K.param_matrix(conv.weight), conv.bias)
            else:
                x = feats_nhwc[-1] if l == nb else last
                wp = K.pack_conv_weight(conv.weight, x.dtype)
                y4 = K.conv2d_nhwc(x, wp, 2, 1, bias=K.f32(conv.bias))
                Bx, h, w, _ = y4.shape
                y = y4.view(Bx * h * w, d)
                last = y4
            off = offsets[l]
            out = src[:, off:off + h * w]
            normed = K.groupnorm_nhwc(y.view(B, h * w, d), gn.weight, gn.bias, gn.num_groups, gn.eps,
                                      out=out, out_batch_stride=S * d)
            if l >= nb and l + 1 < self.num_feature_levels:
                # the next extra level convolves this level's normalised output (:209)
                last = out.reshape(B, h, w, d) if B == 1 else out.contiguous().view(B, h, w, d)
            del normed

    # ------------------------------------------------------------------ forward
    def forward(self, samples, targets: list = None, prev_features=None):
        if not isinstance(samples, NestedTensor):
            samples = nested_tensor_from_tensor_list(samples)
        if not fast_path(self):
            return self._forward_reference(samples, targets, prev_features)
        dt = self.compute_dtype
        device = samples.tensors.device
        feats = self.backbone[0].forward_nhwc(samples.tensors, dt)   # layer1..4 NHWC
        sizes = samples.sizes
        # the padding masks per level depend only on the input mask: cached per mask tensor
        all_masks = [K.cached(samples.mask, ('interp', tuple(f.shape[1:3])),
                              lambda m, hw=tuple(f.shape[1:3]): interp_mask(m, hw)) for f in feats]
        features_all = [NestedTensor(nhwc_as_nchw(f), m, sizes) for f, m in zip(feats, all_masks)]
        features = features_all[-3:]
        cur_nhwc = feats[-3:]
        if prev_features is None:
            prev_features = features
        else:
            prev_features = prev_features[-3:]
        prev_nhwc = [nchw_to_nhwc(f.tensors).to(dt) for f in prev_features] if self.multi_frame_attention else None

        def level_shapes(fn):
            s = [tuple(t.shape[1:3]) for t in fn]
            h, w = s[-1]
            n_extra = self.num_feature_levels - len(fn)
            for _ in range(n_extra):
                h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
                s.append((h, w))
            return s
        cur_shapes = level_shapes(cur_nhwc)
        if self.multi_frame_attention:
            prev_shapes = level_shapes(prev_nhwc)
            shapes_by_frame = [prev_shapes, cur_shapes]
            prev_sizes = getattr(prev_features[0], 'sizes', None)
            key = None if (sizes is None or prev_sizes is None) else ('mf', sizes, prev_sizes, tuple(cur_shapes))
            geo = self._geometry([m for m in all_masks[-3:]], [f.mask for f in prev_features], shapes_by_frame,
                                 key, device)
        else:
            shapes_by_frame = [cur_shapes]
            key = None if sizes is None else ('sf', sizes, tuple(cur_shapes))
            geo = self._geometry(all_masks[-3:], None, shapes_by_frame, key, device)

        B = samples.tensors.shape[0]
        d = self.hidden_dim
        src = torch.empty((B, geo['S'], d), dtype=dt, device=device)
        off = 0
        for f, (fn, fshapes) in enumerate(zip([prev_nhwc, cur_nhwc] if self.multi_frame_attention else [cur_nhwc],
                                              shapes_by_frame)):
            offs = []
            for (h, w) in fshapes:
                offs.append(off)
                off += h * w
            self._project_frame(fn, src, offs)

        hs, memory, init_reference, inter_references, _, _ = self.transformer.forward_flat(
            src, geo['lvl_pos'], geo, self.query_embed.weight, targets)

        nl = hs.shape[0]
        n_cls = self.class_embed[0].weight.shape[0]
        outputs_class = torch.empty((nl,) + tuple(hs.shape[1:3]) + (n_cls,), dtype=torch.float32, device=device)
        outputs_coords = []
        for lvl in range(nl):
            K.linear(hs[lvl], self.class_embed[lvl].weight, self.class_embed[lvl].bias, out_dtype=torch.float32,
                     out=outputs_class[lvl].view(-1, n_cls))
            if not self.with_box_refine:
                tmp = mlp_fast(self.bbox_embed[lvl], hs[lvl])
                outputs_coords.append(K.box_refine(tmp, init_reference, want_input=False)[0])
        # with box refinement the per-layer boxes ARE the decoder's refined references (module doc)
        outputs_coord = inter_references if self.with_box_refine else torch.stack(outputs_coords)
        out = {'pred_logits': outputs_class[-1], 'pred_boxes': outputs_coord[-1], 'hs_embed': hs[-1].float()}
        if self.aux_loss:
            out['aux_outputs'] = self._set_aux_loss(outputs_class, outputs_coord)
        memory_slices = []
        o = 0
        for (h, w) in geo['shapes']:
            memory_slices.append(memory[:, o:o + h * w].permute(0, 2, 1).view(B, d, h, w))
            o += h * w
        return out, targets, features_all, memory_slices, hs

    @torch.jit.unused
    def _set_aux_loss(self, outputs_class, outputs_coord):
        return [{'pred_logits': a, 'pred_boxes': b} for a, b in zip(outputs_class[:-1], outputs_coord[:-1])]

    # ------------------------------------------------------------------ autograd path
    def _input_proj_autograd(self, l, src_nchw):
        """input_proj[l] (Conv2d + GroupNorm, deformable_detr.py:63-71) on kinet autograd
        Functions; src (B, C, h, w) NCHW (a channels-last view of an NHWC buffer) -> NCHW view."""
        conv, gn = self.input_proj[l][0], self.input_proj[l][1]
        x = src_nchw.float().permute(0, 2, 3, 1)
        if not x.is_contiguous():
            x = x.contiguous()
        B, h, w, C = x.shape
        d = conv.out_channels
        if conv.kernel_size == (1, 1) and conv.stride == (1, 1):
            y = A.linear(x.reshape(B * h * w, C), conv.weight.view(d, C), conv.bias)
        else:
            y = A.conv_nhwc(x, conv.weight, conv.bias, conv.stride[0], conv.padding[0])
            h, w = y.shape[1], y.shape[2]
        y = A.group_norm_nhwc(y.reshape(B, h * w, d), gn)
        return y.view(B, h, w, d).permute(0, 3, 1, 2)

    def _forward_reference(self, samples, targets=None, prev_features=None):
        """deformable_detr.py:139-275 op for op (training / autograd) in f32 on kinet autograd
        Functions: backbone convs, input projections, every Linear / LayerNorm / attention of
        the transformer and heads (kinet_amd/autograd.py), MSDeformAttnFunction (HIP fwd/bwd)."""
        body = self.backbone[0]
        xs = body.body.forward_autograd(samples.tensors.float())
        features_all = []
        for i in body.return_idx:
            x = xs[str(i)]
            features_all.append(NestedTensor(x, interp_mask(samples.mask, x.shape[-2:]), samples.sizes))
        # (cached per image geometry: the embedding is a function of the padding mask only)
        pos = [self.backbone._pos(f) for f in features_all]
        features = features_all[-3:]
        prev_features = features if prev_features is None else prev_features[-3:]
        frame_features = [prev_features, features] if self.multi_frame_attention else [features]
        src_list, mask_list, pos_list = [], [], []
        three_d = self.multi_frame_attention and self.multi_frame_encoding
        for frame, frame_feat in enumerate(frame_features):
            pos_list.extend([p[:, frame] for p in pos[-3:]] if three_d else pos[-3:])
            for l, feat in enumerate(frame_feat):
                src, mask = feat.decompose()
                src_list.append(self._input_proj_autograd(l, src))
                mask_list.append(mask)
            n_lv = self.num_feature_levels
            if n_lv > len(frame_feat):
                _len = len(frame_feat)
                for l in range(_len, n_lv):
                    src = self._input_proj_autograd(l, frame_feat[-1].tensors if l == _len else src_list[-1])
                    m = interp_mask(frame_feat[0].mask, src.shape[-2:])
                    pos_l = self.backbone._pos(NestedTensor(src, m, getattr(frame_feat[0], 'sizes', None)))
                    src_list.append(src)
                    mask_list.append(m)
                    pos_list.append(pos_l[:, frame] if three_d else pos_l)
        # padding known from the host-side image sizes (nested_tensor_from_tensor_list pads to the
        # largest image, so equal sizes mean all-False masks): no device -> host mask check
        size_sets = [getattr(samples, 'sizes', None)]
        if self.multi_frame_attention:
            size_sets.append(getattr(prev_features[0], 'sizes', None))
        padded = None if any(z is None for z in size_sets) else any(len(set(z)) > 1 for z in size_sets)
        hs, memory, init_reference, inter_references, _, _ = self.transformer(
            src_list, mask_list, pos_list, self.query_embed.weight, targets, padded=padded)
        outputs_classes, outputs_coords = [], []
        for lvl in range(hs.shape[0]):
            reference = init_reference if lvl == 0 else inter_references[lvl - 1]
            reference = inverse_sigmoid(reference)
            outputs_class = A.linear_module(hs[lvl], self.class_embed[lvl])
            tmp = self.bbox_embed[lvl](hs[lvl])
            if reference.shape[-1] == 4:
                tmp = tmp + reference
            else:
                tmp = torch.cat([tmp[..., :2] + reference, tmp[..., 2:]], -1)
            outputs_classes.append(outputs_class)
            outputs_coords.append(tmp.sigmoid())
        outputs_class = torch.stack(outputs_classes)
        outputs_coord = torch.stack(outputs_coords)
        out = {'pred_logits': outputs_class[-1], 'pred_boxes': outputs_coord[-1], 'hs_embed': hs[-1]}
        if self.aux_loss:
            out['aux_outputs'] = self._set_aux_loss(outputs_class, outputs_coord)
        B, _, c = memory.shape
        memory_slices, o = [], 0
        for s in src_list:
            _, _, h, w = s.shape
            memory_slices.append(memory[:, o:o + h * w].permute(0, 2, 1).view(B, c, h, w))
            o += h * w
        return out, targets, features_all, memory_slices, hs


class DeformablePostProcess(nn.Module):
    """deformable_detr.py:286-334."""

    @torch.no_grad()
    def forward(self, outputs, target_sizes, results_mask=None):
        out_logits, out_bbox = outputs['pred_logits'], outputs['pred_boxes']
        assert len(out_logits) == len(target_sizes)
        assert target_sizes.shape[1] == 2
        prob = out_logits.sigmoid()
        scores, labels = prob.max(-1)
        boxes = box_cxcywh_to_xyxy(out_bbox)
        img_h, img_w = target_sizes.unbind(1)
        scale_fct = torch.stack([img_w, img_h, img_w, img_h], dim=1)
        boxes = boxes * scale_fct[:, None, :]
        results = [{'scores': s, 'scores_no_object': 1 - s, 'labels': l, 'boxes': b}
                   for s, l, b in zip(scores, labels, boxes)]
        if results_mask is not None:
            for i, mask in enumerate(results_mask):
                for k, v in results[i].items():
                    results[i][k] = v[mask]
        return results


class PostProcess(nn.Module):
    """detr.py:891-934 (softmax classifier, the last class is no-object): used by the KineT
    model, which trains without focal loss."""

    @torch.no_grad()
    def forward(self, outputs, target_sizes, results_mask=None):
        out_logits, out_bbox = outputs['pred_logits'], outputs['pred_boxes']
        assert len(out_logits) == len(target_sizes)
        assert target_sizes.shape[1] == 2
        prob = F.softmax(out_logits, -1)
        scores, labels = prob[..., :-1].max(-1)
        boxes = box_cxcywh_to_xyxy(out_bbox)
        img_h, img_w = target_sizes.unbind(1)
        scale_fct = torch.stack([img_w, img_h, img_w, img_h], dim=1)
        boxes = boxes * scale_fct[:, None, :]
        results = [{'scores': s, 'labels': l, 'boxes': b, 'scores_no_object': s_n_o}
                   for s, l, b, s_n_o in zip(scores, labels, boxes, prob[..., -1])]
        if results_mask is not None:
            for i, mask in enumerate(results_mask):
                for k, v in results[i].items():
                    results[i][k] = v[mask]
        return results

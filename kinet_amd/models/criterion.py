"""Set criterion of the training path (src/trackformer/models/detr.py:566-888) with the
sigmoid focal loss (util/misc.py:634-665) and top-k accuracy (util/misc.py:542-557).

Losses 'labels' (focal or weighted CE with the track-query false-positive eos
re-weighting, detr.py:599-643 / :645-703), 'boxes' (L1 + GIoU, :719-751) and
'cardinality' (logging only, :705-717), plus the same set on every auxiliary decoder
output (:858-870).  `num_boxes` is all-reduced over the process group and averaged over
the world size (:841-846) -- the one scalar collective of the criterion.  These are small
ops over (batch, queries, classes) tensors; they run as torch ops on the predictions'
device (the MFMA-bound and gather-bound work is in the detector forward).
"""
import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from kinet_amd.models.misc import box_cxcywh_to_xyxy, generalized_box_iou, host_to_device


def sigmoid_focal_loss(inputs, targets, num_boxes, alpha: float = 0.25, gamma: float = 2):
    """util/misc.py:634-665 (reduction: mean over the last dim, sum, / num_boxes)."""
    prob = inputs.sigmoid()
    ce_loss = F.binary_cross_entropy_with_logits(inputs, targets, reduction="none")
    p_t = prob * targets + (1 - prob) * (1 - targets)
    loss = ce_loss * ((1 - p_t) ** gamma)
    if alpha >= 0:
        alpha_t = alpha * targets + (1 - alpha) * (1 - targets)
        loss = alpha_t * loss
    return loss.mean(1).sum() / num_boxes


@torch.no_grad()
def accuracy(output, target, topk=(1,)):
    """util/misc.py:542-557."""
    if target.numel() == 0:
        return [torch.zeros([], device=output.device)]
    maxk = max(topk)
    batch_size = target.size(0)
    _, pred = output.topk(maxk, 1, True, True)
    pred = pred.t()
    correct = pred.eq(target.view(1, -1).expand_as(pred))
    return [correct[:k].reshape(-1).float().sum(0).mul_(100.0 / batch_size) for k in topk]


def _world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


class SetCriterion(nn.Module):
    """detr.py:566-870."""

    def __init__(self, num_classes, matcher, weight_dict, eos_coef, losses, focal_loss, focal_alpha, focal_gamma,
                 tracking, track_query_false_positive_eos_weight):
        super().__init__()
        self.num_classes = num_classes
        self.matcher = matcher
        self.weight_dict = weight_dict
        self.eos_coef = eos_coef
        self.losses = losses
        empty_weight = torch.ones(self.num_classes + 1)
        empty_weight[-1] = self.eos_coef
        self.register_buffer('empty_weight', empty_weight)
        self.focal_loss = focal_loss
        self.focal_alpha = focal_alpha
        self.focal_gamma = focal_gamma
        self.tracking = tracking
        self.track_query_false_positive_eos_weight = track_query_false_positive_eos_weight

    @staticmethod
    def _get_src_permutation_idx(indices):
        batch_idx = torch.cat([torch.full_like(src, i) for i, (src, _) in enumerate(indices)])
        src_idx = torch.cat([src for (src, _) in indices])
        return batch_idx, src_idx

    def _target_classes(self, src_logits, targets, indices):
        idx = self._get_src_permutation_idx(indices)
        target_classes_o = torch.cat([t["labels"][J] for t, (_, J) in zip(targets, indices)]).to(src_logits.device)
        target_classes = torch.full(src_logits.shape[:2], self.num_classes, dtype=torch.int64, device=src_logits.device)
        target_classes[idx] = target_classes_o
        return idx, target_classes_o, target_classes

    def loss_labels(self, outputs, targets, indices, _, log=True):
        """detr.py:599-643: weighted CE; false-positive track queries lose the no-object
        down-weighting and count as class 0 in the normaliser."""
        src_logits = outputs['pred_logits']
        idx, target_classes_o, target_classes = self._target_classes(src_logits, targets, indices)
        empty_weight = self.empty_weight.to(src_logits.device)
        loss_ce = F.cross_entropy(src_logits.transpose(1, 2), target_classes, weight=empty_weight, reduction='none')
        if self.tracking and self.track_query_false_positive_eos_weight:
            for i, target in enumerate(targets):
                if 'track_query_boxes' in target:
                    fp = target['track_queries_fal_pos_mask'].to(src_logits.device)
                    loss_ce[i, fp] *= 1 / self.eos_coef
                    target_classes = target_classes.clone()
                    target_classes[i, fp] = 0
        loss_ce = loss_ce.sum() / empty_weight[target_classes].sum()
        losses = {'loss_ce': loss_ce}
        if log:
            losses['class_error'] = 100 - accuracy(src_logits[idx], target_classes_o)[0]
        return losses

    def loss_labels_focal(self, outputs, targets, indices, num_boxes, log=True):
        """detr.py:645-703."""
        src_logits = outputs['pred_logits']
        idx, target_classes_o, target_classes = self._target_classes(src_logits, targets, indices)
        onehot = torch.zeros([src_logits.shape[0], src_logits.shape[1], src_logits.shape[2] + 1],
                             dtype=src_logits.dtype, layout=src_logits.layout, device=src_logits.device)
        onehot.scatter_(2, target_classes.unsqueeze(-1), 1)
        onehot = onehot[:, :, :-1]
        loss_ce = sigmoid_focal_loss(src_logits, onehot, num_boxes, alpha=self.focal_alpha, gamma=self.focal_gamma)
        loss_ce = loss_ce * src_logits.shape[1]
        losses = {'loss_ce': loss_ce}
        if log:
            losses['class_error'] = 100 - accuracy(src_logits[idx], target_classes_o)[0]
        return losses

    @torch.no_grad()
    def loss_cardinality(self, outputs, targets, indices, num_boxes):
        """detr.py:705-717."""
        pred_logits = outputs['pred_logits']
        device = pred_logits.device
        tgt_lengths = host_to_device([len(v["labels"]) for v in targets], torch.long, device)
        card_pred = (pred_logits.argmax(-1) != pred_logits.shape[-1] - 1).sum(1)
        return {'cardinality_error': F.l1_loss(card_pred.float(), tgt_lengths.float())}

    def loss_boxes(self, outputs, targets, indices, num_boxes):
        """detr.py:719-751."""
        idx = self._get_src_permutation_idx(indices)
        src_boxes = outputs['pred_boxes'][idx]
        target_boxes = torch.cat([t['boxes'][i] for t, (_, i) in zip(targets, indices)], dim=0).to(src_boxes.device)
        loss_bbox = F.l1_loss(src_boxes, target_boxes, reduction='none')
        loss_giou = 1 - torch.diag(generalized_box_iou(box_cxcywh_to_xyxy(src_boxes), box_cxcywh_to_xyxy(target_boxes),
                                                       self.deferred_checks if src_boxes.is_cuda else None))
        return {'loss_bbox': loss_bbox.sum() / num_boxes, 'loss_giou': loss_giou.sum() / num_boxes}

    def get_loss(self, loss, outputs, targets, indices, num_boxes, **kwargs):
        loss_map = {'labels': self.loss_labels_focal if self.focal_loss else self.loss_labels,
                    'cardinality': self.loss_cardinality, 'boxes': self.loss_boxes}
        if loss not in loss_map:
            raise NotImplementedError(f'loss {loss} is outside the detection hot path')
        return loss_map[loss](outputs, targets, indices, num_boxes, **kwargs)

    def num_boxes(self, outputs, targets):
        """detr.py:841-846: total target count, summed over ranks, averaged, >= 1 (a host
        number on one rank: no device round trip)."""
        n = sum(len(t["labels"]) for t in targets)
        if _world_size() < 2:
            return float(max(n, 1))
        n = torch.as_tensor([n], dtype=torch.float, device=next(iter(outputs.values())).device)
        dist.all_reduce(n)
        return torch.clamp(n / _world_size(), min=1).item()

    def match(self, output_sets, targets):
        """The matcher's indices for every output set, moved to the predictions' device in ONE
        non-blocking copy (the losses index device tensors with them; the reference indexes
        with host tensors, one implicit copy per sample and loss)."""
        from kinet_amd.models.training import glue_timer, to_device
        with glue_timer():
            return self._match(output_sets, targets, to_device)

    def _match(self, output_sets, targets, to_device):
        if hasattr(self.matcher, 'match_many'):
            host = self.matcher.match_many(output_sets, targets)
        else:
            host = [self.matcher(o, targets) for o in output_sets]
        device = output_sets[0]['pred_logits'].device
        flat = [t for per_set in host for pair in per_set for t in pair]
        if device.type != 'cuda' or not flat:
            return host
        dev = to_device(torch.cat([t.long() for t in flat]), device).split([len(t) for t in flat])
        it = iter(dev)
        return [[(next(it), next(it)) for _ in per_set] for per_set in host]

    deferred_checks = None
    # opt-in (the training step sets it around its criterion call): collect the GIoU
    # degenerate-box flags instead of asserting them in loss_boxes; every other caller keeps
    # the reference's immediate assert (util/box_ops.py:44-45)
    defer_box_checks = False

    def pop_deferred_checks(self):
        """The GIoU degenerate-box flags of the last forward as one device bool (None if none):
        the training step asserts it at its loss-finiteness sync instead of two syncs per
        loss_boxes call (util/box_ops.py:44-45)."""
        c, self.deferred_checks = self.deferred_checks, None
        return torch.stack(c).all() if c else None

    def forward(self, outputs, targets):
        self.deferred_checks = [] if self.defer_box_checks else None
        outputs_without_aux = {k: v for k, v in outputs.items() if k != 'aux_outputs'}
        aux = list(outputs.get('aux_outputs', []))
        all_indices = self.match([outputs_without_aux] + aux, targets)
        indices = all_indices[0]
        num_boxes = self.num_boxes(outputs, targets)
        losses = {}
        for loss in self.losses:
            losses.update(self.get_loss(loss, outputs, targets, indices, num_boxes))
        for i, aux_outputs in enumerate(aux):
            indices = all_indices[i + 1]
            for loss in self.losses:
                kwargs = {'log': False} if loss == 'labels' else {}
                l_dict = self.get_loss(loss, aux_outputs, targets, indices, num_boxes, **kwargs)
                losses.update({k + f'_{i}': v for k, v in l_dict.items()})
        return losses


def build_criterion(args, num_classes, matcher):
    """models/__init__.py:125-161 (no masks, no two-stage on this path)."""
    weight_dict = {'loss_ce': args.cls_loss_coef, 'loss_bbox': args.bbox_loss_coef, 'loss_giou': args.giou_loss_coef}
    if args.aux_loss:
        aux = {}
        for i in range(args.dec_layers - 1):
            aux.update({k + f'_{i}': v for k, v in weight_dict.items()})
        weight_dict.update(aux)
    return SetCriterion(num_classes, matcher=matcher, weight_dict=weight_dict, eos_coef=args.eos_coef,
                        losses=['labels', 'boxes', 'cardinality'], focal_loss=args.focal_loss,
                        focal_alpha=args.focal_alpha, focal_gamma=args.focal_gamma, tracking=args.tracking,
                        track_query_false_positive_eos_weight=args.track_query_false_positive_eos_weight)

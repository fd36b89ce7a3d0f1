"""Hungarian matcher of the training path (src/trackformer/models/matcher.py:86-202,
build_matcher :685-712).

The cost matrix (focal or softmax class cost, L1 box cost, -GIoU) is built on the device
where the predictions live; the linear sum assignment stays on the host
(scipy.optimize.linear_sum_assignment, as in the reference, matcher.py:198) -- the
north_star keeps the matcher host-side.  Track queries are forced onto the targets whose
track ids they carry and false-positive track queries are made unmatchable exactly as
matcher.py:177-196 does.
"""
import numpy as np
import torch
from scipy.optimize import linear_sum_assignment
from torch import nn

from kinet_amd.models.misc import box_cxcywh_to_xyxy, generalized_box_iou


class HungarianMatcher(nn.Module):
    """matcher.py:86-202."""

    def __init__(self, cost_class: float = 1, cost_bbox: float = 1, cost_giou: float = 1,
                 focal_loss: bool = False, focal_alpha: float = 0.25, focal_gamma: float = 2.0):
        super().__init__()
        self.cost_class = cost_class
        self.cost_bbox = cost_bbox
        self.cost_giou = cost_giou
        self.focal_loss = focal_loss
        self.focal_alpha = focal_alpha
        self.focal_gamma = focal_gamma
        assert cost_class != 0 or cost_bbox != 0 or cost_giou != 0, "all costs cant be 0"

    @torch.no_grad()
    def cost_matrix(self, outputs, targets):
        """(batch, num_queries, sum_targets) f32 cost on the predictions' device
        (matcher.py:135-171)."""
        batch_size, num_queries = outputs["pred_logits"].shape[:2]
        logits = outputs["pred_logits"].flatten(0, 1).float()
        out_prob = logits.sigmoid() if self.focal_loss else logits.softmax(-1)
        out_bbox = outputs["pred_boxes"].flatten(0, 1).float()
        tgt_ids = torch.cat([v["labels"] for v in targets]).to(logits.device)
        tgt_bbox = torch.cat([v["boxes"] for v in targets]).to(logits.device).float()
        if self.focal_loss:
            a, g = self.focal_alpha, self.focal_gamma
            neg_cost_class = (1 - a) * (out_prob ** g) * (-(1 - out_prob + 1e-8).log())
            pos_cost_class = a * ((1 - out_prob) ** g) * (-(out_prob + 1e-8).log())
            cost_class = pos_cost_class[:, tgt_ids] - neg_cost_class[:, tgt_ids]
        else:
            cost_class = -out_prob[:, tgt_ids]
        cost_bbox = torch.cdist(out_bbox, tgt_bbox, p=1)
        cost_giou = -generalized_box_iou(box_cxcywh_to_xyxy(out_bbox), box_cxcywh_to_xyxy(tgt_bbox))
        c = self.cost_bbox * cost_bbox + self.cost_class * cost_class + self.cost_giou * cost_giou
        return c.view(batch_size, num_queries, -1)

    @torch.no_grad()
    def forward(self, outputs, targets):
        cost_matrix = self.cost_matrix(outputs, targets).cpu()
        sizes = [len(v["boxes"]) for v in targets]
        offsets = np.cumsum([0] + sizes[:-1])
        for i, target in enumerate(targets):
            if 'track_query_match_ids' not in target:
                continue
            # matcher.py:179-196: false-positive track queries match nothing; a true track
            # query is forced onto its target (cost -1 there, inf elsewhere in row/column)
            fal_pos = target['track_queries_fal_pos_mask'].cpu()
            tq_mask = target['track_queries_mask'].cpu()
            match_ids = target['track_query_match_ids'].cpu()
            prop_i = 0
            for j in range(cost_matrix.shape[1]):
                if fal_pos[j]:
                    cost_matrix[i, j] = np.inf
                elif tq_mask[j]:
                    col = int(match_ids[prop_i]) + int(offsets[i])
                    prop_i += 1
                    cost_matrix[i, j] = np.inf
                    cost_matrix[i, :, col] = np.inf
                    cost_matrix[i, j, col] = -1
        indices = [linear_sum_assignment(c[i]) for i, c in enumerate(cost_matrix.split(sizes, -1))]
        return [(torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)) for i, j in indices]


def build_matcher(args):
    """matcher.py:685-712 -- the ordered-query matchers belong to the KineT model (§8(f))."""
    if getattr(args, 'used_ordered_queries', False):
        raise NotImplementedError('ordered-detection matchers belong to the KineT model, outside the hot path')
    return HungarianMatcher(cost_class=args.set_cost_class, cost_bbox=args.set_cost_bbox,
                            cost_giou=args.set_cost_giou, focal_loss=args.focal_loss,
                            focal_alpha=args.focal_alpha, focal_gamma=args.focal_gamma)

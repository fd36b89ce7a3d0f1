"""Hungarian matcher of the training path (src/trackformer/models/matcher.py:86-202,
build_matcher :685-712).

The cost matrix (focal or softmax class cost, L1 box cost, -GIoU) is built batched on the
device where the predictions live and crosses to the host in ONE copy (one for all of the
criterion's final + auxiliary output sets: `match_many`); the linear sum
assignment stays on the host (scipy.optimize.linear_sum_assignment, as in the reference,
matcher.py:198) -- the north_star keeps the matcher host-side.  Track queries are forced
onto the targets whose track ids they carry and false-positive track queries are made
unmatchable with the same result as matcher.py:177-196, but as whole-row / whole-column
tensor writes instead of the reference's Python loop over every query (which, with the
masks on the GPU, synchronises once per query).
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
    def cost_matrix(self, outputs, targets, checks=None):
        """(batch, num_queries, sum_targets) f32 cost on the predictions' device
        (matcher.py:135-171).  checks: see misc.generalized_box_iou."""
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
        cost_giou = -generalized_box_iou(box_cxcywh_to_xyxy(out_bbox), box_cxcywh_to_xyxy(tgt_bbox), checks)
        c = self.cost_bbox * cost_bbox + self.cost_class * cost_class + self.cost_giou * cost_giou
        return c.view(batch_size, num_queries, -1)

    @torch.no_grad()
    def forward(self, outputs, targets):
        return self.match_many([outputs], targets)[0]

    @torch.no_grad()
    def match_many(self, outputs_list, targets):
        """Indices of several output sets against the same targets -- the criterion's final
        and auxiliary decoder outputs (detr.py:819-868 calls the matcher once per set) --
        with ONE device->host synchronisation for all their cost matrices and the track-query
        masks / match ids (to_host), instead of one per set."""
        from kinet_amd.models.training import to_host
        sizes = [len(v["boxes"]) for v in targets]
        offsets = np.cumsum([0] + sizes[:-1])
        tq = [i for i, t in enumerate(targets) if 'track_query_match_ids' in t]
        shapes = {(tuple(o["pred_logits"].shape), tuple(o["pred_boxes"].shape)) for o in outputs_list}
        # the GIoU degenerate-box asserts (util/box_ops.py:44-45) ride on the cost matrix's one host
        # copy instead of synchronising twice per generalized_box_iou call
        checks = []
        if len(outputs_list) > 1 and len(shapes) == 1:
            # every set in one cost computation (the same element-wise ops and per-pair L1 /
            # GIoU, S x fewer launches): rows (set, image, query)
            S, (bsz, nq) = len(outputs_list), outputs_list[0]["pred_logits"].shape[:2]
            both = {k: torch.cat([o[k] for o in outputs_list]) for k in ("pred_logits", "pred_boxes")}
            costs = self.cost_matrix(both, targets, checks).view(S, bsz, nq, -1)
        else:
            costs = torch.stack([self.cost_matrix(o, targets, checks) for o in outputs_list])
        has_chk = bool(checks) and costs.is_cuda
        extra = [torch.stack(checks)] if has_chk else []
        if tq:
            masks = torch.stack([torch.stack([targets[i]['track_queries_fal_pos_mask'],
                                              targets[i]['track_queries_mask']]).to(costs.device) for i in tq])
            ids = [targets[i]['track_query_match_ids'] for i in tq]
            counts = [len(m) for m in ids]
            extra += [masks, torch.cat([m.to(costs.device).long() for m in ids]) if sum(counts)
                      else torch.zeros(0, dtype=torch.long)]
        host = to_host(costs, *extra)
        costs = host[0]
        if has_chk:
            assert bool(host[1].all()), 'degenerate boxes (util/box_ops.py:44-45)'
            host = host[:1] + host[2:]
        elif checks:
            assert all(bool(c) for c in checks)
        forced = []
        if tq:
            masks, ids = host[1], host[2].split(counts)
            # matcher.py:177-196 without its per-query Python loop: a false-positive track
            # query matches nothing (row = inf); the k-th true track query is forced onto
            # target match_ids[k] (its row and that column inf, -1 at the pair)
            for n, i in enumerate(tq):
                fal_pos, tq_mask = masks[n, 0], masks[n, 1]
                rows = (tq_mask & ~fal_pos).nonzero().flatten()
                cols = ids[n][:len(rows)].long() + int(offsets[i])
                forced.append((i, fal_pos | tq_mask, rows, cols))
        result = []
        for cost_matrix in costs:
            for i, rowmask, rows, cols in forced:
                cost_matrix[i, rowmask] = np.inf
                cost_matrix[i, :, cols] = np.inf
                cost_matrix[i, rows, cols] = -1
            indices = [linear_sum_assignment(c[i]) for i, c in enumerate(cost_matrix.split(sizes, -1))]
            result.append([(torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64))
                           for i, j in indices])
        return result


def build_matcher(args):
    """matcher.py:685-712 -- the ordered-query matchers belong to the KineT model (§8(f))."""
    if getattr(args, 'used_ordered_queries', False):
        raise NotImplementedError('ordered-detection matchers belong to the KineT model, outside the hot path')
    return HungarianMatcher(cost_class=args.set_cost_class, cost_bbox=args.set_cost_bbox,
                            cost_giou=args.set_cost_giou, focal_loss=args.focal_loss,
                            focal_alpha=args.focal_alpha, focal_gamma=args.focal_gamma)

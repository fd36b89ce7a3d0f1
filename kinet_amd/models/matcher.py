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


# ------------------------------------------------------------------ KineT (§8(f)2)
# The KineT model is trained to predict its input detections in order: query group k
# (n_assign consecutive object queries) answers input detection k.  These matchers first
# assign input detections to ground-truth boxes (L1 + GIoU LSA, kept below a fixed cost),
# then give each matched target the query group of its detection; track queries override
# the group for the targets they carry.  Host logic (LSA, small index arrays) on the
# device's cost values, as the reference.

def _cxcywh_cost(dets, tgts, w_bbox, w_giou):
    """w_bbox * L1 + w_giou * (-GIoU) between cxcywh box sets (matcher.py:253-261)."""
    return (w_bbox * torch.cdist(dets, tgts, p=1)
            - w_giou * generalized_box_iou(box_cxcywh_to_xyxy(dets), box_cxcywh_to_xyxy(tgts)))


class BasicBoxHungarianMatcher:
    """matcher.py:13-82: LSA between detections [n_det, 5|6] and the targets' boxes (L1 + GIoU,
    + a class-mismatch cost with use_class); returns (target indices, detection indices)."""

    def __init__(self, cost_class: float = 1, cost_bbox: float = 2, cost_giou: float = 2, use_class=False):
        self.cost_class, self.cost_bbox, self.cost_giou, self.use_class = cost_class, cost_bbox, cost_giou, use_class
        assert cost_class != 0 or cost_bbox != 0 or cost_giou != 0, "all costs cant be 0"

    def __call__(self, detections, target):
        out_bbox = detections[:, :4]
        cost = _cxcywh_cost(out_bbox, target["boxes"], self.cost_bbox, self.cost_giou)
        if self.use_class:
            cost = cost + self.cost_class * (target['labels'][None] != detections[:, 5, None]).to(torch.int32)
        rows, cols = linear_sum_assignment(cost.cpu())
        return torch.as_tensor(cols, dtype=torch.int64), torch.as_tensor(rows, dtype=torch.int64)


class _OrderedBase(nn.Module):
    def __init__(self, cost_class, cost_bbox, cost_giou, focal_loss, focal_alpha, focal_gamma):
        super().__init__()
        self.cost_class, self.cost_bbox, self.cost_giou = cost_class, cost_bbox, cost_giou
        self.focal_loss, self.focal_alpha, self.focal_gamma = focal_loss, focal_alpha, focal_gamma
        self.max_cost = - self.cost_giou * 0.1 + self.cost_bbox * 0.6      # (matcher.py:239)
        assert cost_class != 0 or cost_bbox != 0 or cost_giou != 0, "all costs cant be 0"

    def calculate_matching_detections(self, targets):
        """matcher.py:242-271: per image, LSA between the input detections and the targets,
        pairs kept when their cost is below max_cost -> (detection idx, target idx) int64."""
        out = []
        for tgt in targets:
            cost = _cxcywh_cost(tgt["detections"], tgt["boxes"], self.cost_bbox, self.cost_giou).cpu()
            r, c = linear_sum_assignment(cost)
            keep = cost.numpy()[r, c] < self.max_cost
            out.append((r[keep].astype(np.int64), c[keep].astype(np.int64)))
        return out


def _track_overrides(target, targets_idx, num_track_queries):
    """The positive track queries (track_queries_mask[j], j < num_track_queries) of one image:
    (j, target id) pairs with the reference's per-query indexing of track_query_match_ids
    (matcher.py:359-370 / :530-541)."""
    if 'track_query_match_ids' not in target:
        return None
    mask = target['track_queries_mask'][:num_track_queries].cpu().tolist()
    ids = target['track_query_match_ids'].cpu().tolist()
    return [(j, int(ids[j])) for j in range(num_track_queries) if mask[j]]


class OrderDetectionsMatcherTransformer1(_OrderedBase):
    """matcher.py:205-379: every query of a matched detection's group is matched to its target
    (n_assign predictions per target); a positive track query takes over all of its target's
    group entries, or is appended when its target was not matched through a detection."""

    def __init__(self, n_predictions, assignment_predictions, cost_class: float = 1, cost_bbox: float = 1,
                 cost_giou: float = 1, focal_loss: bool = False, focal_alpha: float = 0.25, focal_gamma: float = 2.0):
        super().__init__(cost_class, cost_bbox, cost_giou, focal_loss, focal_alpha, focal_gamma)
        assert n_predictions % assignment_predictions == 0, \
            "[ERROR] Invalid number of predictions/queries and assigned predictions per detection"
        self.n_predictions, self.n_assign = n_predictions, assignment_predictions
        self.max_predictions = n_predictions // assignment_predictions

    @torch.no_grad()
    def forward(self, outputs, targets):
        d2t = self.calculate_matching_detections(targets)
        num_queries = outputs["pred_logits"].shape[1]
        ntq = num_queries - self.n_predictions
        res = []
        for i, target in enumerate(targets):
            det, tgt = d2t[i]
            group = ntq + (det % self.max_predictions) * self.n_assign
            preds = (group[:, None] + np.arange(self.n_assign)[None]).reshape(-1)
            tgts = np.repeat(tgt, self.n_assign)
            ov = _track_overrides(target, tgts, ntq)
            if ov is not None:
                extra_p, extra_t = [], []
                for j, tid in ov:
                    hit = tgts == tid
                    if hit.any():
                        preds[hit] = j
                    else:
                        extra_p.append(j)
                        extra_t.append(tid)
                preds = np.concatenate([preds, np.array(extra_p, dtype=np.int64)])
                tgts = np.concatenate([tgts, np.array(extra_t, dtype=np.int64)])
            res.append((torch.as_tensor(preds, dtype=torch.int64), torch.as_tensor(tgts, dtype=torch.int64)))
        return res


class OrderDetectionsMatcherTransformer2(OrderDetectionsMatcherTransformer1):
    """matcher.py:381-550: the one query of a matched detection's group with the lowest
    prediction-target cost (focal / softmax class + L1 + GIoU, the HungarianMatcher cost;
    first minimum on ties) is matched to its target; positive track queries override or are
    appended as in Transformer1."""

    @torch.no_grad()
    def forward(self, outputs, targets):
        d2t = self.calculate_matching_detections(targets)
        batch_size, num_queries = outputs["pred_logits"].shape[:2]
        hm = HungarianMatcher(self.cost_class, self.cost_bbox, self.cost_giou, self.focal_loss, self.focal_alpha,
                              self.focal_gamma)
        cost = hm.cost_matrix(outputs, targets).cpu()
        sizes = [len(v["boxes"]) for v in targets]
        subs = cost.split(sizes, -1)
        ntq = num_queries - self.n_predictions
        res = []
        for i, target in enumerate(targets):
            det, tgt = d2t[i]
            group = ntq + (det % self.max_predictions) * self.n_assign
            preds = (group[:, None] + np.arange(self.n_assign)[None]).reshape(-1)
            tgts_rep = np.repeat(tgt, self.n_assign)
            cb = subs[i][i, torch.as_tensor(preds), torch.as_tensor(tgts_rep)].view(len(det), self.n_assign)
            best = (torch.argmin(cb, dim=1) + torch.as_tensor(group)).numpy().astype(np.int64)
            tgts = tgt.copy()
            ov = _track_overrides(target, tgts, ntq)
            if ov is not None:
                extra_p, extra_t = [], []
                for j, tid in ov:
                    hit = tgts == tid
                    if hit.any():
                        best[hit] = j
                    else:
                        extra_p.append(j)
                        extra_t.append(tid)
                best = np.concatenate([best, np.array(extra_p, dtype=np.int64)])
                tgts = np.concatenate([tgts, np.array(extra_t, dtype=np.int64)])
            res.append((torch.as_tensor(best, dtype=torch.int64), torch.as_tensor(tgts, dtype=torch.int64)))
        return res


class OrderDetectionsMatcherEncoder(_OrderedBase):
    """matcher.py:554-682: the encoder-only variant predicts its N input detections 1:1, so a
    matched detection's own query (after the track queries and the optional empty start
    token) is matched to its target; track queries come first: those whose target was not
    reached through a detection, then those that were, then the remaining detections."""

    def __init__(self, cost_class: float = 1, cost_bbox: float = 1, cost_giou: float = 1, focal_loss: bool = False,
                 focal_alpha: float = 0.25, focal_gamma: float = 2.0, use_empty_start=True, fix_track_pairing=False):
        super().__init__(cost_class, cost_bbox, cost_giou, focal_loss, focal_alpha, focal_gamma)
        self.start_detection_dim = 1 if use_empty_start else 0
        # reference defect (matcher.py:657-663, :667-676): the track-query predictions are listed
        # [not reached through a detection..., reached...] but their targets [reached...,
        # not reached...], so the two groups are paired crosswise whenever both are non-empty.
        # Kept by default (parity); fix_track_pairing=True pairs each track query with its own
        # target.
        self.fix_track_pairing = fix_track_pairing

    @torch.no_grad()
    def forward(self, outputs, targets):
        d2t = self.calculate_matching_detections(targets)
        ntq = targets[0]['track_query_hs_embeds_meta'].size()[0]
        res = []
        for i, target in enumerate(targets):
            det, tgt = d2t[i]
            if 'track_query_match_ids' in target:
                pm, tm, pu, tu, dm = [], [], [], [], []
                for j, tid in enumerate(target['track_query_match_ids'].cpu().tolist()):
                    tid = int(tid)
                    hit = np.nonzero(tgt == tid)[0]
                    if len(hit) == 0:
                        tu.append(tid)
                        pu.append(j)
                    else:
                        tm.append(tid)
                        pm.append(j)
                        dm.append(hit[0])
                tq_t = tu + tm if self.fix_track_pairing else tm + tu
                if len(det) == len(dm):
                    best = np.array(pu + pm, dtype=np.int64)
                    tgts = np.array(tq_t, dtype=np.int64)
                else:
                    rem = np.setdiff1d(np.arange(len(det)), np.array(dm, dtype=np.int64))
                    best = np.concatenate([np.array(pu + pm, dtype=np.int64),
                                           det[rem] + ntq + self.start_detection_dim])
                    tgts = np.concatenate([np.array(tq_t, dtype=np.int64), tgt[rem]])
            else:
                best, tgts = det + ntq + self.start_detection_dim, tgt
            res.append((torch.as_tensor(best, dtype=torch.int64), torch.as_tensor(tgts, dtype=torch.int64)))
        return res


def build_matcher(args):
    """matcher.py:685-712."""
    if getattr(args, 'used_ordered_queries', False):
        kw = dict(cost_class=args.set_cost_class, cost_bbox=args.set_cost_bbox, cost_giou=args.set_cost_giou,
                  focal_loss=args.focal_loss, focal_alpha=args.focal_alpha, focal_gamma=args.focal_gamma)
        if getattr(args, 'use_encoder_only', False):
            return OrderDetectionsMatcherEncoder(use_empty_start=args.use_empty_start, **kw)
        return OrderDetectionsMatcherTransformer2(args.num_queries, args.num_queries // args.max_number_detection, **kw)
    return HungarianMatcher(cost_class=args.set_cost_class, cost_bbox=args.set_cost_bbox,
                            cost_giou=args.set_cost_giou, focal_loss=args.focal_loss,
                            focal_alpha=args.focal_alpha, focal_gamma=args.focal_gamma)

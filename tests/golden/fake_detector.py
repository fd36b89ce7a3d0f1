"""Deterministic stand-in for the object detector in the tracker fixtures (test
infrastructure): per frame it returns pred_logits / pred_boxes / hs_embed for the K track
queries it is given (their boxes jittered, their embeddings perturbed) followed by Q object
queries, all drawn from a CPU generator seeded by (seed, frame) -- so the reference Tracker
(tests/golden/make_golden.py, CPU) and kinet_amd.tracker.Tracker (GPU) see identical
detector outputs whenever their track states agree."""
import torch


class FakeDetector(torch.nn.Module):
    def __init__(self, num_queries=30, num_classes=20, hidden=16, overflow_boxes=False, seed=0):
        super().__init__()
        self.num_queries = num_queries
        self.overflow_boxes = overflow_boxes
        self.num_classes, self.hidden, self.seed = num_classes, hidden, seed
        self.anchor = torch.nn.Parameter(torch.zeros(1))     # carries the device
        self.frame = 0

    def forward(self, img, targets=None, prev_features=None):
        g = torch.Generator().manual_seed(self.seed * 1000 + self.frame)
        self.frame += 1
        Q, C, d = self.num_queries, self.num_classes, self.hidden
        boxes = torch.cat([torch.rand(Q, 2, generator=g) * 0.8 + 0.1, torch.rand(Q, 2, generator=g) * 0.15 + 0.03], 1)
        logits = torch.randn(Q, C, generator=g) * 1.5 - 1.0
        logits[:, 0] += 1.0
        hs = torch.randn(Q, d, generator=g)
        if targets is not None and len(targets) and 'track_query_boxes' in targets[0]:
            tb = targets[0]['track_query_boxes'].detach().cpu().float()
            th = targets[0]['track_query_hs_embeds'].detach().cpu().float()
            K = tb.shape[0]
            tboxes = (tb + 0.01 * torch.randn(K, 4, generator=g)).clamp(0.01, 0.99)
            tlog = torch.randn(K, C, generator=g) - 2.0
            tlog[:, 0] = torch.randn(K, generator=g) * 1.5 + 0.5
            ths = th + 0.1 * torch.randn(K, d, generator=g)
            boxes, logits, hs = torch.cat([tboxes, boxes]), torch.cat([tlog, logits]), torch.cat([ths, hs])
        dev = self.anchor.device
        out = {'pred_logits': logits[None].to(dev), 'pred_boxes': boxes[None].to(dev), 'hs_embed': hs[None].to(dev)}
        return out, None, ['features of frame %d' % self.frame], None, None


TRACKER_CFGS = {
    # cfgs/track.yaml:28-49 as shipped
    'default': dict(public_detections=False, detection_obj_score_thresh=0.4, track_obj_score_thresh=0.4,
                    detection_nms_thresh=0.9, track_nms_thresh=0.9, steps_termination=1, prev_frame_dist=1,
                    inactive_patience=-1, reid_sim_threshold=0.0, reid_sim_only=False, reid_score_thresh=0.4,
                    reid_greedy_matching=False),
    # re-identification by embedding distance (LSA), tighter NMS, 2-step termination
    'reid_lsa': dict(public_detections=False, detection_obj_score_thresh=0.4, track_obj_score_thresh=0.45,
                     detection_nms_thresh=0.5, track_nms_thresh=0.5, steps_termination=2, prev_frame_dist=1,
                     inactive_patience=3, reid_sim_threshold=6.0, reid_sim_only=False, reid_score_thresh=0.6,
                     reid_greedy_matching=False),
    # public detections gated by IoU >= 0.5
    'public_iou': dict(public_detections='min_iou_0_5', detection_obj_score_thresh=0.4, track_obj_score_thresh=0.45,
                       detection_nms_thresh=0.5, track_nms_thresh=0.5, steps_termination=2, prev_frame_dist=1,
                       inactive_patience=3, reid_sim_threshold=6.0, reid_sim_only=False, reid_score_thresh=0.6,
                       reid_greedy_matching=False),
    # greedy centre-distance re-identification, public detections by centre distance
    'reid_greedy': dict(public_detections='center_distance', detection_obj_score_thresh=0.35,
                        track_obj_score_thresh=0.4, detection_nms_thresh=0.7, track_nms_thresh=0.7,
                        steps_termination=1, prev_frame_dist=1, inactive_patience=5, reid_sim_threshold=0.0,
                        reid_sim_only=False, reid_score_thresh=0.5, reid_greedy_matching=True),
}


def sequence_blobs(seed, frames, size=(480, 640), device='cpu'):
    """Blobs as track.py's loader yields them: img, orig_size, public dets (xyxy, image pixels)."""
    g = torch.Generator().manual_seed(10_000 + seed)
    h, w = size
    out = []
    for _ in range(frames):
        n = 12
        c = torch.rand(n, 2, generator=g) * torch.tensor([w * 0.8, h * 0.8]) + torch.tensor([w * 0.1, h * 0.1])
        wh = torch.rand(n, 2, generator=g) * torch.tensor([w * 0.15, h * 0.15]) + 10
        dets = torch.cat([c - wh / 2, c + wh / 2], 1)
        out.append({'img': torch.zeros(1, 3, 8, 8, device=device), 'orig_size': torch.tensor([[h, w]], device=device),
                    'dets': [dets]})
    return out


def flatten_results(results):
    """{track: {frame: {bbox, score, obj_ind}}} -> (ids (n, 3) [frame, track, obj_ind], vals (n, 5))."""
    rows = sorted((f, t, r) for t, fr in results.items() for f, r in fr.items())
    ids = torch.tensor([[f, t, int(r['obj_ind'])] for f, t, r in rows], dtype=torch.int64).reshape(-1, 3)
    vals = torch.tensor([list(r['bbox']) + [float(r['score'])] for f, t, r in rows], dtype=torch.float32).reshape(-1, 5)
    return ids, vals

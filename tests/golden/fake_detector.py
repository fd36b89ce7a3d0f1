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


# ---- TrackerKinematic (tracker.py:580-959) fixtures ------------------------------------------

class KinetBlobSample:
    """The NestedTensorKinet a KineT tracking loader yields (util/misc.py:445-455): detections and
    metadata of the frame; the tracker only moves it to the device and reads .detections (public
    detections; unused with public_detections False)."""

    def __init__(self, detections, metadata):
        self.detections, self.metadata = detections, metadata

    def to(self, device):
        return KinetBlobSample(self.detections.to(device), self.metadata.to(device))


class FakeKinetDetector(torch.nn.Module):
    """Deterministic stand-in for KinetTracking in the TrackerKinematic fixtures: per frame, for
    the K tracklet queries in targets[0]['track_query_hs_embeds_det'] it returns each trail's
    last relative box (cxcywh; the trail's last 4 values when the tracklets are not encoded, a
    generator draw when they are) jittered, then Q object queries -- all from a CPU generator
    seeded by (seed, frame), so the reference tracker (CPU) and kinet_amd's (GPU) see identical
    outputs whenever their track states agree.  Two classes: label 1 detections are dropped by
    the tracker (n_classes 1)."""

    def __init__(self, num_queries=30, num_classes=2, n_frames=5, encoded=False, overflow_boxes=False, seed=0):
        super().__init__()
        self.num_queries, self.num_classes, self.n_frames = num_queries, num_classes, n_frames
        self.encoded, self.overflow_boxes, self.seed = encoded, overflow_boxes, seed
        self.anchor = torch.nn.Parameter(torch.zeros(1))     # carries the device
        self.frame = 0

    def forward(self, samples, targets=None):
        g = torch.Generator().manual_seed(self.seed * 1000 + 77 + self.frame)
        self.frame += 1
        Q, C = self.num_queries, self.num_classes
        boxes = torch.cat([torch.rand(Q, 2, generator=g) * 0.8 + 0.1, torch.rand(Q, 2, generator=g) * 0.15 + 0.03], 1)
        logits = torch.randn(Q, C, generator=g) * 1.5 - 0.5
        trk = targets[0]['track_query_hs_embeds_det'] if targets else None
        K = trk.shape[0] if trk is not None and trk.dim() == 2 else 0
        if K:
            if self.encoded:
                last = torch.cat([torch.rand(K, 2, generator=g) * 0.8 + 0.1,
                                  torch.rand(K, 2, generator=g) * 0.15 + 0.03], 1)
            else:
                last = trk.detach().cpu().float().view(K, self.n_frames, 4)[:, -1]
            tboxes = (last + 0.01 * torch.randn(K, 4, generator=g)).clamp(0.01, 0.99)
            tlog = torch.randn(K, C, generator=g) - 2.0
            tlog[:, 0] = torch.randn(K, generator=g) * 1.5 + 1.2
            boxes, logits = torch.cat([tboxes, boxes]), torch.cat([tlog, logits])
        dev = self.anchor.device
        out = {'pred_logits': logits[None].to(dev), 'pred_boxes': boxes[None].to(dev),
               'hs_embed': torch.zeros(1, boxes.shape[0], 8, device=dev)}
        return out, targets, ['features of frame %d' % self.frame], None, None


KINEMATIC_CFGS = {
    # cfgs/track_kinet.yaml:28-51 as shipped
    'kinet': dict(public_detections=False, detection_obj_score_thresh=0.75, track_obj_score_thresh=0.8,
                  detection_nms_thresh=0.9, track_nms_thresh=0.0, steps_termination=2, prev_frame_dist=1,
                  inactive_patience=5, reid_sim_threshold=0.0, reid_sim_only=False, reid_score_thresh=0.4,
                  reid_greedy_matching=False, n_classes=1),
    # lower thresholds, track NMS on, 1-step termination, short patience
    'kinet_nms': dict(public_detections=False, detection_obj_score_thresh=0.55, track_obj_score_thresh=0.6,
                      detection_nms_thresh=0.5, track_nms_thresh=0.5, steps_termination=1, prev_frame_dist=1,
                      inactive_patience=2, reid_sim_threshold=0.0, reid_sim_only=False, reid_score_thresh=0.45,
                      reid_greedy_matching=False, n_classes=1),
}


def kinematic_args(encoded=False):
    """The obj_detect_args fields TrackerKinematic reads (cfgs/train_kinet.yaml: 5 previous frames,
    identity tracklet encoding; encoded=True: sine encoding with 8 features)."""
    from argparse import Namespace
    return Namespace(use_class=False, use_empty_start=False, track_prev_frame_range=5,
                     use_encoding_tracklets=encoded, encoding_dim_tracklets=8)


class _Padded:
    """(tensors, mask) with .to(device): the NestedTensor of util/misc.py:407-443."""

    def __init__(self, tensors, mask):
        self.tensors, self.mask = tensors, mask

    def to(self, device):
        return _Padded(self.tensors.to(device), self.mask.to(device))


def kinematic_blobs(seed, frames, size=(480, 640), device='cpu'):
    """Blobs as track.py's KineT loader yields them: (NestedTensorKinet sample of 12 detections
    (cxcywh-like in [0, 1]) + 1 metadata value each, [labels with orig_size])."""
    g = torch.Generator().manual_seed(20_000 + seed)
    h, w = size
    out = []
    for _ in range(frames):
        dets = torch.rand(1, 12, 4, generator=g)
        meta = torch.rand(1, 12, 1, generator=g)
        mask = torch.zeros(1, 12, dtype=torch.bool)
        out.append((KinetBlobSample(_Padded(dets, mask).to(device), _Padded(meta, mask).to(device)),
                    [{'orig_size': torch.tensor([h, w], device=device)}]))
    return out

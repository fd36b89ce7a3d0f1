"""Online multi-object tracker over the kinet_amd detector: the reference's
`Tracker` (src/trackformer/models/tracker.py:18-562, `Track` :1056-1130) with the same
constructor, `reset()`, `step(blob)` and `get_results()`, so src/track.py drives it unchanged
(track.py:127-214: one `step` per frame, results {track_id: {frame: {'bbox', 'score',
'obj_ind'}}}).

Per frame (tracker.py:269-557): the active + inactive tracks become track queries (their
last box, cxcywh normalised by the image size, and their last decoder embedding); one
detector forward with the previous frame's features; post-process; track keep / terminate /
re-identify by score; track NMS; new detections above threshold (optionally gated by public
detections) are re-identified against inactive tracks (embedding-distance LSA) or start new
tracks; detection NMS; results.  Thresholds come from the reference's `tracker_cfg`
(cfgs/track.yaml:28-49).

MI355X-side choices: the detector, post-process, clipping, thresholding and NMS
(kernels.nms, a one-workgroup HIP kernel with torchvision.ops.nms semantics) run on the GPU;
the track bookkeeping is host Python as in the reference, fed by ONE batched device->host
copy of the small per-frame decision arrays instead of a sync per track.  Segmentation masks
and attention maps are outside the detection hot path (generate_attention_maps asserts in
the reference for Deformable DETR, tracker.py:38-40).
"""
from collections import deque

import numpy as np
import torch
from scipy.optimize import linear_sum_assignment

from kinet_amd import kernels as K
from kinet_amd.models.misc import box_xyxy_to_cxcywh


def clip_boxes_to_image(boxes, size):
    """torchvision.ops.clip_boxes_to_image: x to [0, w], y to [0, h]; size = (h, w)."""
    h, w = size[0], size[1]
    x = boxes[..., 0::2].clamp(min=0, max=w)
    y = boxes[..., 1::2].clamp(min=0, max=h)
    return torch.stack([x[..., 0], y[..., 0], x[..., 1], y[..., 1]], -1)


def box_iou(boxes1, boxes2):
    """IoU matrix of xyxy boxes (torchvision.ops.box_iou)."""
    a1 = (boxes1[:, 2] - boxes1[:, 0]) * (boxes1[:, 3] - boxes1[:, 1])
    a2 = (boxes2[:, 2] - boxes2[:, 0]) * (boxes2[:, 3] - boxes2[:, 1])
    lt = torch.max(boxes1[:, None, :2], boxes2[:, :2])
    rb = torch.min(boxes1[:, None, 2:], boxes2[:, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (a1[:, None] + a2 - inter)


class Track:
    """tracker.py:1056-1130."""

    def __init__(self, pos, score, track_id, hs_embed, obj_ind, pos_rel=None, mask=None, attention_map=None):
        self.id = track_id
        self.pos = pos
        self.last_pos = deque([pos.clone()])
        self.last_pos_relative = deque([-1] if pos_rel is None else [pos_rel.clone()])
        self.score = score
        self.ims = deque([])
        self.count_inactive = 0
        self.count_termination = 0
        self.gt_id = None
        self.hs_embed = [hs_embed]
        self.mask = mask
        self.attention_map = attention_map
        self.obj_ind = obj_ind

    def has_positive_area(self):
        return bool(self.pos[2] > self.pos[0] and self.pos[3] > self.pos[1])

    def repeat_last_pos(self):
        self.last_pos.append(self.last_pos[-1])
        self.last_pos_relative.append(self.last_pos_relative[-1])

    def reset_last_pos(self, clear_relative=False):
        """tracker.py:1120-1124.  The reference also clears last_pos_relative, after which its
        repeat_last_pos raises IndexError on the next frame the track is not re-detected
        (tracker.py:1110-1114); this build keeps that list by default.  clear_relative=True
        (tracker cfg `reference_clear_last_pos_relative`) reproduces the reference exactly,
        defect included."""
        self.last_pos.clear()
        if clear_relative:
            self.last_pos_relative.clear()
        self.last_pos.append(self.pos.clone())


class Tracker:
    """tracker.py:18-562 (image detector path)."""

    def __init__(self, obj_detector, obj_detector_post, tracker_cfg, generate_attention_maps=False, logger=None,
                 verbose=False):
        if generate_attention_maps:
            raise NotImplementedError('attention maps need a vanilla-DETR decoder (tracker.py:38-40)')
        self.obj_detector = obj_detector
        self.obj_detector_post = obj_detector_post
        self.detection_obj_score_thresh = tracker_cfg['detection_obj_score_thresh']
        self.track_obj_score_thresh = tracker_cfg['track_obj_score_thresh']
        self.detection_nms_thresh = tracker_cfg['detection_nms_thresh']
        self.track_nms_thresh = tracker_cfg['track_nms_thresh']
        self.public_detections = tracker_cfg['public_detections']
        self.inactive_patience = float(tracker_cfg['inactive_patience'])
        self.reid_sim_threshold = tracker_cfg['reid_sim_threshold']
        self.reid_sim_only = tracker_cfg['reid_sim_only']
        self.generate_attention_maps = False
        self.reid_score_thresh = tracker_cfg['reid_score_thresh']
        self.reid_greedy_matching = tracker_cfg['reid_greedy_matching']
        self.prev_frame_dist = tracker_cfg['prev_frame_dist']
        self.steps_termination = tracker_cfg['steps_termination']
        # compatibility switch for a reference defect (Track.reset_last_pos): False = keep the
        # relative-position history on re-identification (default), True = clear it as the
        # reference does (its next repeat_last_pos then raises IndexError)
        self.reference_clear_last_pos_relative = bool(tracker_cfg.get('reference_clear_last_pos_relative', False))
        self._logger = logger if logger is not None else (lambda *a: None)
        self._verbose = verbose

    @property
    def num_object_queries(self):
        return self.obj_detector.num_queries

    @property
    def device(self):
        return next(self.obj_detector.parameters()).device

    def reset(self, hard=True):
        self.tracks = []
        self.inactive_tracks = []
        self._prev_features = deque([None], maxlen=self.prev_frame_dist)
        if hard:
            self.track_num = 0
            self.results = {}
            self.frame_index = 0
            self.num_reids = 0

    def get_results(self):
        return self.results

    # ------------------------------------------------------------------ bookkeeping
    def _prune_inactive(self):
        """tracker.py:274-277 / :216-219 (one batched positive-area check)."""
        if not self.inactive_tracks:
            return
        pos = torch.stack([t.pos for t in self.inactive_tracks]).cpu()
        ok = ((pos[:, 2] > pos[:, 0]) & (pos[:, 3] > pos[:, 1])).tolist()
        self.inactive_tracks = [t for t, o in zip(self.inactive_tracks, ok)
                                if o and t.count_inactive <= self.inactive_patience]

    def move_tracks_to_inactive(self, inactive_tracks):
        self.tracks = [t for t in self.tracks if t not in inactive_tracks]
        for track in inactive_tracks:
            track.repeat_last_pos()
        self.inactive_tracks += inactive_tracks

    def add_tracks(self, pos, scores, hs_embeds, indices):
        new_track_ids = []
        for i in range(len(pos)):
            self.tracks.append(Track(pos[i], scores[i], self.track_num + i, hs_embeds[i], indices[i]))
            new_track_ids.append(self.track_num + i)
        self.track_num += len(new_track_ids)
        if new_track_ids:
            self._logger(f'INIT TRACK IDS (detection_obj_score_thresh={self.detection_obj_score_thresh}): '
                         f'{new_track_ids}')
        return new_track_ids

    def public_detections_mask(self, new_det_boxes, public_det_boxes):
        """tracker.py:127-170."""
        n = new_det_boxes.size(0)
        if not self.public_detections:
            return torch.ones(n, dtype=torch.bool, device=self.device)
        if not len(public_det_boxes) or not n:
            return torch.zeros(n, dtype=torch.bool, device=self.device)
        mask = torch.zeros(n, dtype=torch.bool)
        if self.public_detections == 'center_distance':
            nb = new_det_boxes.cpu()
            item_size = ((nb[:, 2] - nb[:, 0]) * (nb[:, 3] - nb[:, 1])).numpy().astype(np.float32)
            a = box_xyxy_to_cxcywh(nb).numpy()[:, :2]
            b = box_xyxy_to_cxcywh(public_det_boxes.cpu()).numpy()[:, :2]
            dist3 = ((a.reshape(-1, 1, 2) - b.reshape(1, -1, 2)) ** 2).sum(axis=2)
            for j in range(len(public_det_boxes)):
                i = dist3[:, j].argmin()
                if dist3[i, j] < item_size[i]:
                    dist3[i, :] = 1e18
                    mask[i] = True
        elif self.public_detections == 'min_iou_0_5':
            iou = box_iou(new_det_boxes, public_det_boxes.to(self.device)).cpu()
            for j in range(len(public_det_boxes)):
                i = iou[:, j].argmax()
                if iou[i, j] >= 0.5:
                    iou[i, :] = 0
                    mask[i] = True
        else:
            raise NotImplementedError(self.public_detections)
        return mask.to(self.device)

    def reid(self, new_det_boxes, new_det_scores, new_det_hs_embeds):
        """tracker.py:172-267: re-identify inactive tracks with the new detections."""
        self._prune_inactive()
        n = new_det_boxes.size(0)
        if not self.inactive_tracks or not n:
            return torch.ones(n, dtype=torch.bool, device=self.device)
        if self.reid_greedy_matching:
            nb = box_xyxy_to_cxcywh(new_det_boxes).cpu().numpy()
            ib = box_xyxy_to_cxcywh(torch.stack([t.pos for t in self.inactive_tracks])).cpu().numpy()
            dist_mat = ((ib[:, :2].reshape(-1, 1, 2) - nb[:, :2].reshape(1, -1, 2)) ** 2).sum(axis=2)
            track_size = ib[:, 2] * ib[:, 3]
            item_size = nb[:, 2] * nb[:, 3]
            invalid = (dist_mat > track_size.reshape(-1, 1)) + (dist_mat > item_size.reshape(1, -1))
            dist_mat = dist_mat + invalid * 1e18
            matched = []
            for i in range(dist_mat.shape[0]):
                j = dist_mat[i].argmin()
                if dist_mat[i][j] < 1e16:
                    dist_mat[:, j] = 1e18
                    dist_mat[i, j] = 0.0
                    matched.append([i, j])
            matched = np.array(matched, np.int32).reshape(-1, 2)
            rows, cols = matched[:, 0], matched[:, 1]
        else:
            # F.pairwise_distance(track_sim, det_sim): ||x - y + 1e-6||_2, as one batched op
            sims = torch.stack([t.hs_embed[-1] for t in self.inactive_tracks])
            dist_mat = (sims[:, None, :] - new_det_hs_embeds[None, :, :] + 1e-6).norm(dim=-1).cpu().numpy()
            rows, cols = linear_sum_assignment(dist_mat)
        assigned, remove_inactive = [], []
        for r, c in zip(rows, cols):
            if dist_mat[r, c] <= self.reid_sim_threshold:
                track = self.inactive_tracks[r]
                self._logger(f'REID: track.id={track.id} - count_inactive={track.count_inactive} - '
                             f'to_inactive_frame={self.frame_index - track.count_inactive}')
                track.count_inactive = 0
                track.pos = new_det_boxes[c]
                track.score = new_det_scores[c]
                track.hs_embed.append(new_det_hs_embeds[c])
                track.reset_last_pos(self.reference_clear_last_pos_relative)
                assigned.append(int(c))
                remove_inactive.append(track)
                self.tracks.append(track)
                self.num_reids += 1
        for track in remove_inactive:
            self.inactive_tracks.remove(track)
        mask = torch.ones(n, dtype=torch.bool)
        for c in assigned:
            mask[c] = False
        return mask.to(self.device)

    # ------------------------------------------------------------------ one frame
    @torch.no_grad()
    def step(self, blob):
        """tracker.py:269-557."""
        self._prune_inactive()
        self._logger(f'FRAME: {self.frame_index + 1}')
        for track in self.tracks:
            track.last_pos.append(track.pos.clone())
        img = blob['img'].to(self.device)
        orig_size = blob['orig_size'].to(self.device)
        Q = self.num_object_queries

        target = None
        prev = self.tracks + self.inactive_tracks
        num_prev_track = len(prev)
        if num_prev_track:
            boxes = box_xyxy_to_cxcywh(torch.stack([t.pos for t in prev]).float())
            hw = orig_size[0].float()
            boxes = boxes / torch.stack([hw[1], hw[0], hw[1], hw[0]])
            target = [{'track_query_boxes': boxes,
                       'image_id': torch.tensor([1], device=self.device),
                       'track_query_hs_embeds': torch.stack([t.hs_embed[-1] for t in prev])}]

        outputs, _, features, _, _ = self.obj_detector(img, target, self._prev_features[0])
        hs_embeds = outputs['hs_embed'][0]
        result = self.obj_detector_post['bbox'](outputs, orig_size)[0]
        boxes = result['boxes'] if self.obj_detector.overflow_boxes else clip_boxes_to_image(result['boxes'],
                                                                                              orig_size[0])
        scores, labels = result['scores'], result['labels']
        person = labels == 0
        # every threshold decision of this frame in ONE device -> host copy
        dec = torch.stack([scores > self.track_obj_score_thresh, scores > self.reid_score_thresh,
                           scores > self.detection_obj_score_thresh, person]).cpu()

        if num_prev_track:
            nt = num_prev_track
            track_keep = (dec[0, :nt] & dec[3, :nt]).tolist()
            reid_keep = (dec[1, :nt] & dec[3, :nt]).tolist()
            to_inactive, from_inactive = [], []
            for i, track in enumerate(self.tracks):
                if track_keep[i]:
                    track.score = scores[i]
                    track.hs_embed.append(hs_embeds[i])
                    track.pos = boxes[i]
                    track.count_termination = 0
                else:
                    track.count_termination += 1
                    if track.count_termination >= self.steps_termination:
                        to_inactive.append(track)
            for i, track in enumerate(self.inactive_tracks, start=len(self.tracks)):
                if reid_keep[i]:
                    track.score = scores[i]
                    track.hs_embed.append(hs_embeds[i])
                    track.pos = boxes[i]
                    from_inactive.append(track)
            if to_inactive:
                self._logger(f'NEW INACTIVE TRACK IDS (track_obj_score_thresh={self.track_obj_score_thresh}): '
                             f'{[t.id for t in to_inactive]}')
            self.num_reids += len(from_inactive)
            for track in from_inactive:
                self.inactive_tracks.remove(track)
                self.tracks.append(track)
            self.move_tracks_to_inactive(to_inactive)
            if self.track_nms_thresh and self.tracks:
                keep = set(K.nms(torch.stack([t.pos for t in self.tracks]),
                                 torch.stack([t.score for t in self.tracks]), self.track_nms_thresh).tolist())
                remove = [t for i, t in enumerate(self.tracks) if i not in keep]
                if remove:
                    self._logger(f'REMOVE TRACK IDS (track_nms_thresh={self.track_nms_thresh}): '
                                 f'{[t.id for t in remove]}')
                self.tracks = [t for t in self.tracks if t not in remove]

        # new detections (tracker.py:456-505)
        det_keep = (dec[2, -Q:] & dec[3, -Q:]).nonzero().flatten().to(self.device)
        new_det_boxes = boxes[-Q:][det_keep]
        new_det_scores = scores[-Q:][det_keep]
        new_det_hs_embeds = hs_embeds[-Q:][det_keep]
        new_det_indices = det_keep[:, None]                 # .float().nonzero() indices (:469)
        pub = self.public_detections_mask(new_det_boxes, blob['dets'][0] if 'dets' in blob else [])
        new_det_boxes, new_det_scores = new_det_boxes[pub], new_det_scores[pub]
        new_det_hs_embeds, new_det_indices = new_det_hs_embeds[pub], new_det_indices[pub]
        reid_mask = self.reid(new_det_boxes, new_det_scores, new_det_hs_embeds)
        new_det_boxes, new_det_scores = new_det_boxes[reid_mask], new_det_scores[reid_mask]
        new_det_hs_embeds, new_det_indices = new_det_hs_embeds[reid_mask], new_det_indices[reid_mask]
        new_track_ids = self.add_tracks(new_det_boxes, new_det_scores, new_det_hs_embeds, new_det_indices)

        if self.detection_nms_thresh and self.tracks:
            t_boxes = torch.stack([t.pos for t in self.tracks])
            t_scores = torch.stack([t.score for t in self.tracks]).clone()
            new_ids = set(new_track_ids)
            old = torch.tensor([t.id not in new_ids for t in self.tracks], device=self.device)
            t_scores[old] = float('inf')                       # existing tracks always win (:519)
            keep = set(K.nms(t_boxes, t_scores, self.detection_nms_thresh).tolist())
            remove = [t for i, t in enumerate(self.tracks) if i not in keep]
            if remove:
                self._logger(f'REMOVE TRACK IDS (detection_nms_thresh={self.detection_nms_thresh}): '
                             f'{[t.id for t in remove]}')
            self.tracks = [t for t in self.tracks if t not in remove]

        # results (tracker.py:529-552), one batched copy
        if self.tracks:
            pos = torch.stack([t.pos for t in self.tracks])
            if not self.obj_detector.overflow_boxes:
                pos = clip_boxes_to_image(pos, orig_size[0])
            packed = torch.cat([pos.float(), torch.stack([t.score for t in self.tracks]).float()[:, None],
                                torch.stack([t.obj_ind.reshape(()) for t in self.tracks]).float()[:, None]],
                               1).cpu().numpy()
            for track, row in zip(self.tracks, packed):
                self.results.setdefault(track.id, {})[self.frame_index] = {
                    'bbox': row[:4].copy(), 'score': np.float32(row[4]), 'obj_ind': int(row[5])}
        for t in self.inactive_tracks:
            t.count_inactive += 1
        self.frame_index += 1
        self._prev_features.append(features)
        if self.reid_sim_only:
            self.move_tracks_to_inactive(self.tracks)

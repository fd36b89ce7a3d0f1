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
import math
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


# ---------------------------------------------------------------------------------- KineT
# The kinematic tracker (tracker.py:580-959, TrackKinematic :961-1053) drives the KineT model
# (kinet_amd/models/kinet.py, `KinetTracking`) with each track's trail of the last n_frames
# relative boxes (+ its score trail) as tracklet queries.  As shipped the reference class
# cannot run past its first detections; the defects are fixed here by default and each is
# reproduced (same exception at the same step) when its name is in tracker_cfg
# ['reference_defects'] (tests/golden/make_golden.py gen_tracker_kinematic):
REFERENCE_DEFECTS = (
    # add_tracks passes `confidence=` (tracker.py:868), TrackKinematic.__init__ (:964) has no
    # such argument -> TypeError at the first new track.  Fixed: the [score, class] vector is
    # the track's `metadata`.
    'track_init_confidence_kwarg',
    # get_trail stacks 0-d scores into an (n_frames,) trail (:1039-1045) that step indexes
    # [:, :, :dim_metadata] (:661-662) -> IndexError once a track exists.  Fixed: (n_frames, 1).
    'metadata_trail_rank',
    # SineEncodingTracklet returns (B, n*4*F) (detr_tracking.py:305), step flattens it again
    # with .flatten(1, 2) (:660-662) -> IndexError, and add_tracks encodes a 2-d trail
    # (:869-870) -> IndexError.  Fixed: a 2-d trail gets a batch axis, the encoding is
    # (B, n, 4*F) -- the same values in the same order after the callers' flattens.
    'sine_encoding_rank',
    # Tracker.move_tracks_to_inactive (:88-94) calls track.repeat_last_pos(), which
    # TrackKinematic lacks (its method is repeat_last_state, :1018-1024) -> AttributeError
    # when a track first goes inactive.  Fixed: repeat_last_state.
    'inactive_repeat_method',
)


class IdentityEncoding:
    """detr_tracking.py:310-316."""

    def __call__(self, x):
        return x


class SineEncodingTracklet:
    """detr_tracking.py:286-307: sine / cosine features of tracklet coordinates in [0, 1]
    (x * 2 pi / temperature^(2 floor(i/2) / F), cos of the even, sin of the odd features) --
    (B, n, c) -> (B, n, c*F); `reference_rank` keeps the reference's (B, n*c*F) output and its
    failure on 2-d input."""

    def __init__(self, num_pos_feats=64, temperature=10000, scale=None, reference_rank=False):
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.scale = 2 * math.pi if scale is None else scale   # (unused by the reference's __call__)
        self.reference_rank = reference_rank

    def __call__(self, x):
        if x.dim() == 2:
            if self.reference_rank:
                raise IndexError('too many indices for tensor of dimension 2')   # x[:, :, :, None] (:300)
            x = x[None]
        dim_t = torch.arange(self.num_pos_feats, dtype=torch.float32, device=x.device)
        dim_t = self.temperature ** (2 * (dim_t // 2) / self.num_pos_feats)
        freq = (x[:, :, :, None] * torch.pi * 2) / dim_t
        emb = torch.cat([freq[:, :, :, 0::2].cos(), freq[:, :, :, 1::2].sin()], dim=3)
        return emb.flatten(1) if self.reference_rank else emb.flatten(2)


def generate_pseudo_tracklets(detections, n_frames):
    """detr_tracking.py:319-326: each detection repeated as an n_frames trail."""
    return torch.tile(detections[:, None, :4], [1, n_frames, 1])


class TrackKinematic:
    """tracker.py:961-1053: position / relative-position / score histories of one track."""

    def __init__(self, pos, pos_rel, metadata, metadata_encoded, pos_encoded, track_id, obj_ind, mask=None):
        self.id = track_id
        self.pos = pos
        self.last_pos = deque([pos.clone()])
        self.last_score = deque([metadata[0].clone()])
        self.last_pos_relative = deque([-1] if pos_rel is None else [pos_rel.clone()])
        self.metadata_encoded = metadata_encoded
        self.position_encoded = pos_encoded
        self.mask = mask
        self.obj_ind = obj_ind
        self.count_inactive = 0
        self.count_termination = 0
        self.gt_id = None
        self.metadata = metadata

    def has_positive_area(self):
        return bool(self.pos[2] > self.pos[0] and self.pos[3] > self.pos[1])

    def update_state(self, pos, relative_pos, metadata, encoding_pos, encoding_metadata):
        self.last_pos.append(pos.clone())
        self.last_score.append(metadata[0].clone())
        self.pos = pos
        self.last_pos_relative.append(relative_pos.clone())
        self.metadata_encoded = encoding_metadata
        self.position_encoded = encoding_pos
        self.metadata = metadata

    @property
    def score(self):
        return self.metadata[0]

    def repeat_last_state(self):
        self.last_pos.append(self.last_pos[-1])
        self.last_pos_relative.append(self.last_pos_relative[-1])
        self.last_score.append(self.last_score[-1])

    def get_trail(self, n_frames, reference_rank=False):
        """(n_frames, 4) relative boxes, oldest first, padded with the first one, and the score
        trail: (n_frames, 1) (reference_rank: the reference's (n_frames,))."""
        present = min(n_frames, len(self.last_pos))
        idx = [0] * (n_frames - present) + [len(self.last_pos_relative) - present + i for i in range(present)]
        pos = torch.stack([self.last_pos_relative[i].clone() for i in idx], 0)
        meta = torch.stack([self.last_score[i].clone() for i in idx], 0)
        return pos, (meta if reference_rank else meta[:, None])

    def reset_last_pos(self):
        self.last_pos.clear()
        self.last_pos_relative.clear()
        self.last_pos.append(self.pos.clone())
        self.last_score.clear()


class TrackerKinematic(Tracker):
    """tracker.py:580-959: the online tracker over the KineT kinematic model (its detector input
    is the frame's detections + metadata, its track queries the tracks' box / score trails).
    Same constructor, reset / step / get_results as the reference (track.py:104-107 builds it
    from the detector's args); GPU post-process, thresholds and NMS kernel, one batched
    device -> host copy of the per-frame decisions, host bookkeeping."""

    def __init__(self, obj_detector, obj_detector_post, tracker_cfg, obj_detector_args, generate_attention_maps=False,
                 logger=None, verbose=False):
        super().__init__(obj_detector, obj_detector_post, tracker_cfg, generate_attention_maps, logger, verbose)
        self.n_classes = tracker_cfg['n_classes']
        self.dim_metadata = 1 + self.n_classes if obj_detector_args.use_class else 1
        self.defects = frozenset(tracker_cfg.get('reference_defects', ()))
        unknown = self.defects - set(REFERENCE_DEFECTS)
        if unknown:
            raise ValueError(f'unknown reference_defects {sorted(unknown)} (known: {REFERENCE_DEFECTS})')
        if self.dim_metadata != 1 and 'metadata_trail_rank' not in self.defects:
            # the track keeps only its score history (last_score, :980), so a [score, class]
            # trail of use_class models has no source; the reference fails earlier anyway
            raise NotImplementedError('TrackerKinematic: use_class metadata trails (dim_metadata > 1)')
        self.use_empty_start = obj_detector_args.use_empty_start   # (collate choice of the loader)
        self.n_frames = obj_detector_args.track_prev_frame_range
        self.use_sine_encoding = obj_detector_args.use_encoding_tracklets
        if self.use_sine_encoding:
            rr = 'sine_encoding_rank' in self.defects
            self.encoder_tracklets_det = SineEncodingTracklet(obj_detector_args.encoding_dim_tracklets, reference_rank=rr)
            self.encoder_tracklets_metada = SineEncodingTracklet(obj_detector_args.encoding_dim_tracklets,
                                                                 reference_rank=rr)
        else:
            self.encoder_tracklets_det = IdentityEncoding()
            self.encoder_tracklets_metada = IdentityEncoding()

    def move_tracks_to_inactive(self, inactive_tracks):
        if inactive_tracks and 'inactive_repeat_method' in self.defects:
            raise AttributeError("'TrackKinematic' object has no attribute 'repeat_last_pos'")
        self.tracks = [t for t in self.tracks if t not in inactive_tracks]
        for track in inactive_tracks:
            track.repeat_last_state()
        self.inactive_tracks += inactive_tracks

    def _trail(self, track):
        return track.get_trail(self.n_frames, 'metadata_trail_rank' in self.defects)

    def _update(self, track, box, rel, meta):
        """manage_active_tracks / manage_inactive_tracks body (tracker.py:926-930, :937-941): the
        encodings of the trail BEFORE this update, passed in the reference's argument order
        (metadata encoding into `encoding_pos`, position encoding into `encoding_metadata`; they
        feed nothing the tracker outputs)."""
        pos_trail, meta_trail = self._trail(track)
        track.update_state(box, rel, meta,
                           self.encoder_tracklets_metada(meta_trail.view(1, self.n_frames, self.dim_metadata)).flatten(0),
                           self.encoder_tracklets_det(pos_trail[None]).flatten(0))

    def add_tracks(self, pos, pos_relatives, metadata_trail, pos_trail, indices, num_tracks):
        """tracker.py:858-890."""
        if len(pos) and 'track_init_confidence_kwarg' in self.defects:
            raise TypeError("TrackKinematic.__init__() got an unexpected keyword argument 'confidence'")
        new_track_ids = []
        for i in range(len(pos)):
            self.tracks.append(TrackKinematic(
                pos[i], pos_rel=pos_relatives[i], metadata=metadata_trail[i, -1],
                pos_encoded=self.encoder_tracklets_det(pos_trail[i]).flatten(0),
                metadata_encoded=self.encoder_tracklets_metada(metadata_trail[i, :, :self.dim_metadata]).flatten(0),
                track_id=self.track_num + i, obj_ind=indices[i]))
            new_track_ids.append(self.track_num + i)
        self.track_num += len(new_track_ids)
        if new_track_ids:
            self._logger(f'INIT TRACK IDS (detection_obj_score_thresh={self.detection_obj_score_thresh}): '
                         f'{new_track_ids}')
        return new_track_ids

    @torch.no_grad()
    def step(self, blob):
        """tracker.py:626-856."""
        self._prune_inactive()
        self._logger(f'FRAME: {self.frame_index + 1}')
        dev = self.device
        sample = blob[0].to(dev)
        labels = dict(blob[1][0])
        orig_size = labels['orig_size'].to(dev)[None]
        prev = self.tracks + self.inactive_tracks
        nt = len(prev)
        if nt:
            trails = [self._trail(t) for t in prev]
            det = self.encoder_tracklets_det(torch.stack([p for p, _ in trails], 0))
            meta = self.encoder_tracklets_metada(torch.stack([m for _, m in trails], 0)[:, :, :self.dim_metadata])
            labels['track_query_hs_embeds_det'] = det.flatten(1, 2)
            labels['track_query_hs_embeds_meta'] = meta.flatten(1, 2)
            labels = {k: v.to(dev) for k, v in labels.items()}
        else:
            labels['track_query_hs_embeds_det'] = torch.empty([0])
            labels['track_query_hs_embeds_meta'] = torch.empty([0])
        targets = [{k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in labels.items()}]
        outputs, _, features, _, _ = self.obj_detector(sample, targets)
        result = self.obj_detector_post['bbox'](outputs, orig_size)[0]
        pred_boxes = outputs['pred_boxes'][0, :, :4]
        if self.obj_detector.overflow_boxes:
            boxes, relative_boxes = result['boxes'], pred_boxes
        else:
            boxes, relative_boxes = clip_boxes_to_image(result['boxes'], orig_size[0]), pred_boxes.clamp(0.0, 1.0)
        scores, cls = result['scores'], result['labels']
        # every threshold decision of this frame in ONE device -> host copy
        dec = torch.stack([scores > self.track_obj_score_thresh, scores > self.reid_score_thresh,
                           scores > self.detection_obj_score_thresh, cls == 0, cls < self.n_classes]).cpu()

        if nt:
            track_keep = (dec[0, :nt] & dec[3, :nt]).tolist()
            reid_keep = (dec[1, :nt] & dec[3, :nt]).tolist()
            track_boxes, track_rel = boxes[:nt], pred_boxes[:nt]
            track_meta = torch.stack([scores[:nt], cls[:nt].to(scores.dtype)], dim=1)
            to_inactive, from_inactive = [], []
            for i, track in enumerate(self.tracks):                        # manage_active_tracks (:933-955)
                if track_keep[i]:
                    self._update(track, track_boxes[i], track_rel[i], track_meta[i])
                    track.count_termination = 0
                else:
                    track.count_termination += 1
                    if track.count_termination >= self.steps_termination:
                        to_inactive.append(track)
            for i, track in enumerate(self.inactive_tracks, start=len(self.tracks)):   # (:922-931)
                if reid_keep[i]:
                    self._update(track, track_boxes[i], track_rel[i], track_meta[i])
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

        # new detections (generate_new_tracks, :892-920)
        keep = (dec[2, nt:] & dec[4, nt:]).nonzero().flatten().to(dev)
        new_boxes, new_rel = boxes[nt:][keep], relative_boxes[nt:][keep]
        new_scores, new_cls = scores[nt:][keep], cls[nt:][keep]
        new_indices = keep[:, None]                                   # .float().nonzero() (:907)
        pub = self.public_detections_mask(new_boxes, blob[0].detections)
        new_boxes, new_rel, new_scores, new_indices = new_boxes[pub], new_rel[pub], new_scores[pub], new_indices[pub]
        new_tracklets = generate_pseudo_tracklets(new_rel, self.n_frames)
        new_cls = new_cls[pub] / self.n_classes
        new_meta = torch.tile(torch.stack([new_scores, new_cls.to(new_scores.dtype)], 1)[:, None, :],
                              dims=(1, self.n_frames, 1))
        new_track_ids = self.add_tracks(new_boxes, new_rel, new_meta, new_tracklets, new_indices, nt)

        if self.detection_nms_thresh and self.tracks:                # (:790-808)
            t_boxes = torch.stack([t.pos for t in self.tracks])
            t_scores = torch.stack([t.score for t in self.tracks]).clone()
            new_ids = set(new_track_ids)
            old = torch.tensor([t.id not in new_ids for t in self.tracks], device=dev)
            t_scores[old] = float('inf')
            keep_n = set(K.nms(t_boxes, t_scores, self.detection_nms_thresh).tolist())
            remove = [t for i, t in enumerate(self.tracks) if i not in keep_n]
            if remove:
                self._logger(f'REMOVE TRACK IDS (detection_nms_thresh={self.detection_nms_thresh}): '
                             f'{[t.id for t in remove]}')
            self.tracks = [t for t in self.tracks if t not in remove]

        if self.tracks:                                               # results (:828-841), one copy
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

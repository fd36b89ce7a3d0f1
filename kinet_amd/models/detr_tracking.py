"""Track-query wrapper of the detector (src/trackformer/models/detr_tracking.py:16-283,
DeformableDETRTracking :892-895).

Tracking mode (`model.tracking()`, used by the online tracker, tracker.py:309): the
caller passes `targets=[{'track_query_hs_embeds': (K, d), 'track_query_boxes': (K, 4)}]`
and the previous frame's `features`; the K track queries are prepended to the object
queries inside the transformer (deformable_transformer.py:204-227) -- handled by
kinet_amd.models.deformable_transformer.  Training mode runs the two-pass scheme
(previous frame without grad, Hungarian matching on the host, track-query sampling,
current frame with grad) in kinet_amd.models.training.
"""
import torch
from torch import nn

from kinet_amd.models.deformable_detr import DeformableDETR


class DETRTrackingBase(nn.Module):
    def __init__(self, track_query_false_positive_prob: float = 0.0, track_query_false_negative_prob: float = 0.0,
                 matcher=None, backprop_prev_frame=False):
        self._matcher = matcher
        self._track_query_false_positive_prob = track_query_false_positive_prob
        self._track_query_false_negative_prob = track_query_false_negative_prob
        self._backprop_prev_frame = backprop_prev_frame
        self._tracking = False

    def train(self, mode: bool = True):
        self._tracking = False
        return super().train(mode)

    def tracking(self):
        self.eval()
        self._tracking = True

    def forward(self, samples, targets: list = None, prev_features=None):
        """detr_tracking.py:220-283: with targets and not tracking, training runs the
        two-pass track-query scheme (kinet_amd.models.training), evaluation adds empty
        track-query fields."""
        if targets is not None and not self._tracking:
            from kinet_amd.models import training
            prev_features = training.prepare_track_queries(self, targets, super().forward, prev_features)
        return super().forward(samples, targets, prev_features)


class DeformableDETRTracking(DETRTrackingBase, DeformableDETR):
    def __init__(self, tracking_kwargs, detr_kwargs):
        DeformableDETR.__init__(self, **detr_kwargs)
        DETRTrackingBase.__init__(self, **tracking_kwargs)

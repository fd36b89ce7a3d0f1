"""Configuration values of the detection path (the reference's Sacred YAMLs, as data).

DEFAULTS are the keys of cfgs/train.yaml that build_model and the detector read; NAMED
are the named configs layered on top (cfgs/train_deformable.yaml, train_multi_frame.yaml,
train_tracking.yaml, train_mot17.yaml, train_full_res.yaml, train_kinet.yaml).  `load_args(*names, **kw)`
returns the argparse.Namespace build_model expects (util/misc.py:668-674 equivalent).
"""
from argparse import Namespace

DEFAULTS = dict(
    lr=0.0002, lr_backbone_names=['backbone.0'], lr_backbone=0.00002,
    lr_linear_proj_names=['reference_points', 'sampling_offsets'], lr_linear_proj_mult=0.1, lr_track=0.0001, batch_size=2,
    weight_decay=0.0001, epochs=50, lr_drop=40, clip_max_norm=0.1,
    deformable=False, kine=False, used_ordered_queries=False, use_empty_start=False, use_encoder_only=False,
    use_encoding_tracklets=False, use_encoding_dets=False, encoding_dim_detections=32, encoding_dim_tracklets=32,
    max_number_detection=60, use_class=False, ratio_add_tracklets=1.0,
    with_box_refine=False, two_stage=False, freeze_detr=False,
    backbone='resnet50', dilation=False, position_embedding='sine', num_feature_levels=1,
    enc_layers=6, dec_layers=6, dim_feedforward=2048, hidden_dim=256, activation='relu', dropout=0.1,
    nheads=8, num_queries=100, pre_norm=False, dec_n_points=4, enc_n_points=4,
    tracking=False, tracking_eval=True, track_prev_frame_range=0, track_prev_frame_rnd_augs=0.01,
    track_prev_prev_frame=False, track_backprop_prev_frame=False, track_query_false_positive_prob=0.1,
    track_query_false_negative_prob=0.4, track_query_false_positive_eos_weight=True, track_attention=False,
    multi_frame_attention=False, multi_frame_encoding=True, multi_frame_attention_separate_encoder=True,
    merge_frame_features=False, overflow_boxes=False, masks=False,
    set_cost_class=1.0, set_cost_bbox=5.0, set_cost_giou=2.0, aux_loss=True, mask_loss_coef=1.0,
    dice_loss_coef=1.0, cls_loss_coef=1.0, bbox_loss_coef=5.0, giou_loss_coef=2, eos_coef=0.1,
    focal_loss=False, focal_alpha=0.25, focal_gamma=2, dataset='coco', img_transform={'max_size': 666, 'val_width': 400},
    device='cuda', seed=42, resume='', world_size=0, dist_url='env://',
)

NAMED = {
    'train_deformable': dict(deformable=True, num_feature_levels=4, num_queries=300, dim_feedforward=1024,
                             focal_loss=True, focal_alpha=0.25, focal_gamma=2, cls_loss_coef=2.0,
                             set_cost_class=2.0, overflow_boxes=True, with_box_refine=True, activation='relu'),
    'train_multi_frame': dict(num_queries=500, hidden_dim=288, multi_frame_attention=True,
                              multi_frame_encoding=True, multi_frame_attention_separate_encoder=True),
    'train_tracking': dict(tracking=True, tracking_eval=True, track_prev_frame_range=5,
                           track_query_false_positive_eos_weight=True),
    'train_mot17': dict(dataset='mot', epochs=50, lr_drop=10),
    'train_full_res': dict(img_transform={'max_size': 1920, 'val_width': 1080}),
    # the KineT model; `tracking` comes from train_tracking as in the reference runs
    'train_kinet': dict(dataset='mot_kine', kine=True, position_embedding='sine', multi_frame_encoding=True,
                        track_prev_frame_range=5, use_encoding_tracklets=False, use_encoding_dets=False,
                        encoding_dim_detections=32, encoding_dim_tracklets=8, track_query_false_negative_prob=0.2,
                        num_queries=150, hidden_dim=288, activation='relu', batch_size=8, epochs=500, lr_drop=50,
                        lr_linear_proj_mult=0.5, lr=0.0001, dec_layers=1, enc_layers=1),
}

# cfgs/track.yaml:28-49, the tracker thresholds as shipped
TRACKER_CFG = dict(public_detections=False, detection_obj_score_thresh=0.4, track_obj_score_thresh=0.4,
                   detection_nms_thresh=0.9, track_nms_thresh=0.9, steps_termination=1, prev_frame_dist=1,
                   inactive_patience=-1, reid_sim_threshold=0.0, reid_sim_only=False, reid_score_thresh=0.4,
                   reid_greedy_matching=False)


def load_args(*names, **overrides):
    d = dict(DEFAULTS)
    for n in names:
        n = n[:-5] if n.endswith('.yaml') else n
        d.update(NAMED[n])
    d.update(overrides)
    return Namespace(**d)

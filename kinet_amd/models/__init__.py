"""`build_model(args) -> (model, criterion, postprocessors)` for the detection hot path,
mirroring src/trackformer/models/__init__.py:16-71 (deformable branch).

    from kinet_amd.models import build_model      # instead of trackformer.models
    model, criterion, postprocessors = build_model(args)
    model.set_compute_dtype(torch.bfloat16)        # optional perf mode (default fp32)

`args` is the reference's Namespace (cfgs/train.yaml + named configs).  The deformable image
branch (the hot path) and the KineT kinematic branch (`args.kine`, :72-107,
kinet_amd/models/kinet.py) are built; vanilla DETR / masks raise.
"""
import torch

from kinet_amd.models.backbone import build_backbone
from kinet_amd.models.deformable_detr import DeformableDETR, DeformablePostProcess, PostProcess
from kinet_amd.models.deformable_transformer import build_deforamble_transformer
from kinet_amd.models.detr_tracking import DeformableDETRTracking
from kinet_amd.models.misc import NestedTensor, NestedTensorKinet, nested_tensor_from_tensor_list

NUM_CLASSES = {'coco': 91, 'coco_panoptic': 250, 'coco_person': 20, 'mot': 20, 'mot_crowdhuman': 20,
               'crowdhuman': 20, 'mot_coco_person': 20, 'mot_kine': 1}


def build_model(args):
    if args.dataset not in NUM_CLASSES:
        raise NotImplementedError(args.dataset)
    num_classes = NUM_CLASSES[args.dataset]
    if getattr(args, 'kine', False) and not args.deformable:
        from kinet_amd.models.criterion import build_criterion
        from kinet_amd.models.kinet import build_kinet
        from kinet_amd.models.matcher import build_matcher
        matcher = build_matcher(args)
        model = build_kinet(args, num_classes)
        post = {'bbox': DeformablePostProcess() if args.focal_loss else PostProcess()}
        return model, build_criterion(args, num_classes, matcher), post
    if not args.deformable:
        raise NotImplementedError('vanilla DETR (config 1) is outside the MSDeformAttn hot path')
    if getattr(args, 'masks', False):
        raise NotImplementedError('segmentation heads are outside the hot path')
    backbone = build_backbone(args)
    matcher = None
    try:
        from kinet_amd.models.matcher import build_matcher
        matcher = build_matcher(args)
    except ImportError:
        pass
    detr_kwargs = {
        'backbone': backbone,
        'num_classes': num_classes - 1 if args.focal_loss else num_classes,
        'num_queries': args.num_queries,
        'aux_loss': args.aux_loss,
        'overflow_boxes': args.overflow_boxes,
        'transformer': build_deforamble_transformer(args),
        'num_feature_levels': args.num_feature_levels,
        'with_box_refine': args.with_box_refine,
        'two_stage': args.two_stage,
        'multi_frame_attention': args.multi_frame_attention,
        'multi_frame_encoding': args.multi_frame_encoding,
        'merge_frame_features': args.merge_frame_features,
    }
    if args.tracking:
        tracking_kwargs = {
            'track_query_false_positive_prob': args.track_query_false_positive_prob,
            'track_query_false_negative_prob': args.track_query_false_negative_prob,
            'matcher': matcher,
            'backprop_prev_frame': args.track_backprop_prev_frame}
        model = DeformableDETRTracking(tracking_kwargs, detr_kwargs)
    else:
        model = DeformableDETR(**detr_kwargs)
    criterion = None
    try:
        from kinet_amd.models.criterion import build_criterion
        criterion = build_criterion(args, num_classes, matcher)
    except ImportError:
        pass
    postprocessors = {'bbox': DeformablePostProcess()}
    return model, criterion, postprocessors


__all__ = ['build_model', 'DeformableDETR', 'DeformableDETRTracking', 'DeformablePostProcess', 'PostProcess',
           'NestedTensor', 'NestedTensorKinet', 'nested_tensor_from_tensor_list']

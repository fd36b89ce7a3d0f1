"""Host-side containers and helpers of the detection path, mirroring
src/trackformer/util/misc.py (NestedTensor :407-443, nested_tensor_from_tensor_list
:387-405, inverse_sigmoid :609-613) and util/box_ops.py (:9-21)."""
from typing import List, Optional

import torch
from torch import Tensor


class NestedTensor(object):
    """util/misc.py:407-443.  `sizes` (tuple of per-image (H, W)) is attached when the
    padding mask is fully determined by the image sizes; it keys the per-geometry caches
    (masks, valid ratios, reference points, position embeddings)."""

    def __init__(self, tensors, mask: Optional[Tensor] = None, sizes=None):
        self.tensors = tensors
        self.mask = mask
        self.sizes = sizes

    def to(self, device):
        cast_tensor = self.tensors.to(device)
        cast_mask = self.mask.to(device) if self.mask is not None else None
        return NestedTensor(cast_tensor, cast_mask, self.sizes)

    def decompose(self):
        return self.tensors, self.mask

    def __repr__(self):
        return str(self.tensors)

    def unmasked_tensor(self, index: int):
        tensor = self.tensors[index]
        if not self.mask[index].any():
            return tensor
        h_index = self.mask[index, 0, :].nonzero(as_tuple=True)[0]
        if len(h_index):
            tensor = tensor[:, :, :h_index[0]]
        w_index = self.mask[index, :, 0].nonzero(as_tuple=True)[0]
        if len(w_index):
            tensor = tensor[:, :w_index[0], :]
        return tensor


class NestedTensorKinet(object):
    """util/misc.py:445-459: the KineT model's input -- detections and their metadata, each a
    NestedTensor of (B, n, c) with a (B, n) padding mask."""

    def __init__(self, detections, metadata, img=None):
        self.detections = detections
        self.metadata = metadata

    def to(self, device):
        return NestedTensorKinet(self.detections.to(device), self.metadata.to(device))

    def __repr__(self):
        return str(self.detections) + '\n ' + str(self.metadata)


def nested_tensor_from_tensor_list(tensor_list: List[Tensor]):
    """util/misc.py:387-405: zero-pad to the max (H, W), mask True on padding."""
    if tensor_list[0].ndim != 3:
        raise ValueError('not supported')
    max_size = [max(s) for s in zip(*[list(img.shape) for img in tensor_list])]
    b = len(tensor_list)
    _, h, w = max_size
    sizes = tuple((int(img.shape[1]), int(img.shape[2])) for img in tensor_list)
    dtype, device = tensor_list[0].dtype, tensor_list[0].device
    if all(s == (h, w) for s in sizes):
        tensor = torch.stack(tensor_list, 0) if b > 1 else tensor_list[0][None]
        mask = torch.zeros((b, h, w), dtype=torch.bool, device=device)
        return NestedTensor(tensor, mask, sizes)
    tensor = torch.zeros([b] + max_size, dtype=dtype, device=device)
    mask = torch.ones((b, h, w), dtype=torch.bool, device=device)
    for img, pad_img, m in zip(tensor_list, tensor, mask):
        pad_img[: img.shape[0], : img.shape[1], : img.shape[2]].copy_(img)
        m[: img.shape[1], :img.shape[2]] = False
    return NestedTensor(tensor, mask, sizes)


def host_to_device(values, dtype, device):
    """A small host list / array as a device tensor without a host-side wait: a plain
    torch.as_tensor(..., device=cuda) copies from pageable memory and synchronises the stream,
    which drains the queue the host is running ahead of."""
    t = torch.as_tensor(values, dtype=dtype)
    if torch.device(device).type != 'cuda':
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


def inverse_sigmoid(x, eps=1e-5):
    if x.is_cuda and x.dtype == torch.float32:
        # one HIP kernel each way (csrc/train_ops.hip) instead of 6 / 8 torch launches
        from kinet_amd import autograd as A
        return A.inverse_sigmoid(x, eps)
    x = x.clamp(min=0, max=1)
    x1 = x.clamp(min=eps)
    x2 = (1 - x).clamp(min=eps)
    return torch.log(x1 / x2)


def box_cxcywh_to_xyxy(x):
    x_c, y_c, w, h = x.unbind(-1)
    return torch.stack([(x_c - 0.5 * w), (y_c - 0.5 * h), (x_c + 0.5 * w), (y_c + 0.5 * h)], dim=-1)


def box_xyxy_to_cxcywh(x):
    x0, y0, x1, y1 = x.unbind(-1)
    return torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, (x1 - x0), (y1 - y0)], dim=-1)


def box_area(boxes):
    return (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])


def box_iou(boxes1, boxes2):
    area1, area2 = box_area(boxes1), box_area(boxes2)
    lt = torch.max(boxes1[:, None, :2], boxes2[:, :2])
    rb = torch.min(boxes1[:, None, 2:], boxes2[:, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[:, :, 0] * wh[:, :, 1]
    union = area1[:, None] + area2 - inter
    return inter / union, union


def generalized_box_iou(boxes1, boxes2, checks=None):
    """util/box_ops.py:38-60 (degenerate boxes rejected the same way).  checks: None asserts
    right here, as the reference does (a device -> host sync per assert on GPU tensors); a
    list receives the two device bool flags instead, for the caller to assert at a sync point
    it already has (the matcher's cost-matrix copy, the training step's loss check)."""
    ok1 = (boxes1[:, 2:] >= boxes1[:, :2]).all()
    ok2 = (boxes2[:, 2:] >= boxes2[:, :2]).all()
    if checks is None:
        assert ok1
        assert ok2
    else:
        checks += [ok1, ok2]
    iou, union = box_iou(boxes1, boxes2)
    lt = torch.min(boxes1[:, None, :2], boxes2[:, :2])
    rb = torch.max(boxes1[:, None, 2:], boxes2[:, 2:])
    wh = (rb - lt).clamp(min=0)
    area = wh[:, :, 0] * wh[:, :, 1]
    return iou - (area - union) / area

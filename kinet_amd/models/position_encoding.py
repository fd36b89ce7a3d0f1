"""Sine position encodings of the detection path (src/trackformer/models/position_encoding.py),
computed by the kinet_sine_position_embed kernel (csrc/ops.hip).

They depend only on the padding mask (never on pixel values): the detector's inference path
computes them once per frame geometry, level embedding added, straight into the cached
flattened (B, S, d) buffer (kinet_amd/models/deformable_detr.py); the modules' forward
returns the reference's NCHW layout (a view of the kernel's NHWC rows).
  PositionEmbeddingSine    position_encoding.py:85-121: e = (cumsum - 0.5) / (last + 1e-6) * 2pi
  PositionEmbeddingSine3D  position_encoding.py:12-81:  z / y / x thirds, e = cumsum / (last + 1e-6) * 2pi,
                           z over the `num_frames` axis
dim_t = temperature ** (2 * (k // 2) / num_pos_feats) is evaluated with torch on the host
(f32, the reference's own expression) and cached on the device.
"""
import math

import torch
from torch import nn

from kinet_amd import kernels as K


class _SineBase(nn.Module):
    three_d = False

    def __init__(self, num_pos_feats=64, temperature=10000, normalize=False, scale=None):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        if scale is not None and normalize is False:
            raise ValueError("normalize should be True if scale is passed")
        self.scale = 2 * math.pi if scale is None else scale
        self._dim_t = {}

    def dim_t(self, device):
        key = str(device)
        d = self._dim_t.get(key)
        if d is None:
            k = torch.arange(self.num_pos_feats, dtype=torch.float32)
            d = (self.temperature ** (2 * (k // 2) / self.num_pos_feats)).to(device)
            self._dim_t[key] = d
        return d

    @property
    def channels(self):
        return (3 if self.three_d else 2) * self.num_pos_feats

    def rows(self, mask, frame=0, level_embed=None, out=None, out_batch_stride=None, out_dtype=torch.float32):
        """(B, H*W, C) NHWC rows of the embedding (+ level_embed) for `frame`."""
        return K.sine_position_embed(mask, self.dim_t(mask.device), self.num_pos_feats, self.three_d, frame,
                                     getattr(self, 'frames', 1), self.normalize, self.scale, level_embed, out,
                                     out_batch_stride, out_dtype)


class PositionEmbeddingSine(_SineBase):
    def embed_mask(self, mask):
        """mask (B, H, W) bool -> (B, 2*num_pos_feats, H, W) f32 (NCHW view)."""
        B, H, W = mask.shape
        return self.rows(mask).view(B, H, W, self.channels).permute(0, 3, 1, 2)

    def forward(self, tensor_list):
        return self.embed_mask(tensor_list.mask)


class PositionEmbeddingSine3D(_SineBase):
    three_d = True

    def __init__(self, num_pos_feats=64, num_frames=2, temperature=10000, normalize=False, scale=None):
        super().__init__(num_pos_feats, temperature, normalize, scale)
        self.frames = num_frames

    def embed_mask(self, mask):
        """mask (B, H, W) -> (B, frames, 3*num_pos_feats, H, W) f32."""
        B, H, W = mask.shape
        return torch.stack([self.rows(mask, f).view(B, H, W, self.channels).permute(0, 3, 1, 2)
                            for f in range(self.frames)], 1)

    def forward(self, tensor_list):
        return self.embed_mask(tensor_list.mask)


def build_position_encoding(args):
    """position_encoding.py:187-214 (image branches)."""
    if getattr(args, 'kine', False):
        raise NotImplementedError('KineT detection-box encodings are outside the image hot path')
    if args.multi_frame_attention and args.multi_frame_encoding:
        n_steps, fn = args.hidden_dim // 3, PositionEmbeddingSine3D
    else:
        n_steps, fn = args.hidden_dim // 2, PositionEmbeddingSine
    if args.position_embedding in ('v2', 'sine'):
        return fn(n_steps, normalize=True)
    raise ValueError(f"not supported {args.position_embedding}")

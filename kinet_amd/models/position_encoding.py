"""Sine position encodings of the detection path (src/trackformer/models/position_encoding.py).

They depend only on the padding mask (never on pixel values), so the detector computes
them once per frame geometry and caches them (kinet_amd/models/deformable_detr.py);
this module holds the arithmetic, identical to the reference:
  PositionEmbeddingSine    position_encoding.py:85-121 (normalize=True: (cumsum-0.5)/(last+eps)*2pi)
  PositionEmbeddingSine3D  position_encoding.py:12-81  (2-frame z axis; z/y/x thirds)
"""
import math

import torch
from torch import nn


class PositionEmbeddingSine(nn.Module):
    def __init__(self, num_pos_feats=64, temperature=10000, normalize=False, scale=None):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        if scale is not None and normalize is False:
            raise ValueError("normalize should be True if scale is passed")
        self.scale = 2 * math.pi if scale is None else scale

    def embed_mask(self, mask):
        """mask (B, H, W) bool -> (B, 2*num_pos_feats, H, W) f32."""
        not_mask = ~mask
        y_embed = not_mask.cumsum(1, dtype=torch.float32)
        x_embed = not_mask.cumsum(2, dtype=torch.float32)
        if self.normalize:
            eps = 1e-6
            y_embed = (y_embed - 0.5) / (y_embed[:, -1:, :] + eps) * self.scale
            x_embed = (x_embed - 0.5) / (x_embed[:, :, -1:] + eps) * self.scale
        dim_t = torch.arange(self.num_pos_feats, dtype=torch.float32, device=mask.device)
        dim_t = self.temperature ** (2 * (dim_t // 2) / self.num_pos_feats)
        pos_x = x_embed[:, :, :, None] / dim_t
        pos_y = y_embed[:, :, :, None] / dim_t
        pos_x = torch.stack((pos_x[:, :, :, 0::2].sin(), pos_x[:, :, :, 1::2].cos()), dim=4).flatten(3)
        pos_y = torch.stack((pos_y[:, :, :, 0::2].sin(), pos_y[:, :, :, 1::2].cos()), dim=4).flatten(3)
        return torch.cat((pos_y, pos_x), dim=3).permute(0, 3, 1, 2)

    def forward(self, tensor_list):
        return self.embed_mask(tensor_list.mask)


class PositionEmbeddingSine3D(nn.Module):
    def __init__(self, num_pos_feats=64, num_frames=2, temperature=10000, normalize=False, scale=None):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        self.frames = num_frames
        if scale is not None and normalize is False:
            raise ValueError("normalize should be True if scale is passed")
        self.scale = 2 * math.pi if scale is None else scale

    def embed_mask(self, mask):
        """mask (B, H, W) -> (B, frames, 3*num_pos_feats, H, W) f32."""
        n, h, w = mask.shape
        mask = mask.view(n, 1, h, w).expand(n, self.frames, h, w)
        not_mask = ~mask
        z_embed = not_mask.cumsum(1, dtype=torch.float32)
        y_embed = not_mask.cumsum(2, dtype=torch.float32)
        x_embed = not_mask.cumsum(3, dtype=torch.float32)
        if self.normalize:
            eps = 1e-6
            z_embed = z_embed / (z_embed[:, -1:, :, :] + eps) * self.scale
            y_embed = y_embed / (y_embed[:, :, -1:, :] + eps) * self.scale
            x_embed = x_embed / (x_embed[:, :, :, -1:] + eps) * self.scale
        dim_t = torch.arange(self.num_pos_feats, dtype=torch.float32, device=mask.device)
        dim_t = self.temperature ** (2 * (dim_t // 2) / self.num_pos_feats)
        pos_x = x_embed[:, :, :, :, None] / dim_t
        pos_y = y_embed[:, :, :, :, None] / dim_t
        pos_z = z_embed[:, :, :, :, None] / dim_t
        pos_x = torch.stack((pos_x[..., 0::2].sin(), pos_x[..., 1::2].cos()), dim=5).flatten(4)
        pos_y = torch.stack((pos_y[..., 0::2].sin(), pos_y[..., 1::2].cos()), dim=5).flatten(4)
        pos_z = torch.stack((pos_z[..., 0::2].sin(), pos_z[..., 1::2].cos()), dim=5).flatten(4)
        return torch.cat((pos_z, pos_y, pos_x), dim=4).permute(0, 1, 4, 2, 3)

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

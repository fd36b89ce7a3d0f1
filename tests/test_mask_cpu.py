"""interp_mask (backbone.py:89 nearest resize of the padding mask) as an index gather must
equal F.interpolate(mask[None].float(), size).bool()[0] exactly (CPU)."""
import torch
import torch.nn.functional as F

from kinet_amd.models.backbone import interp_mask


def test_interp_mask_matches_interpolate():
    g = torch.Generator().manual_seed(0)
    for H, W in [(800, 1333), (37, 41), (7, 9), (1000, 1500)]:
        m = torch.rand(2, H, W, generator=g) < 0.5
        for h, w in [(100, 167), (50, 84), (25, 42), (13, 21), (H // 3 + 1, W // 5 + 2), (H, W), (2 * H, 3 * W)]:
            a = interp_mask(m, (h, w))
            b = F.interpolate(m[None].float(), size=(h, w)).to(torch.bool)[0]
            assert a.shape == b.shape and torch.equal(a, b), (H, W, h, w)

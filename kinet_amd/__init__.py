"""kinet_amd -- MI355X-native (gfx950) rebuild of the TrackFormer/KineTTracker per-frame
detection hot path: ResNet backbone -> input projections -> Deformable-DETR encoder /
decoder (MSDeformAttn) -> class/box heads, behind the reference's own APIs:

  * `MultiScaleDeformableAttention` extension module (ms_deform_attn_forward/backward)
  * `MSDeformAttnFunction`, `MSDeformAttn`            (kinet_amd.msda)
  * `build_model(args)` / `model(samples, targets, prev_features)`  (kinet_amd.models)

All compute runs in hand-written HIP kernels in kinet_amd/_lib/libkinet_amd.so.
"""
import sys as _sys

from kinet_amd import MultiScaleDeformableAttention as _msda_ext

# satisfy `import MultiScaleDeformableAttention as MSDA` (ms_deform_attn_func.py:11)
_sys.modules.setdefault('MultiScaleDeformableAttention', _msda_ext)

__version__ = '0.1.0'

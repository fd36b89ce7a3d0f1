"""ResNet-50/101 backbone of the detection path, NHWC, run by the kinet_amd implicit-GEMM
conv kernel with FrozenBatchNorm2d folded into the epilogue.

Mirrors src/trackformer/models/backbone.py (FrozenBatchNorm2d :22-58, BackboneBase
:61-91, Backbone :94-108, Joiner :180-194, build_backbone :197-230).  The ResNet body
follows torchvision's v1.5 definition (the reference instantiates
torchvision.models.resnet50/101, backbone.py:102): 7x7/2 stem, 3x3/2 max-pool,
Bottleneck blocks with the stride on the 3x3 conv and a 1x1 strided downsample on the
first block of each stage.  Module/parameter names equal torchvision's, so reference
state_dicts (`backbone.0.body.layer1.0.conv1.weight`, ...) load unchanged.
"""
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from kinet_amd import autograd as A
from kinet_amd import kernels as K
from kinet_amd.models.misc import NestedTensor
from kinet_amd.models.position_encoding import build_position_encoding


class FrozenBatchNorm2d(nn.Module):
    """backbone.py:22-58; folded to (scale, bias) = (w*rsqrt(rv+1e-5), b - rm*scale)."""

    def __init__(self, n):
        super().__init__()
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))
        self._fold = None

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict,
                              missing_keys, unexpected_keys, error_msgs):
        state_dict.pop(prefix + 'num_batches_tracked', None)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict,
                                      missing_keys, unexpected_keys, error_msgs)

    def folded(self):
        key = tuple((b.data_ptr(), b._version) for b in (self.weight, self.bias, self.running_mean, self.running_var))
        if self._fold is None or self._fold[0] != key:
            scale = self.weight * (self.running_var + 1e-5).rsqrt()
            bias = self.bias - self.running_mean * scale
            self._fold = (key, scale.float().contiguous(), bias.float().contiguous())
        return self._fold[1], self._fold[2]

    def forward(self, x):   # NCHW reference semantics (used by the autograd path)
        scale, bias = self.folded()
        return x * scale.reshape(1, -1, 1, 1) + bias.reshape(1, -1, 1, 1)


# Block i's conv3 and block i+1's conv1 as one launch (kinet_bottleneck_pair) for the stages
# whose bottleneck width is in FUSE_PAIR_WIDTHS; False runs every conv on its own (A/B:
# tools/bneck_ab.py, bench.py --pair-widths).  Round 4 kept stages 2-3 (128 / 256) as two launches:
# at batch 16 the pair kernel's 256-row tiles left a half-empty last round
# (profiles/r04h_bneck_ab.log).  At the round-6 bench batches (24 / 12 / 4 frames, three batches in
# flight) the pairs win at every width: config 2 1344 / 1357 -> 1386 / 1382 frames/s, config 3
# 616 / 613 -> 619 / 624, config 5 274 / 276 -> 282 / 282 (A B A B on one box,
# profiles/r06c_ab_summary.txt, r06d_ab_summary.txt)
FUSE_BOTTLENECK_PAIRS = True
FUSE_PAIR_WIDTHS = (64, 128, 256)
# 16-bit stem straight from the f32 image (kinet_stem_conv_image); False: pack_image_kwfold +
# the folded conv (A/B: bench.py --stem-image 0)
STEM_FROM_IMAGE = True


def conv_bn(x, conv, bn, relu, residual=None, cin_pad=None):
    """NHWC conv + folded BN (+ residual) (+ ReLU) in one kernel launch."""
    w = K.pack_conv_weight(conv.weight, x.dtype, cin_pad)
    scale, bias = bn.folded()
    return K.conv2d_nhwc(x, w, conv.stride[0], conv.padding[0], scale=scale, bias=bias, relu=relu,
                         residual=residual)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        if dilation != 1:
            raise NotImplementedError('dilated (DC5) ResNet is not on the configured hot path')
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = FrozenBatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = FrozenBatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = FrozenBatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward_nhwc(self, x):
        out = conv_bn(x, self.conv1, self.bn1, True)
        out = conv_bn(out, self.conv2, self.bn2, True)
        identity = x if self.downsample is None else conv_bn(x, self.downsample[0], self.downsample[1], False)
        return conv_bn(out, self.conv3, self.bn3, True, residual=identity)

    def forward_autograd(self, x):
        """Training path (NHWC, f32): the same conv + folded-BN (+ residual) + ReLU sequence on
        kinet_amd.autograd Functions (kinet kernels forward and backward)."""
        out = A.conv_nhwc(x, self.conv1.weight, None, 1, 0, *self.bn1.folded(), relu=True)
        out = A.conv_nhwc(out, self.conv2.weight, None, self.conv2.stride[0], 1, *self.bn2.folded(), relu=True)
        identity = x
        if self.downsample is not None:
            ds, bn = self.downsample[0], self.downsample[1]
            identity = A.conv_nhwc(x, ds.weight, None, ds.stride[0], 0, *bn.folded(), relu=False)
        return A.conv_nhwc(out, self.conv3.weight, None, 1, 0, *self.bn3.folded(), relu=True, residual=identity)


def _pair_ok(dtype, blk, nxt):
    return (FUSE_BOTTLENECK_PAIRS and blk.conv3.in_channels in FUSE_PAIR_WIDTHS
            and K.bottleneck_pair_supported(dtype, blk.conv3.weight, nxt.conv1.weight))


def forward_layer_nhwc(layer, x, t1=None, next_block=None):
    """One ResNet stage over NHWC x -> (stage output, next_block's conv1 output or None).
    With FUSE_BOTTLENECK_PAIRS the chain conv3 (+ residual + ReLU) of block i -> conv1 of block
    i+1 runs as one kinet_bottleneck_pair launch: the block output is written once (the next
    block's residual) and not re-read by the next conv1.  `next_block` (the next stage's first
    block) extends the chain across the stage boundary where the pair kernel covers it (stage 1
    -> 2: its conv1 is stride 1); `t1` = this stage's first conv1 output when the previous stage
    computed it.  Same math as Bottleneck.forward_nhwc per block (torchvision, backbone.py:102)."""
    blocks = list(layer)
    b0 = blocks[0]
    if t1 is None:
        t1 = conv_bn(x, b0.conv1, b0.bn1, True)
    identity = x if b0.downsample is None else conv_bn(x, b0.downsample[0], b0.downsample[1], False)
    t_next = None
    for i, blk in enumerate(blocks):
        t2 = conv_bn(t1, blk.conv2, blk.bn2, True)
        last = i + 1 == len(blocks)
        nxt = next_block if last else blocks[i + 1]
        if (nxt is not None and nxt.conv1.stride == (1, 1) and _pair_ok(t2.dtype, blk, nxt)
                and t2.numel() * 4 * t2.element_size() < 2 ** 31):   # the kernel's 32-bit offsets
            s3, b3 = blk.bn3.folded()
            s1, b1 = nxt.bn1.folded()
            packed = K.bottleneck_pack(blk.conv3.weight, nxt.conv1.weight, s3, s1, t2.dtype)
            identity, t1 = K.bottleneck_pair(t2, identity, packed, b3, b1)
            if last:
                t_next = t1
        else:
            identity = conv_bn(t2, blk.conv3, blk.bn3, True, residual=identity)
            if not last:
                t1 = conv_bn(identity, nxt.conv1, nxt.bn1, True)
    return identity, t_next


class ResNetBody(nn.Module):
    """torchvision ResNet up to layer4 (what IntermediateLayerGetter keeps, backbone.py:81)."""

    def __init__(self, layers, dilation=False):
        super().__init__()
        if dilation:
            raise NotImplementedError('dilated (DC5) ResNet is not on the configured hot path')
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = FrozenBatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], 2)
        self.layer3 = self._make_layer(256, layers[2], 2)
        self.layer4 = self._make_layer(512, layers[3], 2)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * 4:
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                                       FrozenBatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * 4
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward_nhwc(self, img_nchw, dtype):
        """img (B, 3, H, W) f32 -> [layer1, layer2, layer3, layer4] NHWC in dtype."""
        # stem (torchvision conv1 7x7/2 + FrozenBN + ReLU): the 7 horizontal taps are folded
        # into 24 channels while packing the image, so the conv runs as 7x1 with strides
        # (2, 1): K = 7*24 = 168 instead of 7*7*8 = 392 (kinet_pack_image_kwfold)
        x, t1 = self._stem_stage1(img_nchw, dtype, self.layer2[0])
        outs = [x]
        stages = (self.layer2, self.layer3, self.layer4)
        for k, layer in enumerate(stages):
            x, t1 = forward_layer_nhwc(layer, x, t1, stages[k + 1][0] if k + 1 < len(stages) else None)
            outs.append(x)
        return outs

    def forward_autograd(self, img_nchw):
        """Training path -> OrderedDict like IntermediateLayerGetter, NCHW views of NHWC f32
        tensors.  The stem and layer1 are frozen in every configuration (backbone.py:69-71
        trains only layer2-4), so they run the inference kernels without a graph; layer2-4 run
        on differentiable kinet Functions."""
        frozen = [p for m in (self.conv1, self.layer1) for p in m.parameters()]
        if any(p.requires_grad for p in frozen):
            raise NotImplementedError('training the ResNet stem / layer1 is not supported '
                                      '(the reference freezes them, backbone.py:69-71)')
        with torch.no_grad():
            x = self.forward_nhwc_stem_layer1(img_nchw, torch.float32)
        outs = [x]
        for layer in (self.layer2, self.layer3, self.layer4):
            for blk in layer:
                x = blk.forward_autograd(x)
            outs.append(x)
        return OrderedDict((str(i), nhwc_as_nchw(o)) for i, o in enumerate(outs))

    def forward_nhwc_stem_layer1(self, img_nchw, dtype):
        return self._stem_stage1(img_nchw, dtype, None)[0]

    def _stem_stage1(self, img_nchw, dtype, next_block):
        """stem + layer1 -> (layer1 output, next_block's conv1 output when the last stage-1 pair
        computed it, else None)."""
        c1 = self.conv1
        kh, kw = c1.kernel_size
        cg = (3 * kw + 7) // 8 * 8
        scale, bias = self.bn1.folded()
        if STEM_FROM_IMAGE and dtype in (torch.bfloat16, torch.float16):
            # the folded rows built in LDS from the f32 image (no packed copy of the image)
            x = K.stem_conv_image(img_nchw, K.pack_stem_weight(c1.weight, dtype, cg), scale, bias, dtype)
        else:
            x = K.pack_image_kwfold(img_nchw, dtype, kw, c1.stride[1], c1.padding[1], cg)
            x = K.conv2d_nhwc(x, K.pack_stem_weight(c1.weight, dtype, cg), (c1.stride[0], 1),
                              (c1.padding[0], 0), scale=scale, bias=bias, relu=True)
        x = K.maxpool_3x3s2(x)
        return forward_layer_nhwc(self.layer1, x, None, next_block)

    def forward(self, x):
        return self.forward_autograd(x)


def nhwc_as_nchw(x):
    """(B, H, W, C) contiguous -> (B, C, H, W) view (channels_last strides, no copy)."""
    return x.permute(0, 3, 1, 2)


def nchw_to_nhwc(x):
    """Accept a (B, C, H, W) tensor (e.g. prev_features from a previous frame) as NHWC."""
    y = x.permute(0, 2, 3, 1)
    return y if y.is_contiguous() else y.contiguous()


_NEAREST_IDX = {}


def _nearest_index(n_in, n_out, device):
    """Source indices of F.interpolate(mode='nearest') along one axis: min(floor(dst * (in /
    out)), in - 1) with the scale and the product in float32, as ATen's nearest_idx."""
    key = (n_in, n_out, str(device))
    idx = _NEAREST_IDX.get(key)
    if idx is None:
        scale = np.float32(n_in) / np.float32(n_out)
        src = np.floor(np.arange(n_out, dtype=np.float32) * scale).astype(np.int64)
        idx = torch.from_numpy(np.minimum(src, n_in - 1)).to(device)
        _NEAREST_IDX[key] = idx
    return idx


def interp_mask(mask, size):
    """backbone.py:89: nearest-neighbour resize of the padding mask, F.interpolate(mask[None]
    .float(), size).bool()[0] done as one gather of the output-sized mask (the float round trip
    over the full-resolution mask is ~30 us per batch-8 level on the GPU)."""
    h, w = int(size[0]), int(size[1])
    H, W = mask.shape[-2:]
    if mask.numel() == 0 or h == 0 or w == 0:
        return F.interpolate(mask[None].float(), size=size).to(torch.bool)[0]
    ih = _nearest_index(H, h, mask.device)
    iw = _nearest_index(W, w, mask.device)
    return mask[:, ih[:, None], iw[None, :]]


class BackboneBase(nn.Module):
    def __init__(self, body: nn.Module, train_backbone: bool, return_interm_layers: bool):
        super().__init__()
        for name, parameter in body.named_parameters():
            if (not train_backbone or 'layer2' not in name and 'layer3' not in name and 'layer4' not in name):
                parameter.requires_grad_(False)
        if return_interm_layers:
            self.strides = [4, 8, 16, 32]
            self.num_channels = [256, 512, 1024, 2048]
            self.return_idx = [0, 1, 2, 3]
        else:
            self.strides = [32]
            self.num_channels = [2048]
            self.return_idx = [3]
        self.body = body

    def forward_nhwc(self, img, dtype):
        outs = self.body.forward_nhwc(img, dtype)
        return [outs[i] for i in self.return_idx]

    def forward(self, tensor_list: NestedTensor, dtype=None):
        """backbone.py:83-91 -> {name: NestedTensor}; tensors are NCHW views of NHWC buffers."""
        dtype = dtype or torch.float32
        xs = self.forward_nhwc(tensor_list.tensors, dtype)
        out = OrderedDict()
        for i, x in enumerate(xs):
            mask = interp_mask(tensor_list.mask, x.shape[1:3])
            out[str(i)] = NestedTensor(nhwc_as_nchw(x), mask, tensor_list.sizes)
        return out


class Backbone(BackboneBase):
    """backbone.py:94-108 (ResNet with frozen BatchNorm; pretrained ImageNet weights are a
    remote fetch in the reference and are not fetched here -- load a state_dict instead)."""

    def __init__(self, name: str, train_backbone: bool, return_interm_layers: bool, dilation: bool):
        layers = {'resnet50': [3, 4, 6, 3], 'resnet101': [3, 4, 23, 3]}.get(name)
        if layers is None:
            raise ValueError(f'unsupported backbone {name}')
        super().__init__(ResNetBody(layers, dilation), train_backbone, return_interm_layers)


class Joiner(nn.Sequential):
    """backbone.py:180-194 (+ the `strides` attribute the reference forgot, :183)."""

    def __init__(self, backbone, position_embedding):
        super().__init__(backbone, position_embedding)
        self.num_channels = backbone.num_channels
        self.strides = backbone.strides

    def forward(self, tensor_list: NestedTensor, dtype=None):
        xs = self[0](tensor_list, dtype)
        out, pos = [], []
        for x in xs.values():
            out.append(x)
            pos.append(self._pos(x))
        return out, pos

    def _pos(self, x):
        """The position embedding of level x (a function of its padding mask only).  When the mask
        is fully determined by the image sizes (NestedTensor.sizes), the embedding is cached per
        (sizes, batch, level height / width, dtype, device) -- not per channel count, which it does
        not depend on -- in a small LRU: the training path's op-for-op forward otherwise
        recomputes 2 x 4 levels x frames of it per step, and multi-scale training cycles through
        geometries, so the least recently used entry goes first."""
        if x.sizes is None:
            return self[1](x).to(x.tensors.dtype)
        t = x.tensors
        key = (x.sizes, t.shape[0], t.shape[-2], t.shape[-1], t.dtype, str(t.device))
        cache = self.__dict__.get('_pos_cache')
        if cache is None:
            from collections import OrderedDict
            cache = self.__dict__['_pos_cache'] = OrderedDict()
        p = cache.get(key)
        if p is None:
            p = cache[key] = self[1](x).to(t.dtype)
            while len(cache) > self.POS_CACHE_ENTRIES:
                cache.popitem(last=False)
        else:
            cache.move_to_end(key)
        return p

    POS_CACHE_ENTRIES = 8


def build_backbone(args):
    return_interm_layers = args.masks or (args.num_feature_levels > 1)
    position_embedding = build_position_encoding(args)
    backbone = Backbone(args.backbone, args.lr_backbone > 0, return_interm_layers, args.dilation)
    return Joiner(backbone, position_embedding)

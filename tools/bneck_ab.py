"""A/B of the fused bottleneck pair (kinet_bottleneck_pair) at config 2, batch 16: per stage,
the pair launch against conv3 (+ residual + ReLU) followed by the next conv1 as two launches,
and the whole ResNet-50 body forward with FUSE_BOTTLENECK_PAIRS on / off (HIP events,
interleaved repeats).  usage: python tools/bneck_ab.py [--batch 16] [--iters 20] [--reps 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kinet_amd import kernels as K  # noqa: E402
from kinet_amd.models import backbone as BB  # noqa: E402


def time_call(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--reps', type=int, default=3)
    a = ap.parse_args()
    B, dt = a.batch, torch.bfloat16
    torch.manual_seed(0)
    body = BB.ResNetBody([3, 4, 6, 3]).cuda().eval()
    for D, DB, (H, W) in ((64, 64, (200, 334)), (64, 128, (200, 334)), (128, 128, (100, 167)), (256, 256, (50, 84))):
        F_ = 4 * D
        blk, nxt = BB.Bottleneck(F_, D).cuda(), BB.Bottleneck(F_, DB).cuda()
        x = torch.relu(torch.randn(B, H, W, D, device='cuda')).to(dt)
        res = torch.randn(B, H, W, F_, device='cuda').to(dt)
        s3, b3 = blk.bn3.folded()
        s1, b1 = nxt.bn1.folded()
        packed = K.bottleneck_pack(blk.conv3.weight, nxt.conv1.weight, s3, s1, dt)

        def fused():
            K.bottleneck_pair(x, res, packed, b3, b1)

        def plain():
            y = BB.conv_bn(x, blk.conv3, blk.bn3, True, residual=res)
            BB.conv_bn(y, nxt.conv1, nxt.bn1, True)
        time_call(plain, 5)
        for r in range(a.reps):
            tf, tp = time_call(fused, a.iters) * 1e3, time_call(plain, a.iters) * 1e3
            M = B * H * W
            gb = (M * D + M * DB + 2 * M * F_) * 2 / 1e9
            print(f'D={D} DB={DB} M={M}: pair {tf:.1f} us ({gb / tf * 1e3:.2f} TB/s algorithmic) | conv3 + conv1 {tp:.1f} us '
                  f'| saved {tp - tf:.1f} us', flush=True)
    img = torch.randn(B, 3, 800, 1333, device='cuda')

    def run(flag):
        def f():
            BB.FUSE_BOTTLENECK_PAIRS = flag
            BB.FUSE_PAIR_WIDTHS = (64,)
            body.forward_nhwc(img, dt)
        return f
    with torch.no_grad():
        run(True)()
        run(False)()
        for r in range(a.reps):
            t1, t0 = time_call(run(True), max(3, a.iters // 4)), time_call(run(False), max(3, a.iters // 4))
            print(f'ResNet-50 body batch {B}: fused pairs {t1:.3f} ms | unfused {t0:.3f} ms', flush=True)
    BB.FUSE_BOTTLENECK_PAIRS = True


if __name__ == '__main__':
    main()

"""Time the tap-folded ResNet stem at batch B: pack (f32 NCHW -> folded bf16) and the 7x1
(2, 1)-strided conv under each gemm_kernel tile.  python tools/stem_probe.py [B]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import timeit  # noqa: E402


def main():
    from kinet_amd import kernels as K, _native
    L = _native.lib()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dt = torch.bfloat16
    img = torch.randn(B, 3, 800, 1333, device='cuda')
    w = torch.randn(64, 3, 7, 7, device='cuda') * 0.1
    scale, bias = torch.rand(64, device='cuda') + 0.5, torch.randn(64, device='cuda')
    t = timeit(lambda: K.pack_image_kwfold(img, dt, 7, 2, 3, 24), iters=10)
    xp = K.pack_image_kwfold(img, dt, 7, 2, 3, 24)
    print(f'pack_image_kwfold: {t * 1e3:.1f} us ({(img.numel() * 4 + xp.numel() * 2) / t / 1e9:.2f} TB/s)')
    t = timeit(lambda: K.pack_image(img, dt, 8), iters=10)
    print(f'pack_image (8 ch): {t * 1e3:.1f} us')
    wp = K.pack_stem_weight(w, dt, 24)
    for flags, what in [(0, 'stem kernel (stem.hip)'), (32, 'resident-weight conv-row kernel')]:
        L.kinet_gemm_set_flags(flags)
        t = timeit(lambda: K.conv2d_nhwc(xp, wp, (2, 1), (3, 0), scale=scale, bias=bias, relu=True), iters=10)
        print(f'folded conv, {what}: {t * 1e3:.1f} us')
    L.kinet_gemm_set_flags(32 | 4)   # tiled kernel only
    for bm, bn in [(0, 0), (128, 64), (64, 64)]:
        L.kinet_gemm_force_tile(bm, bn)
        t = timeit(lambda: K.conv2d_nhwc(xp, wp, (2, 1), (3, 0), scale=scale, bias=bias, relu=True), iters=10)
        print(f'folded conv tile {bm}x{bn}: {t * 1e3:.1f} us')
    L.kinet_gemm_force_tile(0, 0)
    L.kinet_gemm_set_flags(0)


if __name__ == '__main__':
    main()

#!/usr/bin/env python
"""Kernel-level microbenchmarks (HIP events, same stream) for tuning:
  * GEMM / conv at the detector's shapes and at a square reference size,
  * per-launch-shape profile of one detector forward (config 2, bf16).
    python tools/bench_kernels.py [gemm] [model] [msda]
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def gemm():
    from kinet_amd import kernels as K
    dt = torch.bfloat16
    print('--- GEMM (bf16 in/out, bias) ---')
    for M, N, Kd in [(4096, 4096, 4096), (8192, 8192, 8192), (88892, 256, 256), (88892, 384, 256),
                     (88892, 1024, 256), (88892, 256, 1024), (1200, 256, 256), (1200, 512, 256), (1200, 1024, 256), (1200, 384, 256)]:
        x = torch.randn(M, Kd, device='cuda', dtype=dt)
        w = torch.randn(N, Kd, device='cuda') * 0.02
        b = torch.randn(N, device='cuda')
        ms = timeit(lambda: K.linear(x, w, b))
        print(f'M={M:6d} N={N:5d} K={Kd:5d}: {ms * 1e3:8.1f} us  {2 * M * N * Kd / ms / 1e9:7.1f} TF/s')
    print('--- conv NHWC (bf16) ---')
    for B, H, W, Cin, Cout, k, s in [(4, 200, 334, 64, 64, 3, 1), (4, 200, 334, 64, 256, 1, 1),
                                     (4, 200, 334, 256, 64, 1, 1), (4, 100, 167, 128, 128, 3, 1),
                                     (4, 50, 84, 256, 256, 3, 1), (4, 25, 42, 512, 512, 3, 1),
                                     (4, 50, 84, 1024, 256, 1, 1), (4, 800, 1333, 8, 64, 7, 2)]:
        x = torch.randn(B, H, W, Cin, device='cuda', dtype=dt)
        w = K.pack_conv_weight(torch.randn(Cout, Cin, k, k, device='cuda') * 0.02, dt)
        p = k // 2
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        ms = timeit(lambda: K.conv2d_nhwc(x, w, s, p))
        fl = 2 * B * Ho * Wo * Cout * k * k * Cin
        print(f'B{B} {H}x{W} {Cin}->{Cout} k{k}s{s}: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s')


def ffn():
    from kinet_amd import kernels as K
    dt = torch.bfloat16
    print('--- FFN sub-layer: fused kernel vs two GEMMs (bf16, d=256, F=1024, LN) ---')
    for M in [2400, 88892, 177784]:
        lin1, lin2, norm = torch.nn.Linear(256, 1024).cuda(), torch.nn.Linear(1024, 256).cuda(), torch.nn.LayerNorm(256).cuda()
        x = torch.randn(M, 256, device='cuda', dtype=dt)
        fused = timeit(lambda: K.ffn_fused(x, lin1, lin2, norm))
        two = timeit(lambda: K.linear(K.linear(x, lin1.weight, lin1.bias, relu=True), lin2.weight, lin2.bias,
                                      residual=x, ln=(norm.weight, norm.bias, norm.eps)))
        fl = 4 * M * 256 * 1024
        if M == 177784:
            from kinet_amd import _native
            for dbg in (1,):
                _native.lib().kinet_ffn_set_debug(dbg)
                t = timeit(lambda: K.ffn_fused(x, lin1, lin2, norm))
                print(f'   [debug {dbg}: {"no weight DMA" if dbg == 1 else "no MFMA" if dbg == 2 else "neither"}] {t * 1e3:7.1f} us')
            _native.lib().kinet_ffn_set_debug(0)
        print(f'M={M:7d}: fused {fused * 1e3:7.1f} us {fl / fused / 1e9:6.0f} TF/s | two GEMMs {two * 1e3:7.1f} us '
              f'{fl / two / 1e9:6.0f} TF/s')


def model():
    from kinet_amd import _native
    from kinet_amd.models import build_model, nested_tensor_from_tensor_list
    from kinet_amd.models.config import load_args
    m, _, _ = build_model(load_args('train_deformable'))
    m = m.cuda().eval().set_compute_dtype(torch.bfloat16)
    nb = int(os.environ.get('KINET_BENCH_BATCH', '8'))
    frames = nested_tensor_from_tensor_list([torch.randn(3, 800, 1333, device='cuda') for _ in range(nb)])
    with torch.no_grad():
        for _ in range(3):
            m(frames)
        torch.cuda.synchronize()
        _native.trace_begin()
        m(frames)
        tr = _native.trace_end()
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for name, work, s, e in tr:
        key = (work.get('family', name), work.get('shape', ''))
        a = agg[key]
        a[0] += 1
        a[1] += s.elapsed_time(e)
        a[2] += work.get('flops', 0)
        a[3] += work.get('bytes', 0)
    tot = sum(v[1] for v in agg.values())
    print(f'--- one forward, {nb} frames: {tot:.3f} ms device ---')
    for (f, sh), (n, ms, fl, by) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f'{f:8s} {str(sh):38s} n={n:3d} {ms:7.3f} ms {100 * ms / tot:5.1f}%  '
              f'{fl / ms / 1e9 if ms else 0:7.1f} TF/s  {by / ms / 1e6 if ms else 0:7.1f} GB/s')


if __name__ == '__main__':
    which = sys.argv[1:] or ['gemm', 'model']
    if 'rwsmall' in which:  # route small-M K<=256 GEMMs to the resident-weight kernel too
        from kinet_amd import _native
        _native.lib().kinet_gemm_set_flags(8)
        print('[bench_kernels] GEMM flags = 8 (resident-weight kernel from M >= 256)')
    if 'norw' in which:    # never use the resident-weight streaming kernel
        from kinet_amd import _native
        _native.lib().kinet_gemm_set_flags(4)
        print('[bench_kernels] GEMM flags = 4 (no resident-weight kernel)')
    if 'big' in which:     # the 8-wave LDS-DMA tiles wherever eligible
        from kinet_amd import _native
        _native.lib().kinet_gemm_set_flags(2)
        print('[bench_kernels] GEMM flags = 2 (8-wave LDS-DMA tiles)')
    if 'gemm' in which:
        gemm()
    if 'ffn' in which:
        ffn()
    if 'model' in which:
        model()

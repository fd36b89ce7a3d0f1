"""Per-launch table of one inference forward of a bench workload (default config 2) (bench.py's model and input), aggregated
by (kernel entry point, shape): launches, average us, achieved TFLOP/s and GB/s from the
algorithmic flops / bytes each launch reports, sorted by total time.  HIP events around every
launch on one stream (kinet_amd._native.trace_begin / trace_end).

usage: python tools/launch_table.py [--workload config2|config3|config5] [--batch N] [--top 40]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from kinet_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='config2', choices=sorted(bench.WORKLOADS))
    ap.add_argument('--batch', type=int, default=None, help='default: the workload\'s bench batch')
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--gemm-flags', type=int, default=0, help='kinet_gemm_set_flags value (A/B runs)')
    ap.add_argument('--filter', default='', help='only rows whose shape contains this text')
    ap.add_argument('--ffn-knob', type=int, default=0, help='kinet_ffn_set_debug value (A/B runs)')
    a = ap.parse_args()
    if a.gemm_flags:
        _native.lib().kinet_gemm_set_flags(a.gemm_flags)
    if a.ffn_knob:
        _native.lib().kinet_ffn_set_debug(a.ffn_knob)
    wl = bench.WORKLOADS[a.workload]
    a.batch = a.batch or wl['batch']
    dev = torch.device('cuda', 0)
    dt = {'bf16': torch.bfloat16, 'f16': torch.float16, 'f32': torch.float32}[wl['dtype']]
    model = bench.build(dev, dt, wl)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(a.batch, 3, wl['h'], wl['w'], device=dev, generator=g)
    extra = ()
    if wl['K']:
        # tracking inputs as bench.run_workload builds them: K track queries per frame and the
        # previous frame's features
        K_, d = wl['K'], model.hidden_dim
        with torch.no_grad():
            feats = model(list(torch.randn(a.batch, 3, wl['h'], wl['w'], device=dev, generator=g)))[2]
        boxes = torch.cat([torch.rand(a.batch, K_, 2, generator=g, device=dev) * 0.8 + 0.1,
                           torch.rand(a.batch, K_, 2, generator=g, device=dev) * 0.2 + 0.02], -1)
        hs = torch.randn(a.batch, K_, d, generator=g, device=dev)
        extra = ([{'track_query_hs_embeds': hs[b], 'track_query_boxes': boxes[b]} for b in range(a.batch)], feats)
    with torch.no_grad():
        for _ in range(2):
            model(list(x), *extra)
    torch.cuda.synchronize()
    _native.trace_begin()
    try:
        with torch.no_grad():
            model(list(x), *extra)
    finally:
        trace = _native.trace_end()
    torch.cuda.synchronize()
    agg = {}
    tot = 0.0
    for name, work, s, e in trace:
        ms = s.elapsed_time(e)
        tot += ms
        key = (name, str(work.get('shape', '')))
        r = agg.setdefault(key, [0, 0.0, 0.0, 0.0])
        r[0] += 1
        r[1] += ms
        r[2] += work.get('flops', 0.0)
        r[3] += work.get('bytes', 0.0)
    print(f'total traced device time {tot:.3f} ms over {len(trace)} launches (batch {a.batch})')
    rows = [kv for kv in sorted(agg.items(), key=lambda kv: -kv[1][1]) if a.filter in kv[0][1]]
    for (name, shape), (n, ms, fl, by) in rows[:a.top]:
        t = ms * 1e-3
        print(f'{ms / tot * 100:5.1f}% {n:3d} x {ms / n * 1e3:8.1f} us  {fl / t / 1e12 if t else 0:7.1f} TF/s '
              f'{by / t / 1e9 if t else 0:7.0f} GB/s  {name} {shape}')


if __name__ == '__main__':
    main()

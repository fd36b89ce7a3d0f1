"""Probe: which host ops of one batch-8 forward issue device-to-device memcpys
(rocprof shows them as __amd_rocclr_copyBuffer).  python tools/copy_probe.py"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from kinet_amd.models import nested_tensor_from_tensor_list
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    model = bench.build(dev, torch.bfloat16, bench.WORKLOADS['config2'])
    x = nested_tensor_from_tensor_list([torch.randn(3, 800, 1333, device=dev) for _ in range(8)])
    with torch.no_grad():
        for _ in range(2):
            model(x)
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
            model(x)
            torch.cuda.synchronize()
    names = ('aten::copy_', 'aten::clone', 'aten::contiguous', 'aten::cat', 'aten::stack', 'aten::to',
             'aten::_to_copy', 'aten::index', 'aten::repeat', 'aten::expand', 'aten::zeros', 'aten::fill_')
    from collections import Counter
    cnt = Counter()
    for e in prof.events():
        if e.name in names:
            st = [f for f in (e.stack or []) if 'kinet_amd' in f][:2]
            cnt[(e.name, str(e.input_shapes)[:60], ' <- '.join(st))] += 1
    for (n, shp, st), c in sorted(cnt.items(), key=lambda kv: -kv[1]):
        print(f'{c:3d}  {n:18s} {shp:60s} {st}')


if __name__ == '__main__':
    main()

"""Probe: capture one detection forward per in-flight slot in a HIP graph and replay it (bench
config 2: batch 16, 3 slots on 3 streams).  Checks the replayed outputs are bit-identical to the
eager forward's and times eager vs replay with the bench's stream pipelining.

    python tools/graph_probe.py [--steps 30] [--batch 16] [--streams 3] [--workload config2]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from kinet_amd.models import nested_tensor_from_tensor_list
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=30)
    ap.add_argument('--batch', type=int, default=None)
    ap.add_argument('--streams', type=int, default=None)
    ap.add_argument('--workload', default='config2')
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    B, nst = a.batch or wl['batch'], a.streams or wl['streams']
    dt = {'bf16': torch.bfloat16, 'f16': torch.float16, 'f32': torch.float32}[wl['dtype']]
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    model = bench.build(dev, dt, wl)
    g = torch.Generator(device=dev).manual_seed(1234)
    batches = [nested_tensor_from_tensor_list([torch.randn(3, wl['h'], wl['w'], generator=g, device=dev)
                                               for _ in range(B)]) for _ in range(nst)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(nst)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream(dev))

    def eager(i):
        with torch.no_grad(), torch.cuda.stream(streams[i % nst]):
            return model(batches[i % nst])

    for i in range(4):
        eager(i)
        torch.cuda.synchronize()
    refs = []
    for k in range(nst):
        o = eager(k)
        torch.cuda.synchronize()
        refs.append({key: o[0][key].clone() for key in ('pred_logits', 'pred_boxes')})

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    t_eager = timed(eager)
    graphs, outs = [], []
    pool = torch.cuda.graph_pool_handle()
    for k in range(nst):
        gr = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(gr, pool=pool, stream=streams[k]):
            outs.append(model(batches[k]))
        graphs.append(gr)
    torch.cuda.synchronize()

    def replay(i):
        with torch.cuda.stream(streams[i % nst]):
            graphs[i % nst].replay()

    for i in range(2 * nst):
        replay(i)
    torch.cuda.synchronize()
    for k in range(nst):
        for key in ('pred_logits', 'pred_boxes'):
            d = (outs[k][0][key].float() - refs[k][key].float()).abs().max().item()
            print(f'slot {k} {key}: max|graph replay - eager| = {d:.3e}', flush=True)
    t_graph = timed(replay)
    t_eager2 = timed(eager)
    t_graph2 = timed(replay)
    print(f'{a.workload} batch {B} x {nst} streams: eager {t_eager:.2f} / {t_eager2:.2f} ms per step '
          f'({B * 1e3 / t_eager:.1f} / {B * 1e3 / t_eager2:.1f} frames/s), graph replay {t_graph:.2f} / {t_graph2:.2f} '
          f'ms ({B * 1e3 / t_graph:.1f} / {B * 1e3 / t_graph2:.1f} frames/s)', flush=True)


if __name__ == '__main__':
    main()

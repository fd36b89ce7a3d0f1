"""Probe: capture one batch-8 detection forward per in-flight slot in a HIP graph and replay it.
Checks the replayed outputs are bit-identical to the eager forward's and times eager vs replay
with the bench's two-stream pipelining.   python tools/graph_probe.py [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from kinet_amd.models import nested_tensor_from_tensor_list
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    model = bench.build(dev, torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(1234)
    nst = 2
    batches = [nested_tensor_from_tensor_list([torch.randn(3, 800, 1333, generator=g, device=dev) for _ in range(8)])
               for _ in range(nst)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(nst)]

    def eager(i):
        with torch.no_grad(), torch.cuda.stream(streams[i % nst]):
            return model(batches[i % nst])

    for i in range(4):
        ref = eager(i)
    torch.cuda.synchronize()
    refs = []
    for k in range(nst):   # one batch in flight at a time, outputs cloned: the ground truth per slot
        o = eager(k)
        torch.cuda.synchronize()
        refs.append(({key: o[0][key].clone() for key in ('pred_logits', 'pred_boxes', 'hs_embed')},))
    o = eager(0)
    torch.cuda.synchronize()
    for key in ('pred_logits', 'pred_boxes', 'hs_embed'):
        d = (o[0][key].float() - refs[0][0][key].float()).abs().max().item() if key in refs[0][0] else float('nan')
        print(f'slot 0 {key}: max|serial eager rerun - serial eager| = {d:.3e}')
    from kinet_amd import kernels as K
    hs = o[0]['hs_embed'].to(torch.bfloat16)
    cls = model.class_embed[-1]
    y0 = K.linear(hs, cls.weight, cls.bias, out_dtype=torch.float32)
    torch.cuda.synchronize()
    yref = hs.float() @ cls.weight.to(torch.bfloat16).float().t() + cls.bias.float()
    worst = 0.0
    for _ in range(20):
        y = K.linear(hs, cls.weight, cls.bias, out_dtype=torch.float32)
        torch.cuda.synchronize()
        worst = max(worst, (y - y0).abs().max().item())
    print(f'class head {tuple(hs.shape)}x{tuple(cls.weight.shape)}: rerun spread {worst:.3e}, '
          f'vs torch fp32 {(y0 - yref).abs().max().item():.3e}, vs pred_logits {(y0 - o[0]["pred_logits"]).abs().max().item():.3e}')
    last = {}

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    def eager_keep(i):
        last[i % nst] = eager(i)

    t_eager = timed(eager_keep)
    for k in range(nst):
        for key in ('pred_logits', 'pred_boxes'):
            d = (last[k][0][key].float() - refs[k][0][key].float()).abs().max().item()
            print(f'slot {k} {key}: max|pipelined eager - serial eager| = {d:.3e}')

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

    for i in range(4):
        replay(i)
    torch.cuda.synchronize()
    for k in range(nst):
        for key in ('pred_logits', 'pred_boxes'):
            d = (outs[k][0][key].float() - refs[k][0][key].float()).abs().max().item()
            print(f'slot {k} {key}: max|graph - eager| = {d:.3e}')
    t_graph = timed(replay)
    print(f'eager {t_eager:.3f} ms/batch ({8e3 / t_eager:.0f} frames/s) | graph {t_graph:.3f} ms/batch '
          f'({8e3 / t_graph:.0f} frames/s)')


if __name__ == '__main__':
    main()

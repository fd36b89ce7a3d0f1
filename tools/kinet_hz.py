#!/usr/bin/env python
"""KineT model forward throughput on one MI355X: the shipped
cfgs/train_kinet.yaml model (d=288, 150 object queries, 1 encoder + 1 decoder layer per
stream) over synthetic detection frames -- tracking-style (batch 1, `--dets` detections, `--tracklets`
tracklet queries of `track_prev_frame_range` boxes) and batched (training-style batch 8,
no tracklets).  Random-init weights; detections are N(0,1)-free uniform boxes.

    python tools/kinet_hz.py [--dets 60] [--tracklets 30] [--iters 200]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dets', type=int, default=60)
    ap.add_argument('--tracklets', type=int, default=30)
    ap.add_argument('--iters', type=int, default=200)
    a = ap.parse_args()
    from kinet_amd.models import NestedTensor, NestedTensorKinet, build_model
    from kinet_amd.models.config import load_args
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model, _, _ = build_model(load_args('train_kinet', tracking=True, device='cuda'))
    model = model.to(dev)
    model.tracking()
    g = torch.Generator(device=dev).manual_seed(3)

    def frame(B, n):
        wh = torch.rand(B, n, 2, generator=g, device=dev) * 0.2 + 0.02
        cxcy = torch.rand(B, n, 2, generator=g, device=dev) * (1 - wh) + wh / 2
        mask = torch.zeros(B, n, dtype=torch.bool, device=dev)
        return NestedTensorKinet(NestedTensor(torch.cat([cxcy, wh], -1), mask),
                                 NestedTensor(torch.rand(B, n, 1, generator=g, device=dev), mask))

    res = {}
    for name, B, Kq in (('tracking_b1', 1, a.tracklets), ('batched_b8', 8, 0)):
        for dt in (torch.float32, torch.bfloat16):
            model.set_compute_dtype(dt)
            s = frame(B, a.dets)
            tg = None
            if Kq:
                tg = [{'track_query_hs_embeds_det': torch.rand(Kq, model.dim_tracklets_det, generator=g, device=dev),
                       'track_query_hs_embeds_meta': torch.rand(Kq, model.dim_tracklets_meta, generator=g, device=dev)}
                      for _ in range(B)]
            with torch.no_grad():
                for _ in range(10):
                    model(s, tg)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    model(s, tg)
                torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / a.iters
            key = f'{name}_{str(dt).split(".")[-1]}'
            res[key] = {'ms_per_forward': el * 1e3, 'frames_per_s': B / el}
            # the same forward replayed from a HIP graph (models/kinet.py graph_kinet_forward)
            from kinet_amd.models.kinet import graph_kinet_forward
            call = graph_kinet_forward(model, s, tg)
            for _ in range(10):
                call(s, tg)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                call(s, tg)
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / a.iters
            res[key + '_graph'] = {'ms_per_forward': el * 1e3, 'frames_per_s': B / el}
    print(json.dumps({'metric': 'KineT forward (cfgs/train_kinet.yaml model), frames/s', 'dets': a.dets,
                      'tracklets': a.tracklets, 'results': res}))


if __name__ == '__main__':
    main()

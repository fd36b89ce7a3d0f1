#!/usr/bin/env python
"""KineT tracking throughput: kinet_amd.tracker.TrackerKinematic driving the KineT kinematic
model (kinet_amd/models/kinet.py, cfgs/train_kinet.yaml: d = 288, 150 queries, 1 / 1 layers,
5-frame identity-encoded trails) over synthetic detection sequences, one step per frame as
src/track.py does (the reference reports 'RUNTIME ALL SEQS ... (x Hz)', track.py:209-214).

Synthetic: per frame --dets detections (cxcywh in [0, 1]) with a confidence value, random-init
weights; the class bias is set so that about --objects of the 150 queries pass the
cfgs/track_kinet.yaml thresholds (0.75 / 0.8), so the tracklet-query path runs from frame 2 on.

    python tools/kinet_track_hz.py [--seqs 4] [--frames 50] [--dtype bf16]
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seqs', type=int, default=4)
    ap.add_argument('--frames', type=int, default=50)
    ap.add_argument('--dets', type=int, default=40)
    ap.add_argument('--objects', type=int, default=30)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'f16', 'f32'])
    a = ap.parse_args()
    from fake_detector import KinetBlobSample, _Padded, kinematic_args
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    from kinet_amd.tracker import TrackerKinematic
    dev = torch.device('cuda', 0)
    args = load_args('train_kinet', tracking=True, device='cuda')
    torch.manual_seed(0)
    model, _, post = build_model(args)
    model = model.to(dev)
    model.tracking()
    model.set_compute_dtype({'bf16': torch.bfloat16, 'f16': torch.float16, 'f32': torch.float32}[a.dtype])
    cfg = dict(public_detections=False, detection_obj_score_thresh=0.75, track_obj_score_thresh=0.8,
               detection_nms_thresh=0.9, track_nms_thresh=0.0, steps_termination=2, prev_frame_dist=1,
               inactive_patience=5, reid_sim_threshold=0.0, reid_sim_only=False, reid_score_thresh=0.4,
               reid_greedy_matching=False, n_classes=1)
    ta = kinematic_args(False)
    ta.track_prev_frame_range = args.track_prev_frame_range

    def blobs(seed):
        g = torch.Generator().manual_seed(seed)
        out = []
        for _ in range(a.frames):
            wh = torch.rand(1, a.dets, 2, generator=g) * 0.1 + 0.02
            c = torch.rand(1, a.dets, 2, generator=g) * 0.8 + 0.1
            dets = torch.cat([c, wh], -1)
            meta = torch.rand(1, a.dets, 1, generator=g) * 0.5 + 0.5
            mask = torch.zeros(1, a.dets, dtype=torch.bool)
            out.append((KinetBlobSample(_Padded(dets, mask).to(dev), _Padded(meta, mask).to(dev)),
                        [{'orig_size': torch.tensor([1080, 1920], device=dev)}]))
        return out
    # class head: random-init logits are nearly equal across queries, so widen them first, then
    # set the bias so that about --objects queries pass the detection threshold on frame 0
    with torch.no_grad():
        model.class_embed.weight.normal_(0.0, 0.5, generator=torch.Generator(device=dev).manual_seed(1))
        b0 = blobs(0)[0][0]
        out = model(b0, None)[0]
        lg = out['pred_logits'][0].float().max(-1).values
        kth = lg.sort(descending=True).values[min(a.objects, lg.numel()) - 1]
        model.class_embed.bias += float(math.log(0.85 / 0.15) - kth)
    hz, tracks = [], []
    for s in range(a.seqs + 1):                      # sequence 0: warm-up
        tracker = TrackerKinematic(model, post, cfg, ta)
        tracker.reset()
        seq = blobs(100 + s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for blob in seq:
            tracker.step(blob)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if s:
            hz.append(a.frames / dt)
            tracks.append(tracker.track_num)
    print(json.dumps({'metric': 'KineT tracking frames/s (TrackerKinematic.step, batch 1)', 'value': sum(hz) / len(hz),
                      'unit': 'frames/s', 'per_seq': hz, 'tracks_per_seq': tracks, 'frames': a.frames,
                      'detections_per_frame': a.dets, 'dtype': a.dtype,
                      'model': 'KinetTracking d=288, 150 queries, 1/1 layers, 5-frame trails, random init'}))


if __name__ == '__main__':
    main()

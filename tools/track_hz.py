#!/usr/bin/env python
"""End-to-end tracking throughput (the reference reports it as
'RUNTIME ALL SEQS ... (x Hz)', track.py:209-214): kinet_amd.tracker.Tracker driving the
kinet_amd detector (config 3 tracking stack: multi-frame DeformableDETRTracking, d=288,
500 queries, prev-frame features, track queries) over synthetic sequences, one frame per
step as track.py does.

Synthetic: N(0,1) frames of --height x --width, random-init weights, the class bias
calibrated on frame 0 so that --objects queries (default 40, a MOT17-like crowd) pass the
cfgs/track.yaml detection threshold as persons; with the reference init's -4.6 prior bias no
detection would pass 0.4 and the track-query path would never run.

    python tools/track_hz.py [--seqs 8] [--frames 30] [--dtype f16]
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seqs', type=int, default=8)
    ap.add_argument('--frames', type=int, default=30)
    ap.add_argument('--height', type=int, default=800)
    ap.add_argument('--width', type=int, default=1333)
    ap.add_argument('--objects', type=int, default=40, help='detections above threshold on frame 0')
    ap.add_argument('--profile', action='store_true', help='cProfile the timed loop (top functions to stderr)')
    ap.add_argument('--dtype', default='f16', choices=['bf16', 'f16', 'f32'])
    a = ap.parse_args()
    from kinet_amd.models import build_model
    from kinet_amd.models.config import TRACKER_CFG, load_args
    from kinet_amd.tracker import Tracker
    dev = torch.device('cuda', 0)
    args = load_args('train_deformable', 'train_multi_frame', 'train_tracking', dataset='mot', device='cuda')
    torch.manual_seed(0)
    model, _, post = build_model(args)
    model = model.to(dev)
    model.tracking()
    model.set_compute_dtype({'bf16': torch.bfloat16, 'f16': torch.float16, 'f32': torch.float32}[a.dtype])
    g = torch.Generator(device=dev).manual_seed(7)
    frames = [torch.randn(1, 3, a.height, a.width, generator=g, device=dev) for _ in range(4)]
    size = torch.tensor([[a.height, a.width]], device=dev)
    # calibrate the class bias on frame 0 so that about --objects queries score above the
    # detection threshold as persons (class 0) and no other class competes
    with torch.no_grad():
        for ce in model.class_embed:
            ce.bias.fill_(-20.0)
            ce.bias[0] = 0.0
        logits = model(frames[0])[0]['pred_logits'][0, :, 0].float()
        thr = math.log(TRACKER_CFG['detection_obj_score_thresh'] / (1 - TRACKER_CFG['detection_obj_score_thresh']))
        b = thr - torch.sort(logits, descending=True)[0][a.objects].item()
        for ce in model.class_embed:
            ce.bias[0] = b
    tracker = Tracker(model, post, dict(TRACKER_CFG))
    # warm-up sequence (kernel caches, geometry)
    tracker.reset()
    for i in range(3):
        tracker.step({'img': frames[i % 4], 'orig_size': size, 'dets': [torch.zeros(0, 4)]})
    torch.cuda.synchronize()
    n_frames, n_tracks, tq = 0, 0, []
    prof = None
    if a.profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for s in range(a.seqs):
        tracker.reset()
        for f in range(a.frames):
            tq.append(len(tracker.tracks) + len(tracker.inactive_tracks))
            tracker.step({'img': frames[(s + f) % 4], 'orig_size': size, 'dets': [torch.zeros(0, 4)]})
            n_frames += 1
        n_tracks += len(tracker.get_results())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats('tottime').print_stats(30)
    # where a frame's time goes: the detector forward alone with K ~ the mean track-query count
    # (device-synchronised per frame), and its host enqueue time (no sync)
    kq = max(1, int(round(sum(tq) / len(tq))))
    tgt = [{'track_query_boxes': torch.rand(kq, 4, generator=g, device=dev) * 0.5 + 0.1,
            'track_query_hs_embeds': torch.randn(kq, model.hidden_dim, generator=g, device=dev),
            'image_id': torch.tensor([1], device=dev)}]
    with torch.no_grad():
        _, _, feats, _, _ = model(frames[0])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(20):
            model(frames[i % 4], tgt, feats)
            torch.cuda.synchronize()
        det_ms = (time.perf_counter() - t1) / 20 * 1e3
        t1 = time.perf_counter()
        for i in range(20):
            model(frames[i % 4], tgt, feats)
        host_ms = (time.perf_counter() - t1) / 20 * 1e3
        torch.cuda.synchronize()
    print(json.dumps({'metric': 'tracking Hz (track.py:209-214), one frame per step', 'value': n_frames / el,
                      'unit': 'frames/s', 'frames': n_frames, 'seqs': a.seqs, 'seconds': el,
                      'tracks_per_seq': n_tracks / a.seqs, 'mean_track_queries': sum(tq) / len(tq),
                      'dtype': a.dtype, 'frame': [3, a.height, a.width],
                      'detector_ms_per_frame_synced': det_ms, 'detector_host_enqueue_ms': host_ms,
                      'tracker_ms_per_frame': el / n_frames * 1e3,
                      'config': 'config3 tracking stack (multi-frame deformable, d=288, 500 queries), '
                                'cfgs/track.yaml tracker_cfg'}))


if __name__ == '__main__':
    main()

#!/usr/bin/env python
"""Throughput benchmark of the detection hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1], cfgs/train_deformable.yaml): ResNet-50 +
Deformable-DETR (d=256, 4 levels, 8 heads, 4 points, FFN 1024, 6/6 layers, 300 queries,
iterative box refinement, 91 focal logits) on synthetic 3x800x1333 frames, bf16 compute,
all kernels hand-written HIP (kinet_amd).  One step = one detection forward over a batch
of `--batch` frames per GPU whose pixels are already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--workload config2|config3|config5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (driver)

`--workload config5` (BASELINE.json configs[4], cfgs/train_full_res.yaml): ResNet-101,
d=288 (head_dim 36), 500 object + 20 track queries, separate per-frame encoders and an
8-level decoder over [current, prev] memory, fp16, 1080x1920 frames; one step = one
tracking forward per frame with the previous frame's features (resident in HBM, as the
online tracker holds them) -- the HBM-stress case for MSDeformAttn (S = 43,110 per frame).

Multi-GPU: frames are independent -> one replica per GPU, no data-path collective
("scaling": "weak"); a barrier + max-over-ranks wall time brackets the timed region.  The
config-4 `train` sub-object runs its DDP step (RCCL gradient all-reduce) over the same ranks.
`--gpus N` alone (no WORLD_SIZE from a launcher) starts N rank processes itself before any GPU
call; n_gpus is the process group's size.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MFMA_PEAK_TFLOPS = {'bf16': 2500.0, 'f16': 2500.0, 'f32': 157.3}   # dense
# per-launch HBM bytes from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over this bench command
# (tools/pmc_traffic.py; FETCH_SIZE x2 on gfx950 per MI355X_MICROARCH.md "HBM")
PMC_TRAFFIC = os.path.join(HERE, 'profiles', 'pmc_traffic.json')
# MFMA-pipe utilisation per kernel group from a rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE
# pass over the config-2 forward (tools/pmc_mfma.py)
PMC_MFMA = os.path.join(HERE, 'profiles', 'pmc_mfma.json')

WORKLOADS = {
    # batch per in-flight slot: the interleaved --batch sweeps of round 5 (profiles/r05zz_batch_sweep.txt)
    # -- config 2: 16 -> 1314-1321, 24 -> 1352-1358, 28 -> 1353-1355, 32 -> 1299-1302 frames/s;
    # config 3: 8 -> 610-613, 12 -> 627-630, 16 -> 616; config 5: 4, 6, 8 within 1 %.  Round 6, with
    # the bottleneck pairs at every width (profiles/r06e_batch_sweep.txt): config 2 24 -> 1366 / 1372,
    # 28 -> 1378 / 1380, 32 -> 1338 / 1333; 24 with 4 batches in flight 1352 / 1352
    'config2': dict(cfgs=('train_deformable',), over={}, h=800, w=1333, batch=28, streams=3, dtype='bf16',
                    K=0, desc='config2 cfgs/train_deformable.yaml: R-50 Deformable-DETR inference forward, '
                              'd=256, 4 levels, 6/6 layers, 300 queries, box refine'),
    'config3': dict(cfgs=('train_deformable', 'train_multi_frame', 'train_tracking'), over=dict(dataset='mot'),
                    h=800, w=1333, batch=12, streams=3, dtype='f16', K=20,
                    desc='config3 tracking forward (cfgs/train_tracking.yaml on the multi-frame d=288 stack): R-50, '
                         '500 object + 20 track queries (SURVEY 8(d) row 3), separate per-frame encoders (L=4), 8-level decoder, '
                         'prev-frame features resident, 800x1333 frame pairs'),
    'config5': dict(cfgs=('train_deformable', 'train_multi_frame', 'train_tracking', 'train_full_res'),
                    over=dict(dataset='mot', backbone='resnet101'), h=1080, w=1920, batch=4, streams=3, dtype='f16',
                    K=20, desc='config5 cfgs/train_full_res.yaml: R-101 multi-frame tracking forward, d=288, '
                               '500 object + 20 track queries, separate per-frame encoders (L=4), 8-level decoder, '
                               'prev-frame features resident'),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--workload', default='config2', choices=sorted(WORKLOADS))
    ap.add_argument('--batch', type=int, default=None, help='frames per GPU per step')
    ap.add_argument('--streams', type=int, default=None,
                    help='batches in flight per GPU, each on its own HIP stream (serving-style pipelining)')
    ap.add_argument('--graph', type=int, default=1,
                    help='1: each in-flight slot\'s forward captured once in a HIP graph after the warm-up and '
                         'replayed for the timed steps (bit-identical to eager, tools/graph_probe.py); 0: eager')
    ap.add_argument('--height', type=int, default=None)
    ap.add_argument('--width', type=int, default=None)
    ap.add_argument('--dtype', default=None, choices=['bf16', 'f16', 'f32'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-train', action='store_true', help='skip the config-4 training sub-benchmark')
    ap.add_argument('--no-config5', action='store_true', help='skip the config-5 sub-benchmark of the default line')
    ap.add_argument('--no-config3', action='store_true', help='skip the config-3 sub-benchmark of the default line')
    ap.add_argument('--config5-steps', type=int, default=8)
    ap.add_argument('--config3-steps', type=int, default=8)
    ap.add_argument('--train-steps', type=int, default=10)
    ap.add_argument('--cpu-seconds', type=float, default=20.0, help='bound on the CPU baseline sample')
    ap.add_argument('--ffn-knob', type=int, default=0,
                    help='fused-FFN tile A/B knob (kinet_ffn_set_debug: 2 = 4 waves x 32 rows at D = 256)')
    ap.add_argument('--gemm-flags', type=int, default=0,
                    help='diagnostic kernel-selection flags (kinet_gemm_set_flags, csrc/gemm.hip) for A/B runs; '
                         'per calling thread, so the train leg\'s autograd backward (torch\'s engine thread) '
                         'keeps the default kernels')
    ap.add_argument('--msda-records', type=int, default=1,
                    help='1: encoder MSDA calls through the sampling records (kinet_msda_sample_records); '
                         '0: the f16 offsets / logits path (A/B)')
    ap.add_argument('--bneck-pairs', type=int, default=1,
                    help='1: ResNet stage-1 bottleneck pairs (conv3 -> next conv1) as one launch '
                         '(kinet_bottleneck_pair); 0: every conv on its own (A/B)')
    ap.add_argument('--pair-widths', default=None,
                    help='comma list of bottleneck widths whose conv3 -> next conv1 run as one kinet_bottleneck_pair '
                         'launch (backbone.FUSE_PAIR_WIDTHS; A/B)')
    ap.add_argument('--share-pos', type=int, default=1,
                    help='1: unpadded frames read one shared position embedding in the encoder projections '
                         '(DeformableTransformer.share_frame_pos); 0: per-frame rows (A/B)')
    ap.add_argument('--enc-strips', type=int, default=0,
                    help='strips per head map of the encoder sampler (kernels.msda_encoder_set_strips; 0 = the '
                         "plan's own choice; A/B)")
    ap.add_argument('--stem-image', type=int, default=1,
                    help='1: the stem conv reads the f32 image directly (kinet_stem_conv_image); '
                         '0: pack_image_kwfold + the folded conv (A/B)')
    ap.add_argument('--ddp-find-unused', type=int, default=1,
                    help='train leg: DistributedDataParallel find_unused_parameters (1 = the reference, '
                         'train.py:89-91; 0 skips the extra graph traversal -- every parameter gets a gradient)')
    ap.add_argument('--detail', default=None,
                    help='where the full JSON record goes (default gpurun_out/bench_detail.json); stdout '
                         'carries the compact line')
    ap.add_argument('--cpu-stub', action='store_true',
                    help='tests only: run the launch/timing skeleton with a tiny CPU model over gloo')
    a = ap.parse_args()
    wl = WORKLOADS[a.workload]
    for k, wk in (('batch', 'batch'), ('streams', 'streams'), ('height', 'h'), ('width', 'w'), ('dtype', 'dtype')):
        if getattr(a, k) is None:
            setattr(a, k, wl[wk])
    return a


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`--gpus N` without an external launcher (no WORLD_SIZE in the environment): start N
    worker processes of this script, one per GPU, each with RANK / LOCAL_RANK / WORLD_SIZE
    and a 127.0.0.1 rendezvous -- as torch.distributed.run would (util/misc.py:515-538 reads
    the same variables).  This parent has not touched the GPU (nothing before this call
    initialises HIP) and stays alive as the children's supervisor: it waits for them, stops
    the others when one fails (a peer blocked in a collective would otherwise hang) and
    exits with the first non-zero status."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.2)
    return rc


def setup_dist(a):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if a.cpu_stub:
        if world > 1:
            dist.init_process_group('gloo')
        return world, rank, torch.device('cpu')
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        world = dist.get_world_size()   # the process group's own count, reported as n_gpus
    else:
        torch.cuda.set_device(0)
    if world != a.gpus:
        raise SystemExit(f'bench.py: --gpus {a.gpus} but the process group has {world} ranks')
    return world, rank, torch.device('cuda', local if world > 1 else 0)


def stub_main(a, world, rank, dev):
    """--cpu-stub: the launch / rendezvous / timing / reporting skeleton of main() with a
    tiny CPU stand-in for the detector (tests only: checks that `--gpus N` yields N ranks
    and an n_gpus = N line without a GPU)."""
    x = torch.randn(a.batch, 64)
    w = torch.randn(64, 64)
    for _ in range(max(1, a.warmup)):
        x = torch.tanh(x @ w)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        x = torch.tanh(x @ w)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        assert dist.get_world_size() == a.gpus
    if rank == 0:
        print(json.dumps({'metric': 'cpu stub', 'value': a.batch * a.steps * world / elapsed, 'unit': 'frames/s',
                          'n_gpus': world, 'world_size': dist.get_world_size() if world > 1 else 1,
                          'steps': a.steps, 'warmup': a.warmup, 'scaling': 'weak', 'stub': True}))
    if world > 1:
        dist.destroy_process_group()


def build(dev, dtype, wl):
    from kinet_amd.models import build_model
    from kinet_amd.models.config import load_args
    torch.manual_seed(0)
    model, _, _ = build_model(load_args(*wl['cfgs'], device='cuda', **wl['over']))
    model = model.to(dev).eval()
    if wl['K']:
        model.tracking()
    model.set_compute_dtype(dtype)
    return model


def roofline_split(trace, steps_traced, peak_tflops):
    """GEMM / conv launches split at the ridge point (dense MFMA peak / HBM peak, flop per
    byte): the compute-bound ones held against the MFMA peak, the HBM-bound ones (1x1 convs and
    K <= 256 projections over hundreds of thousands of rows) against HBM -- plus the fused FFN
    and the multi-tap (3x3 / 7x1) convolutions on their own, the kernels north_star's MFMA
    target names.  Algorithmic flops / bytes per launch over HIP-event launch times."""
    ridge = peak_tflops * 1e12 / (HBM_PEAK_GBS * 1e9)
    acc = {k: {'launches': 0, 'ms': 0.0, 'flops': 0.0, 'bytes': 0.0} for k in ('compute', 'hbm', 'ffn', 'conv_kxk')}
    for name, work, s, e in trace:
        fam = work.get('family')
        fl, by = work.get('flops', 0.0), work.get('bytes', 0.0)
        if fam not in ('gemm', 'conv') or not fl or not by:
            continue
        ms = s.elapsed_time(e)
        keys = ['compute' if fl / by >= ridge else 'hbm']
        shape = work.get('shape', ())
        if shape and shape[0] == 'ffn':
            keys.append('ffn')
        if fam == 'conv' and len(shape) >= 6 and shape[5] > 1:
            keys.append('conv_kxk')
        for k in keys:
            a = acc[k]
            a['launches'] += 1
            a['ms'] += ms
            a['flops'] += fl
            a['bytes'] += by
    out = {'ridge_flop_per_byte': ridge}
    for k, a in acc.items():
        if not a['launches']:
            continue
        t = a['ms'] * 1e-3
        ent = {'launches_per_step': a['launches'] / steps_traced, 'ms_per_step': a['ms'] / steps_traced}
        if k == 'hbm':
            ent.update(achieved=a['bytes'] / t / 1e9, unit='GB/s', peak=HBM_PEAK_GBS,
                       frac=a['bytes'] / t / 1e9 / HBM_PEAK_GBS)
        else:
            ent.update(achieved=a['flops'] / t / 1e12, unit='TFLOP/s', peak=peak_tflops,
                       frac=a['flops'] / t / 1e12 / peak_tflops)
        out[k] = ent
    return out


def summarize_trace(trace, steps_traced=1):
    fam = {}
    msda = []
    for name, work, s, e in trace:
        ms = s.elapsed_time(e)
        f = work.get('family', name)
        a = fam.setdefault(f, {'ms': 0.0, 'flops': 0.0, 'bytes': 0.0, 'launches': 0})
        a['ms'] += ms
        a['flops'] += work.get('flops', 0.0)
        a['bytes'] += work.get('bytes', 0.0)
        a['launches'] += 1
        if f == 'msda':
            msda.append((work.get('Lq'), work.get('S'), ms, work['bytes'], work.get('kernel', '?')))
        elif work.get('role') == 'msda_prep':
            # the projection that prepares an MSDA call (sampling records / offsets + logits):
            # Lq = rows per frame, S = None (it is neither an encoder nor a decoder sampler launch)
            msda.append((work['shape'][0], None, ms, work['bytes'], name, 'prep'))
    for a in fam.values():
        for k in ('ms', 'flops', 'bytes', 'launches'):
            a[k] /= steps_traced
    return fam, msda


def decoder_touched_bytes(model, samples, extra):
    """Bytes the decoder's sampling kernel must move per call: the value rows (pixel, head)
    its bilinear corners actually touch -- counted from the sampling locations of one more
    forward -- plus its offsets / logits, references and output.  The decoder's 300 queries x
    8 heads x 16 samples touch a small part of each value map, so the whole map is not the
    compulsory traffic of that kernel."""
    from kinet_amd import kernels as K
    calls = []
    orig = K.msda_fused

    def spy(value, spatial_shapes, offlog, reference_points, n_heads, n_levels, n_points, query_attn_mask=None,
            want_loc_attw=False, head_major=False, out_dtype=None, query_tile_order=None):
        out = orig(value, spatial_shapes, offlog, reference_points, n_heads, n_levels, n_points, query_attn_mask,
                   want_loc_attw, head_major, out_dtype, query_tile_order)
        S = value.shape[2] if head_major else value.shape[1]
        if not want_loc_attw and offlog.shape[1] != S:
            calls.append((value, spatial_shapes, offlog, reference_points, n_heads, n_levels, n_points,
                          query_attn_mask, head_major, out_dtype))
        return out
    K.msda_fused = spy
    try:
        with torch.no_grad():
            model(samples, *extra)
    finally:
        K.msda_fused = orig
    res = []
    for value, ss, offlog, ref, M, L, P, qm, hm, od in calls:
        o, loc, _ = orig(value, ss, offlog, ref, M, L, P, qm, True, hm, od)
        B, Lq = loc.shape[:2]
        D = value.shape[-1]
        S = value.shape[2] if hm else value.shape[1]
        keys = []
        start = 0
        bm = (torch.arange(B, device=loc.device)[:, None, None, None] * M +
              torch.arange(M, device=loc.device)[None, None, :, None])          # (B, 1, M, 1)
        for l, (H, W) in enumerate(ss.tolist()):
            x, y = loc[:, :, :, l, :, 0], loc[:, :, :, l, :, 1]                   # (B, Lq, M, P)
            h, w = y * H - 0.5, x * W - 0.5
            inside = (h > -1) & (w > -1) & (h < H) & (w < W)
            hl, wl = torch.floor(h).long(), torch.floor(w).long()
            for dy in (0, 1):
                for dx in (0, 1):
                    r, c = hl + dy, wl + dx
                    ok = inside & (r >= 0) & (r < H) & (c >= 0) & (c < W)
                    k = (bm * S + start + r * W + c)[ok]
                    keys.append(k)
            start += H * W
        rows = torch.unique(torch.cat(keys)).numel()
        res.append(rows * D * value.element_size() + offlog.numel() * offlog.element_size() + ref.numel() * 4
                   + o.numel() * o.element_size())
    return statistics.mean(res) if res else None


def kernel_names(launches):
    """The kernel instantiation(s) the traced MSDA launches ran (reported by kinet_amd.kernels
    from the launcher's own dispatch), as rocprofv3 names them."""
    return ' | '.join(sorted({m[4] for m in launches}))


def pmc_traffic(key):
    """(bytes per launch, provenance) of kernel `key` = '<workload>:<kernel name>' from the
    committed PMC summary (tools/pmc_traffic.py), or (None, None)."""
    try:
        with open(PMC_TRAFFIC) as f:
            d = json.load(f)
        k = d['kernels'][key]
        return k['hbm_bytes_per_launch'], d['sources'].get(key.split(':')[0])
    except (OSError, KeyError, ValueError):
        return None, None


def pmc_mfma_util():
    """Counter-measured MFMA busy fraction of the committed pass (groups + provenance), or None."""
    try:
        with open(PMC_MFMA) as f:
            d = json.load(f)
        return {'groups': d['groups'], 'source': d.get('source'),
                'definition': 'SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) over the group\'s '
                              'dispatches: the fraction of matrix-core cycles kept busy (1.0 = the dense peak '
                              'at the clock the kernels ran)'}
    except (OSError, KeyError, ValueError):
        return None


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for ln in f:
                if ln.startswith('model name'):
                    return ln.split(':', 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(seconds):
    """Reference CPU path (ms_deform_attn_core_pytorch, restated in oracle/msda_oracle.py)
    on one frame's MSDA work of the same workload: 6 encoder calls (Lq = S = 22,223) and
    6 decoder calls (Lq = 300), fp32, all host threads; plus the config-5 encoder call
    (S = 43,110 at 1080x1920, head_dim 36) that SURVEY 8(d) names."""
    from oracle.msda_oracle import core_pytorch
    # the box's CPU share (OMP_NUM_THREADS=16 there); os.cpu_count() reports the whole host
    threads = int(os.environ.get('OMP_NUM_THREADS') or torch.get_num_threads() or 1)
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    shapes = torch.tensor([[100, 167], [50, 84], [25, 42], [13, 21]], dtype=torch.long)
    S = int((shapes[:, 0] * shapes[:, 1]).sum())
    M, D, L, P = 8, 32, 4, 4
    value = torch.randn(1, S, M, D, generator=g)

    def call(Lq):
        loc = torch.rand(1, Lq, M, L, P, 2, generator=g)
        attw = torch.rand(1, Lq, M, L, P, generator=g)
        attw /= attw.sum((-1, -2), keepdim=True)
        t0 = time.perf_counter()
        core_pytorch(value, shapes, loc, attw)
        return time.perf_counter() - t0

    call(S)   # warm-up
    enc, dec = [], []
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < seconds and len(enc) < 7:
        enc.append(call(S))
        dec.append(call(300))
    t_enc, t_dec = statistics.median(enc), statistics.median(dec)
    frame_s = 6 * t_enc + 6 * t_dec
    # config 5 encoder call: 4 levels of a 1080x1920 frame, d=288 (M=8, D=36), Lq = S
    shapes5 = torch.tensor([[135, 240], [68, 120], [34, 60], [17, 30]], dtype=torch.long)
    S5 = int((shapes5[:, 0] * shapes5[:, 1]).sum())
    value5 = torch.randn(1, S5, M, 36, generator=g)
    loc5 = torch.rand(1, S5, M, L, P, 2, generator=g)
    attw5 = torch.rand(1, S5, M, L, P, generator=g)
    attw5 /= attw5.sum((-1, -2), keepdim=True)
    t5 = []
    for _ in range(2):
        t0 = time.perf_counter()
        core_pytorch(value5, shapes5, loc5, attw5)
        t5.append(time.perf_counter() - t0)
    return {'value': 1.0 / frame_s, 'unit': 'frames/s (MSDA share only; upper bound of the CPU detector)',
            'cores': threads, 'cpu_model': cpu_model(), 'kind': 'port',
            'sample': f'{len(enc)} frames of MSDeformAttn work on the host CPU: 6 encoder calls '
                      f'(Lq=S={S}, median {t_enc * 1e3:.1f} ms) + 6 decoder calls (Lq=300, median '
                      f'{t_dec * 1e3:.2f} ms), fp32 ms_deform_attn_core_pytorch restatement; plus 2 config-5 '
                      f'encoder calls (Lq=S={S5}, D=36, min {min(t5) * 1e3:.1f} ms)',
            'msda_encoder_ms_per_call': t_enc * 1e3, 'msda_decoder_ms_per_call': t_dec * 1e3,
            'config5_msda_encoder_ms_per_call': min(t5) * 1e3}


def train_leg(a, dev, world):
    """The config-4 training sub-benchmark.  Under `--gpus N` it runs on the bench's own RCCL
    group; at N = 1 (no launcher, no group) the step still runs under DistributedDataParallel
    over a 1-rank "nccl" group created here, in this process -- RCCL initialisation, the DDP
    reducer's bucketed all-reduce and find_unused_parameters (train.py:88-91) then run on the
    hardware exactly as at N > 1; the group is destroyed after the leg."""
    from kinet_amd.train import benchmark_train
    own = False
    if world == 1 and not dist.is_initialized():
        dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{_free_port()}', rank=0, world_size=1,
                                device_id=dev)
        own = True
    try:
        return benchmark_train(steps=a.train_steps, warmup=2, device=dev,
                               find_unused_parameters=bool(a.ddp_find_unused))
    finally:
        if own:
            dist.destroy_process_group()


def run_workload(a, name, dev, world, rank, batch, streams, height, width, dtype_name, steps, warmup):
    """Time `steps` forwards of workload `name` (WORKLOADS) after `warmup`, then trace 3 more on
    one stream.  Returns (elapsed seconds (max over ranks), trace families, MSDA launches,
    GEMM/conv roofline split, decoder touched bytes).  With one batch in flight the library's
    launch-fill policy is "solo" (kinet_set_solo_launch: partial-round shapes on smaller tiles)."""
    from kinet_amd import _native
    old = _native.lib().kinet_set_solo_launch(1 if max(1, streams) == 1 else 0)
    try:
        return _run_workload(a, name, dev, world, rank, batch, streams, height, width, dtype_name, steps, warmup)
    finally:
        _native.lib().kinet_set_solo_launch(old)


def _run_workload(a, name, dev, world, rank, batch, streams, height, width, dtype_name, steps, warmup):
    from kinet_amd import _native
    from kinet_amd.models import nested_tensor_from_tensor_list
    wl = WORKLOADS[name]
    dtype = {'bf16': torch.bfloat16, 'f16': torch.float16, 'f32': torch.float32}[dtype_name]
    model = build(dev, dtype, wl)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    # one independent batch per in-flight slot (distinct requests, all resident in HBM)
    nst = max(1, streams)
    batches = [nested_tensor_from_tensor_list([torch.randn(3, height, width, generator=g, device=dev)
                                               for _ in range(batch)]) for _ in range(nst)]
    extra = [() for _ in range(nst)]
    if wl['K']:
        # tracking step inputs per slot: K track queries per frame (hs embeddings + boxes of
        # the previous frame's detections) and the previous frame's backbone features
        K_, d = wl['K'], model.hidden_dim
        for i in range(nst):
            prev = nested_tensor_from_tensor_list([torch.randn(3, height, width, generator=g, device=dev)
                                                   for _ in range(batch)])
            with torch.no_grad():
                feats = model(prev)[2]
            boxes = torch.cat([torch.rand(batch, K_, 2, generator=g, device=dev) * 0.8 + 0.1,
                               torch.rand(batch, K_, 2, generator=g, device=dev) * 0.2 + 0.02], -1)
            hs = torch.randn(batch, K_, d, generator=g, device=dev)
            targets = [{'track_query_hs_embeds': hs[b], 'track_query_boxes': boxes[b]} for b in range(batch)]
            extra[i] = (targets, feats)
        torch.cuda.synchronize()
    strs = [torch.cuda.Stream(device=dev) for _ in range(nst)]
    for st in strs:   # the input batches were written on the default stream
        st.wait_stream(torch.cuda.current_stream(dev))
    samples = batches[0]

    def step(i=0):
        with torch.no_grad():
            if nst == 1:
                return model(batches[0], *extra[0])
            # step i runs batch i % nst on its own stream: the decoder / small-kernel phases of
            # one batch overlap the backbone of the next (no host syncs anywhere in a forward)
            with torch.cuda.stream(strs[i % nst]):
                return model(batches[i % nst], *extra[i % nst])

    eager_step = step
    for i in range(max(1, warmup)):
        out = step(i)
        if i == 0:
            # step 0 fills the weight-pack / geometry caches on its stream; the other
            # streams read them from step 1 on
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    graphed = False
    graph_check = None
    if getattr(a, 'graph', 0):
        # one HIP graph per in-flight slot: the whole forward of that slot's batch (the same
        # kernels, buffers and streams as the eager step), replayed for every timed step; each
        # slot captures into its OWN memory pool (the slots replay concurrently on their streams)
        eager = []
        for k in range(nst):   # the eager outputs of every slot, kept to check the replays against
            o = step(k)
            # step k ran on strs[k]: wait for it before copying its outputs on this stream
            torch.cuda.synchronize()
            eager.append((o[0]['pred_logits'].clone(), o[0]['pred_boxes'].clone()))
        torch.cuda.synchronize()
        try:
            graphs, gouts = [], []
            for k in range(nst):
                gr = torch.cuda.CUDAGraph()
                with torch.no_grad(), torch.cuda.graph(gr, pool=torch.cuda.graph_pool_handle(), stream=strs[k]):
                    gouts.append(model(batches[k], *extra[k]))
                graphs.append(gr)
            torch.cuda.synchronize()

            def step(i=0):   # noqa: F811
                with torch.cuda.stream(strs[i % nst]):
                    graphs[i % nst].replay()
                return gouts[i % nst]
            for i in range(2 * nst):   # every slot replayed twice, concurrently with the others
                out = step(i)
            torch.cuda.synchronize()
            # the forward is deterministic (fixed-order reductions): replays must equal eager bit for bit
            same = all(torch.equal(gouts[k][0]['pred_logits'], eager[k][0]) and
                       torch.equal(gouts[k][0]['pred_boxes'], eager[k][1]) for k in range(nst))
            if same:
                graphed, graph_check = True, 'replays bit-identical to eager (every slot)'
            else:
                diffs = [float((gouts[k][0]['pred_logits'].float() - eager[k][0].float()).abs().max()) for k in range(nst)]
                print(f'[bench] {name}: graph replay differs from eager (max |dlogits| per slot {diffs}), timing eager',
                      file=sys.stderr)
                graph_check = 'replay differed from eager: timed eager'
                del graphs, gouts
                step = eager_step
        except RuntimeError as ex:   # a capture-unsafe host sync: stay eager (reported in the line)
            print(f'[bench] {name}: HIP graph capture failed ({str(ex)[:120]}), timing eager', file=sys.stderr)
            graph_check = 'capture failed: timed eager'
            step = eager_step
            torch.cuda.synchronize()
        del eager
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        out = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    assert torch.isfinite(out[0]['pred_boxes']).all()
    del out
    if graphed:
        del graphs, gouts
    run_workload.graphed[name] = graphed
    run_workload.graph_check[name] = graph_check

    # roofline pass: HIP events around every launch of 3 more steps, one stream (the traced
    # kernel durations must not overlap)
    _native.trace_begin()
    try:
        for _ in range(3):
            with torch.no_grad():
                model(samples, *extra[0])
    finally:
        trace = _native.trace_end()
    torch.cuda.synchronize()
    fam, msda = summarize_trace(trace, 3)
    dec_touched = decoder_touched_bytes(model, samples, extra[0])
    split = roofline_split(trace, 3, MFMA_PEAK_TFLOPS[dtype_name])
    del model, batches, extra, trace
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return elapsed, fam, msda, split, dec_touched


run_workload.graphed = {}
run_workload.graph_check = {}


def msda_roofline(name, msda, dec_touched):
    """The MSDA HBM roofline of one workload's traced launches: the encoder kernel (the
    headline: the kernel with the most MSDA device time) with the decoder kernel and all
    launches beside it; PMC traffic from the committed per-kernel summary."""
    if not msda:
        return None
    prep = [m for m in msda if len(m) > 5]
    msda = [m for m in msda if len(m) == 5]
    enc = [m for m in msda if m[0] == m[1]]
    dec = [m for m in msda if m[0] != m[1]]

    def roof(launches, kname, pmc_name):
        t_ms = sum(m[2] for m in launches)
        t_b = sum(m[3] for m in launches)
        ach_ = t_b / (t_ms * 1e-3) / 1e9
        traffic, src = pmc_traffic(pmc_name) if pmc_name else (None, None)
        return {'bound': 'hbm', 'kernel': kname, 'achieved': ach_, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': ach_ / HBM_PEAK_GBS, 'traffic': traffic, 'traffic_source': src,
                'algorithmic_bytes_per_launch': t_b / len(launches),
                'avg_launch_ms': t_ms / len(launches), 'launches_per_step': len(launches) / 3}
    # PMC summaries are keyed '<workload>:<kernel base name>' (tools/pmc_traffic.py)
    def base(launches):
        return name + ':' + launches[0][4].split('<')[0]
    if enc:
        r = roof(enc, '%s (encoder launches, Lq = S = %d)' % (kernel_names(enc), enc[0][0]), base(enc))
        if dec:
            r['decoder_kernel'] = roof(dec, '%s (decoder launches)' % kernel_names(dec), base(dec))
            # the decoder held against the bytes it must touch (value rows its corners reach),
            # not the whole value map
            if dec_touched:
                dk = r['decoder_kernel']
                ach = dec_touched / (dk['avg_launch_ms'] * 1e-3) / 1e9
                dk.update(algorithmic_bytes_per_launch=dec_touched, achieved=ach, frac=ach / HBM_PEAK_GBS,
                          bytes_basis='value rows touched by the bilinear corners (counted from one forward) + '
                                      'offsets/logits + references + output')
        r['all_msda_launches'] = roof(msda, 'encoder + decoder launches', None)
    else:
        r = roof(msda, '%s (all launches)' % kernel_names(msda), None)
    r['encoder_launch'] = {'ms': statistics.mean(m[2] for m in enc) if enc else None,
                           'bytes': enc[0][3] if enc else None}
    r['decoder_launch'] = {'ms': statistics.mean(m[2] for m in dec) if dec else None,
                           'bytes': dec[0][3] if dec else None}
    if enc:
        # one encoder MSDA call = the projection that prepares it (records GEMM, or the head-major
        # offsets / logits GEMM) + the sampler.  The encoder's prep launches are those with
        # B*Lq = B*S rows: the decoder's run on the query rows only.
        cand = [m for m in prep if m[0] % enc[0][0] == 0]
        rows = max(m[0] for m in cand) if cand else None
        ep = [m for m in cand if m[0] == rows]
        if ep and len(ep) == len(enc):
            p_ms = statistics.mean(m[2] for m in ep)
            p_b = ep[0][3]
            c_ms = p_ms + r['avg_launch_ms']
            c_b = p_b + r['algorithmic_bytes_per_launch']
            r['encoder_call'] = {
                'ms': c_ms, 'prep_ms': p_ms, 'sampler_ms': r['avg_launch_ms'],
                'prep_kernel': ep[0][4].split('(')[0][:120],
                'bytes': c_b, 'prep_bytes': p_b, 'sampler_bytes': r['algorithmic_bytes_per_launch'],
                'achieved': c_b / (c_ms * 1e-3) / 1e9, 'unit': 'GB/s', 'peak': HBM_PEAK_GBS,
                'frac': c_b / (c_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                'basis': 'prep GEMM (input rows + weights + records or offsets/logits out) + sampler '
                         '(value + records or offsets/logits + output), HIP events, single stream'}
    return r


def _r(x, n=4):
    """x rounded to n significant digits (floats only)."""
    if isinstance(x, float):
        return float('%.*g' % (n, x)) if x == x else x
    return x


def _kname(k):
    """'msda_enc_kernel<kinet::bf16_t, 1, 2, false, true> (encoder launches, ...)' -> short form."""
    if not k:
        return k
    return k.split(' (')[0].replace('kinet::', '').replace(', ', ',')


def _roof_c(r, keys=('frac', 'achieved', 'avg_launch_ms', 'algorithmic_bytes_per_launch', 'traffic')):
    if not r:
        return None
    out = {'kernel': _kname(r.get('kernel'))}
    out.update({k: _r(r.get(k)) for k in keys if r.get(k) is not None})
    return out


def _msda_c(roof):
    """The MSDA roofline of one workload, compact: encoder sampler (+ traffic), decoder sampler
    (touched-bytes basis), and the whole encoder call (prep GEMM + sampler)."""
    if not roof:
        return None
    out = {'bound': roof.get('bound'), 'unit': roof.get('unit'), 'peak': roof.get('peak')}
    out.update(_roof_c(roof))
    out['launches_per_step'] = _r(roof.get('launches_per_step'))
    if roof.get('traffic'):
        out['traffic_x_algorithmic'] = _r(roof['traffic'] / roof['algorithmic_bytes_per_launch'], 3)
    if roof.get('decoder_kernel'):
        out['decoder_kernel'] = _roof_c(roof['decoder_kernel'])
        if roof['decoder_kernel'].get('bytes_basis'):
            out['decoder_kernel']['basis'] = 'touched value rows + offsets/logits + refs + output'
    ec = roof.get('encoder_call')
    if ec:
        out['encoder_call'] = {k: _r(ec[k]) for k in ('ms', 'prep_ms', 'sampler_ms', 'bytes', 'frac')}
    return out


def _split_c(split):
    if not split:
        return None
    return {k: {'frac': _r(v['frac'], 3), 'ms_per_step': _r(v['ms_per_step'], 3), 'unit': v['unit']}
            for k, v in split.items() if isinstance(v, dict)}


def _sub_c(c):
    """config3 / config5 sub-object, compact."""
    if not c:
        return None
    return {'workload': c['workload'].split(':')[0], 'value': _r(c['value']), 'unit': c['unit'],
            'ms_per_step': _r(c['ms_per_step']), 'frames_per_gpu_per_step': c['frames_per_gpu_per_step'],
            'in_flight_batches': c['in_flight_batches'], 'frame': c['frame'], 'dtype': c['dtype'],
            'launch': c['launch'], 'graph_check': c.get('graph_check'),
            'msda_roofline': _msda_c(c.get('roofline')),
            'gemm_conv_split': _split_c(c.get('roofline_gemm_conv_split')),
            'device_ms_per_step_by_family': {k: _r(v, 3) for k, v in c['device_ms_per_step_by_family'].items()}}


def _train_c(t):
    if not t:
        return None
    hg = t.get('host_glue') or {}
    mb = t.get('msda_bwd_roofline') or {}
    dg = t.get('dense_grad_roofline') or {}
    return {'metric': t['metric'], 'value': _r(t['value']), 'unit': t['unit'], 's_per_step': _r(t['s_per_step']),
            'steps': t['steps'], 'loss': _r(t['loss']), 'parallelism': t['config']['parallelism'],
            'host_glue_ms': _r(hg.get('ms_per_step')), 'host_only_ms': _r(hg.get('host_only_ms_per_step')),
            'msda_bwd': {'kernel': _kname(mb.get('kernel')), 'frac': _r(mb.get('frac')),
                         'avg_launch_ms': _r(mb.get('avg_launch_ms'))} if mb else None,
            'dense_grad': {'frac': _r(dg.get('frac')), 'achieved': _r(dg.get('achieved')), 'unit': dg.get('unit'),
                           'device_ms_per_step': _r(dg.get('device_ms_per_step'))} if dg else None}


def compact_line(full, detail_path):
    """The stdout line: the driver contract's keys, every roofline / sub-benchmark number DESIGN.md
    quotes, rounded to 4 significant digits, without the long provenance strings (those stay in
    the full record at `detail_path`) -- so the whole line fits the driver's stdout tail."""
    line = {k: _r(full[k]) for k in ('metric', 'value', 'unit', 'n_gpus', 'world_size', 'steps', 'warmup',
                                       'ms_per_step', 'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'data',
                                       'config')}
    line['roofline'] = _msda_c(full['roofline']) if full['roofline'].get('bound') == 'hbm' else full['roofline']
    if line['roofline'] and full['roofline'].get('traffic_source'):
        line['roofline']['traffic_pmc'] = 'rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes (profiles/pmc_traffic.json)'
    rm = full['roofline_mfma']
    pmc = (rm.get('pmc_mfma_util') or {}).get('groups') or {}
    line['roofline_mfma'] = {'bound': 'mfma', 'kernel': 'all GEMM + conv launches', 'achieved': _r(rm['achieved']),
                             'peak': rm['peak'], 'unit': rm['unit'], 'frac': _r(rm['frac']), 'traffic': None,
                             'device_ms_per_step': _r(rm['device_ms_per_step']),
                             'algorithmic_flops_per_frame': _r(rm['algorithmic_flops_per_frame']),
                             'pmc_mfma_busy': {k: _r(v['util'], 3) for k, v in pmc.items()} or None}
    line['roofline_gemm_conv_split'] = _split_c(full['roofline_gemm_conv_split'])
    line['msda_ms_per_call'] = {k: _r(v) for k, v in full['msda_ms_per_call'].items()}
    line['device_ms_per_step_by_family'] = {k: _r(v, 3) for k, v in full['device_ms_per_step_by_family'].items()}
    line['config3'] = _sub_c(full.get('config3'))
    line['config5'] = _sub_c(full.get('config5'))
    line['train'] = _train_c(full.get('train'))
    cb = full.get('cpu_baseline')
    line['cpu_baseline'] = None if not cb else {
        'value': _r(cb['value']), 'unit': cb['unit'], 'cores': cb['cores'], 'kind': cb['kind'],
        'cpu_model': cb.get('cpu_model'), 'sample': cb['sample'],
        'msda_encoder_ms_per_call': _r(cb['msda_encoder_ms_per_call']),
        'config5_msda_encoder_ms_per_call': _r(cb['config5_msda_encoder_ms_per_call'])}
    line['detail'] = detail_path
    return line


def main():
    a = parse()
    if a.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(a.gpus))
    world, rank, dev = setup_dist(a)
    if a.cpu_stub:
        return stub_main(a, world, rank, dev)
    wl = WORKLOADS[a.workload]
    from kinet_amd import _native
    if a.gemm_flags:
        _native.lib().kinet_gemm_set_flags(a.gemm_flags)
    if a.ffn_knob:
        _native.lib().kinet_ffn_set_debug(a.ffn_knob)
    from kinet_amd import kernels as K
    K.MSDA_RECORDS[0] = bool(a.msda_records)
    if a.enc_strips:
        K.msda_encoder_set_strips(a.enc_strips)
    from kinet_amd.models import backbone as BB
    BB.FUSE_BOTTLENECK_PAIRS = bool(a.bneck_pairs)
    from kinet_amd.models.deformable_transformer import DeformableTransformer
    DeformableTransformer.share_frame_pos = bool(a.share_pos)
    if a.pair_widths is not None:
        BB.FUSE_PAIR_WIDTHS = tuple(int(v) for v in a.pair_widths.split(',') if v)
    BB.STEM_FROM_IMAGE = bool(a.stem_image)
    elapsed, fam, msda, split, dec_touched = run_workload(a, a.workload, dev, world, rank, a.batch, a.streams,
                                                          a.height, a.width, a.dtype, a.steps, a.warmup)

    # config 5 (BASELINE configs[4], the HBM-stress MSDA case) beside the headline: a short
    # timed run of its own workload with its own MSDA roofline (not part of `value`)
    c5 = None
    if a.workload == 'config2' and not a.no_config5:
        w5 = WORKLOADS['config5']
        el5, fam5, msda5, split5, dt5 = run_workload(a, 'config5', dev, world, rank, w5['batch'], w5['streams'],
                                                   w5['h'], w5['w'], w5['dtype'], a.config5_steps, 2)
        c5 = {'workload': w5['desc'], 'value': w5['batch'] * a.config5_steps * world / el5, 'unit': 'frames/s',
              'launch': 'HIP graph replay' if run_workload.graphed.get('config5') else 'eager',
              'graph_check': run_workload.graph_check.get('config5'),
              'frames_per_gpu_per_step': w5['batch'], 'in_flight_batches': w5['streams'],
              'frame': [3, w5['h'], w5['w']], 'dtype': w5['dtype'], 'steps': a.config5_steps, 'warmup': 2,
              'ms_per_step': el5 / a.config5_steps * 1e3,
              'roofline': msda_roofline('config5', msda5, dt5),
              'roofline_gemm_conv_split': split5,
              'device_ms_per_step_by_family': {k: round(v['ms'], 4) for k, v in fam5.items()}}

    # config 3 (BASELINE configs[2], the tracking forward on the d=288 stack at 800x1333) the same way
    c3 = None
    if a.workload == 'config2' and not a.no_config3:
        w3 = WORKLOADS['config3']
        el3, fam3, msda3, split3, dt3 = run_workload(a, 'config3', dev, world, rank, w3['batch'], w3['streams'],
                                                   w3['h'], w3['w'], w3['dtype'], a.config3_steps, 2)
        c3 = {'workload': w3['desc'], 'value': w3['batch'] * a.config3_steps * world / el3, 'unit': 'frames/s',
              'launch': 'HIP graph replay' if run_workload.graphed.get('config3') else 'eager',
              'graph_check': run_workload.graph_check.get('config3'),
              'frames_per_gpu_per_step': w3['batch'], 'in_flight_batches': w3['streams'],
              'frame': [3, w3['h'], w3['w']], 'dtype': w3['dtype'], 'steps': a.config3_steps, 'warmup': 2,
              'ms_per_step': el3 / a.config3_steps * 1e3,
              'roofline': msda_roofline('config3', msda3, dt3),
              'roofline_gemm_conv_split': split3,
              'device_ms_per_step_by_family': {k: round(v['ms'], 4) for k, v in fam3.items()}}

    # config-4 training step (BASELINE configs[3]): every rank runs the DDP step, gradients
    # all-reduced over RCCL -- the path whose 1 -> 8 GPU scaling north_star targets
    train = None
    if not a.no_train and a.workload == 'config2':
        train = train_leg(a, dev, world)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a.cpu_seconds)

    if rank == 0:
        frames_total = a.batch * a.steps * world
        value = frames_total / elapsed
        dt_name = a.dtype
        mfma_ms = sum(fam[f]['ms'] for f in ('gemm', 'conv') if f in fam)
        mfma_flops = sum(fam[f]['flops'] for f in ('gemm', 'conv') if f in fam)
        # Headline roofline: the MSDA sampling kernel with the most device time in the
        # rocprofv3 summary (profiles/): config 2's encoder kernel (6 launches per frame
        # batch), the 6 decoder launches beside it
        msda_roof = msda_roofline(a.workload, msda, dec_touched)
        enc = [m for m in msda if m[0] == m[1]]
        dec = [m for m in msda if m[0] != m[1]]
        msda_enc_ms = statistics.mean(m[2] for m in enc) if enc else None
        msda_dec_ms = statistics.mean(m[2] for m in dec) if dec else None
        mfma_ach = mfma_flops / (mfma_ms * 1e-3) / 1e12 if mfma_ms else 0.0
        mfma_roof = {'bound': 'mfma', 'kernel': 'all GEMM + conv launches (gemm_kernel, gemm_rw_kernel)',
                     'achieved': mfma_ach, 'peak': MFMA_PEAK_TFLOPS[dt_name], 'unit': 'TFLOP/s',
                     'frac': mfma_ach / MFMA_PEAK_TFLOPS[dt_name], 'traffic': None,
                     'algorithmic_flops_per_frame': mfma_flops / a.batch,
                     'device_ms_per_step': mfma_ms,
                     'pmc_mfma_util': pmc_mfma_util() if a.workload == 'config2' else None}
        roofline = msda_roof or mfma_roof
        line = {
            'metric': 'frames/sec (3x800x1333, 300 obj+track queries) at 1/2/4/8 GPUs; MSDeformAttn ms/call',
            'value': value, 'unit': 'frames/s', 'n_gpus': world, 'world_size': world,
            'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': elapsed / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': dt_name,
            'data': 'synthetic N(0,1) 3x%dx%d frames, random-init weights (reference init)' % (a.height, a.width),
            'config': {'workload': wl['desc'],
                       'frames_per_gpu_per_step': a.batch, 'in_flight_batches': max(1, a.streams),
                       'frame': [3, a.height, a.width],
                       'launch': 'HIP graph replay per in-flight slot' if run_workload.graphed.get(a.workload)
                                 else 'eager',
                       'graph_check': run_workload.graph_check.get(a.workload),
                       'parallelism': f'replicas x{world}'},
            'roofline': roofline,
            'roofline_mfma': mfma_roof,
            'roofline_gemm_conv_split': split,
            'msda_ms_per_call': {'encoder': msda_enc_ms, 'decoder': msda_dec_ms},
            'device_ms_per_step_by_family': {k: round(v['ms'], 4) for k, v in fam.items()},
            'config3': c3,
            'config5': c5,
            'cpu_baseline': cpu,
            'train': train,
        }
        detail = a.detail or os.path.join('gpurun_out', 'bench_detail.json')
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail)), exist_ok=True)
            with open(detail, 'w') as f:
                json.dump(line, f)
        except OSError:
            detail = None
        print(json.dumps(compact_line(line, detail), separators=(',', ':')))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

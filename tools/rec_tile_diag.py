"""Round-5 diagnosis of the 32-row records tile: the records GEMM
(kinet_msda_sample_records) with 32-row tiles against the default 16-row tile on the round-4
problem (config-2 level shapes, batch 2, 8 heads), three runs per variant, so a data-dependent
logic error (same words every run) is told apart from a timing race (words vary run to run).

  flag 16384          32-row tile, 2-slot ring, 2 workgroups per CU (the round-4 variant)
  flag 16384 | 32768  the same + 32 idle wait states between the MFMAs and the epilogue
  flag 16384 | 65536  the same + vmcnt(0) lgkmcnt(0) + workgroup barrier before the epilogue
  flag 16384 | 262144 the same with only a scheduling barrier between the MFMAs and the epilogue
  flag 16384 | 524288 the level reductions through ds_bpermute instead of v_permlane16/32_swap

    python tools/rec_tile_diag.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from kinet_amd import _native  # noqa: E402
from kinet_amd import kernels as K  # noqa: E402
from test_msda_gpu import _record_problem  # noqa: E402


def run(args, kw, flags):
    old = _native.lib().kinet_gemm_set_flags(flags)
    try:
        r, fb = K.msda_sample_records(*args, **kw)
        torch.cuda.synchronize()
    finally:
        _native.lib().kinet_gemm_set_flags(old)
    return r.clone()


def main():
    shapes = ((100, 167), (50, 84), (25, 42), (13, 21))
    for seed, masked in ((43, False), (77, True)):
        x, pos, w, bias, ref, qmask, raw = _record_problem(shapes, 2, 2.0 if seed == 43 else 3.0, seed, 2, masked)
        args = (x.cuda(), w.cuda(), bias.cuda(), 8, ref.cuda(), shapes)
        kw = dict(x_add=pos.cuda(), query_attn_mask=qmask.cuda() if qmask is not None else None)
        base = run(args, kw, 0)
        again = run(args, kw, 8192)
        print(f'seed {seed} masked {masked}: records {tuple(base.shape)}; 16-row 2-WG ring vs default: '
              f'{int((again != base).sum())} words differ', flush=True)
        for name, fl in (('32-row', 16384), ('32-row+nop', 16384 | 32768), ('32-row+drain', 16384 | 65536),
                         ('32-row+schedbarrier', 16384 | 262144), ('32-row+no-permlane', 16384 | 524288)):
            prev = None
            for rep in range(3):
                r = run(args, kw, fl)
                d = (r != base)
                n = int(d.sum())
                fields = d.reshape(-1, base.shape[-1]).sum(0).tolist()
                rows = d.reshape(-1, base.shape[-1]).any(1).nonzero().flatten()
                same = None if prev is None else bool((r == prev).all())
                print(f'  {name} run {rep}: {n} words differ, fields {[(i, c) for i, c in enumerate(fields) if c]}, '
                      f'rows {len(rows)} (row-in-tile of the first: {[(int(q) % (base.shape[1] * base.shape[2])) % 32 for q in rows[:8]]}), '
                      f'identical to previous run: {same}', flush=True)
                prev = r


def timing(batch=16, iters=20):
    """Each records-GEMM variant alone at the config-2 encoder call (batch 16), HIP events,
    interleaved twice."""
    shapes = ((100, 167), (50, 84), (25, 42), (13, 21))
    x, pos, w, bias, ref, qmask, raw = _record_problem(shapes, batch, 2.0, 43, 2, False)
    args = (x.cuda(), w.cuda(), bias.cuda(), 8, ref.cuda(), shapes)
    kw = dict(x_add=pos.cuda())
    variants = (('16-row 3 WG/CU (default)', 0), ('16-row 2 WG/CU 4-slot', 8192),
                ('32-row + schedbarrier', 16384 | 262144), ('32-row + nop', 16384 | 32768))
    res = {n: [] for n, _ in variants}
    for _ in range(2):
        for n, fl in variants:
            old = _native.lib().kinet_gemm_set_flags(fl)
            try:
                K.msda_sample_records(*args, **kw)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(iters):
                    K.msda_sample_records(*args, **kw)
                e.record()
                torch.cuda.synchronize()
                res[n].append(s.elapsed_time(e) / iters * 1e3)
            finally:
                _native.lib().kinet_gemm_set_flags(old)
    for n, t in res.items():
        print(f'  {n}: {" / ".join(f"{v:.1f}" for v in t)} us per call (batch {batch})', flush=True)


if __name__ == '__main__':
    main()
    if '--time' in sys.argv:
        timing()

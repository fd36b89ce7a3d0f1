#!/usr/bin/env python
"""Per-kernel launch durations from a rocprofv3 kernel trace, split into ALL dispatches (what
`--stats` averages) and ISOLATED dispatches (no other kernel running at any moment of the
dispatch).  bench.py measures its roofline kernels with HIP events over single-stream steps, so
its launches are the isolated ones; the timed steps run several batches in flight on separate
streams, where a one-workgroup-per-CU kernel shares the chip and its dispatch interval
stretches.  This file is the cross-check between the rocprof summary and the bench line.
usage: python tools/trace_isolated.py TRACE_DIR OUT.json [BENCH_JSON] [substring ...]"""
import csv
import glob
import json
import os
import sys


def main():
    tdir, out = sys.argv[1], sys.argv[2]
    bench = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3].endswith('.json') else None
    subs = [s for s in sys.argv[(4 if bench else 3):]] or ['msda_enc_kernel', 'gemm_rw_kernel', 'msda_fused_fast_kernel']
    files = glob.glob(os.path.join(tdir, '**', '*kernel_trace.csv'), recursive=True)
    if not files:
        raise SystemExit(f'no kernel trace under {tdir}')
    ev = []
    for f in files:
        for r in csv.DictReader(open(f)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    ev.sort()
    n = len(ev)
    iso = [False] * n
    run_end = -1
    for i, (s, e, _) in enumerate(ev):
        nxt = ev[i + 1][0] if i + 1 < n else None
        iso[i] = run_end <= s and (nxt is None or nxt >= e)
        run_end = max(run_end, e)
    res = {}
    for i, (s, e, name) in enumerate(ev):
        key = next((k for k in subs if k in name), None)
        if key is None:
            continue
        d = res.setdefault(name, {'match': key, 'all': [], 'isolated': []})
        d['all'].append(e - s)
        if iso[i]:
            d['isolated'].append(e - s)
    summary = {}
    for name, d in res.items():
        a, b = d['all'], d['isolated']
        summary[name] = {'all_calls': len(a), 'all_avg_us': sum(a) / len(a) / 1e3,
                         'isolated_calls': len(b), 'isolated_avg_us': (sum(b) / len(b) / 1e3) if b else None}
    doc = {'trace_dir': tdir, 'dispatches': n, 'kernels': summary}
    if bench:
        line = json.loads(open(bench).read().strip().splitlines()[-1])
        r = line['roofline']
        doc['bench_roofline'] = {'kernel': r.get('kernel'), 'avg_launch_us': r.get('avg_launch_ms', 0) * 1e3,
                                 'achieved': r.get('achieved'), 'frac': r.get('frac')}
    json.dump(doc, open(out, 'w'), indent=1)
    for name, s in sorted(summary.items(), key=lambda kv: -kv[1]['all_calls'] * kv[1]['all_avg_us'])[:12]:
        print(f"{s['all_calls']:5d} all {s['all_avg_us']:8.1f} us | {s['isolated_calls']:4d} isolated "
              f"{(s['isolated_avg_us'] or 0):8.1f} us  {name[:90]}")


if __name__ == '__main__':
    main()

"""Reduce rocprofv3 output directories to small per-kernel summaries (run on the GPU box
right after profiling, so the bulky per-dispatch CSVs need not travel back).

usage: python tools/pmc_summary.py OUT.json DIR [DIR ...]

For every `*_counter_collection.csv` under DIR: per kernel name, the number of
dispatches and the sum of each counter.  For every `*_kernel_trace.csv`: per kernel
name, dispatch count and total/average duration.  FETCH_SIZE/WRITE_SIZE are in KiB
(rocprofv3's derived-counter unit); the gfx950 FETCH_SIZE x2 correction of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) is applied by the consumer
(bench.py), not here, so the raw values stay visible.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(path):
    with open(path, newline='') as f:
        yield from csv.DictReader(f)


def summarize(dirs):
    out = {'counters': {}, 'kernels': {}}
    cnt = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in dirs:
        for p in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            for r in _rows(p):
                name = r.get('Kernel_Name', '?')
                cnt[name][r['Counter_Name']] += float(r['Counter_Value'])
                disp[name].add((p, r.get('Dispatch_Id') or r.get('Correlation_Id')))
        for p in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
            for r in _rows(p):
                name = r.get('Kernel_Name', '?')
                k = out['kernels'].setdefault(name, {'calls': 0, 'total_ns': 0})
                k['calls'] += 1
                k['total_ns'] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    for name, c in cnt.items():
        out['counters'][name] = {'dispatches': len(disp[name]), **c}
    for k in out['kernels'].values():
        k['avg_ns'] = k['total_ns'] / max(k['calls'], 1)
    return out


def main():
    dst, dirs = sys.argv[1], sys.argv[2:]
    s = summarize(dirs)
    with open(dst, 'w') as f:
        json.dump(s, f, indent=1, sort_keys=True)
    print(f'[pmc_summary] {len(s["counters"])} kernels with counters, '
          f'{len(s["kernels"])} traced kernels -> {dst}')


if __name__ == '__main__':
    main()

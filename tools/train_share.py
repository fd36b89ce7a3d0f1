"""Split the device time of a rocprofv3 --stats csv into kinet kernels, torch (ATen) kernels and
runtime copies/fills, and list the top non-kinet kernels.

    python tools/train_share.py profiles/<tag>_train_kernel_stats.csv [out.json]
"""
import csv
import json
import sys


def family(name):
    if 'kinet::' in name or name.startswith('_ZN5kinet'):
        return 'kinet'
    if name.startswith('__amd_rocclr'):
        return 'runtime_copy_fill'
    return 'torch'


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    fam = {}
    for r in rows:
        f = family(r['Name'])
        d = fam.setdefault(f, {'ms': 0.0, 'calls': 0})
        d['ms'] += float(r['TotalDurationNs']) / 1e6
        d['calls'] += int(r['Calls'])
    for d in fam.values():
        d['share'] = d['ms'] / (tot / 1e6)
    top = sorted((r for r in rows if family(r['Name']) != 'kinet'), key=lambda r: -float(r['TotalDurationNs']))[:12]
    out = {'source': sys.argv[1], 'total_device_ms': tot / 1e6, 'families': fam,
           'top_non_kinet': [{'ms': float(r['TotalDurationNs']) / 1e6, 'calls': int(r['Calls']),
                              'name': r['Name'][:140]} for r in top]}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], 'w').write(s + '\n')


if __name__ == '__main__':
    main()

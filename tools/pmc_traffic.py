"""Per-launch HBM traffic of each kernel from two rocprofv3 PMC passes (one FETCH_SIZE, one
WRITE_SIZE -- they do not fit one pass on gfx950) summarised by tools/pmc_summary.py.

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 / dispatches: rocprofv3 reports
both in KiB; on gfx950 FETCH_SIZE counts exactly half of the bytes of wide streaming reads
(MI355X_MICROARCH.md "HBM"), WRITE_SIZE is exact for 16-byte stores.  Kernel names are
shortened to the template name (e.g. msda_fused_fast_kernel) when that is unambiguous.

usage: python tools/pmc_traffic.py FETCH.json WRITE.json OUT.json "provenance text" [WORKLOAD]

The per-kernel entries are keyed '<WORKLOAD>:<short name>' (default workload config2) and
MERGED into OUT when it exists, so one file holds the passes of several workloads
(bench.py looks its MSDA kernels up there).
"""
import os
import json
import re
import sys


def _mangled_name(name):
    """Last <len><ident> component of an Itanium nested name (_ZN...<len>name I...): rocprofv3
    leaves some kernel names mangled in its counter-collection CSVs."""
    i, last = (3, None) if name.startswith("_ZN") else (2, None)
    while i < len(name) and name[i].isdigit():
        j = i
        while j < len(name) and name[j].isdigit():
            j += 1
        n = int(name[i:j])
        last = name[j:j + n]
        i = j + n
    return last


def short(name):
    if name.startswith('_Z'):
        m = _mangled_name(name)
        if m:
            return m
    m = re.search(r'(\w+)<', name) or re.search(r'(\w+)\(', name)
    return m.group(1) if m else name


def main():
    fetch, write = (json.load(open(p))['counters'] for p in sys.argv[1:3])
    wl = sys.argv[5] if len(sys.argv) > 5 else 'config2'
    out = {'sources': {}, 'kernels': {}, 'by_full_name': {}}
    if os.path.exists(sys.argv[3]):
        old = json.load(open(sys.argv[3]))
        if 'sources' in old:
            out = old
    out['sources'][wl] = sys.argv[4] if len(sys.argv) > 4 else ''
    for k in [k for k in out['kernels'] if k.startswith(wl + ':')] + \
             [k for k in out['by_full_name'] if k.startswith(wl + ':')]:
        out['kernels'].pop(k, None)
        out['by_full_name'].pop(k, None)
    agg = {}
    for name, c in fetch.items():
        w = write.get(name, {})
        nf, nw = c.get('dispatches', 0), w.get('dispatches', 0)
        if not nf or not nw:
            continue
        f_b = 2.0 * c.get('FETCH_SIZE', 0.0) * 1024 / nf
        w_b = w.get('WRITE_SIZE', 0.0) * 1024 / nw
        out['by_full_name'][wl + ':' + name] = {'fetch_bytes_x2': f_b, 'write_bytes': w_b,
                                                'hbm_bytes_per_launch': f_b + w_b, 'dispatches': nf}
        a = agg.setdefault(short(name), [0.0, 0])
        a[0] += (f_b + w_b) * nf
        a[1] += nf
    for k, (b, n) in agg.items():
        out['kernels'][wl + ':' + k] = {'hbm_bytes_per_launch': b / n, 'dispatches': n}
    json.dump(out, open(sys.argv[3], 'w'), indent=1, sort_keys=True)
    print(f'[pmc_traffic] {len(agg)} kernels of {wl} -> {sys.argv[3]}')


if __name__ == '__main__':
    main()

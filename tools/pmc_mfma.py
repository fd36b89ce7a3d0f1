"""MFMA-pipe utilisation per kernel from a rocprofv3 counter pass:

    rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE ... -- python bench.py ...
    python tools/pmc_summary.py S.json DIR          # per-kernel counter sums + traced durations
    python tools/pmc_mfma.py OUT.json S.json [provenance]

SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core busy cycles summed over the chip's SIMDs (one
v_mfma_f32_16x16x32_bf16 = 16 cycles, a 32x32x16 = 32: MI355X_MICROARCH.md cycle constants);
GRBM_GUI_ACTIVE is the GPU-active cycle count summed over the 8 XCDs.  Per kernel:
  util  = MFMA busy cycles / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)   -- the fraction of the matrix
          cores' cycles the kernel kept busy while it ran (the "rocprof-reported MFMA
          utilisation" of north_star; the dense bf16 peak is util = 1);
  clock = GRBM_GUI_ACTIVE / 8 / duration                          -- the clock it ran at.
Dispatches of one kernel name are summed (the ratio is a time-weighted mean).
"""
import json
import sys

SIMDS = 1024   # 256 CUs x 4 SIMDs (MI355X)


def main():
    dst, src = sys.argv[1], sys.argv[2]
    prov = sys.argv[3] if len(sys.argv) > 3 else ''
    s = json.load(open(src))
    out = {'source': prov, 'method': __doc__.strip().splitlines()[0], 'kernels': {}}
    for name, c in s.get('counters', {}).items():
        busy, gui = c.get('SQ_VALU_MFMA_BUSY_CYCLES'), c.get('GRBM_GUI_ACTIVE')
        if not busy or not gui:
            continue
        tr = s.get('kernels', {}).get(name, {})
        ent = {'dispatches': c.get('dispatches'), 'mfma_busy_cycles': busy, 'gui_active_cycles': gui,
               'util': busy / (gui / 8.0 * SIMDS)}
        if tr.get('total_ns'):
            ent['clock_ghz'] = gui / 8.0 / tr['total_ns']
            ent['avg_ns'] = tr['avg_ns']
        out['kernels'][name] = ent
    # groups: every kernel that issued MFMAs; the fused FFN; the direct / pair conv kernels
    groups = {'all_mfma_kernels': lambda n: True, 'ffn_fused': lambda n: 'ffn_fused' in n,
              'direct_conv_and_pairs': lambda n: 'conv3x3' in n or 'bneck' in n or 'stem' in n}
    out['groups'] = {}
    for g, sel in groups.items():
        ks = [e for n, e in out['kernels'].items() if sel(n)]
        if ks:
            b = sum(e['mfma_busy_cycles'] for e in ks)
            a = sum(e['gui_active_cycles'] for e in ks)
            out['groups'][g] = {'kernels': len(ks), 'util': b / (a / 8.0 * SIMDS)}
    with open(dst, 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)
    top = sorted(out['kernels'].items(), key=lambda kv: -kv[1]['mfma_busy_cycles'])[:12]
    for name, e in top:
        print(f"{e['util']:.3f}  {e.get('clock_ghz', 0):.2f} GHz  {name[:110]}")


if __name__ == '__main__':
    main()

"""Condensed outline of one kernel in a hipcc --save-temps .s file: labels, waits,
barriers, global/buffer memory ops and branches; runs of MFMA / ds_read / ds_write
collapsed to counts.  usage: python tools/asm_outline.py FILE.s SYMBOL_SUBSTRING [max_lines]"""
import sys


def outline(path, sub, limit=200):
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if sub in l and l.split(':')[0].endswith(sub.split()[-1]) or
                 (sub in l and l.endswith(sub) is False and l.startswith('_Z') and ':' in l and sub in l.split(':')[0]))
    out, run, cnt = [], None, 0

    def flush():
        nonlocal run, cnt
        if run:
            out.append(f'   [{cnt} x {run}]')
        run, cnt = None, 0
    for l in lines[start + 1:]:
        t = l.strip()
        if t.startswith('.Lfunc_end'):
            break
        if not t or t.startswith(';') or (t.startswith('.') and not t.startswith('.LBB')):
            continue
        op = t.split()[0]
        key = 'mfma' if op.startswith('v_mfma') else 'ds_read' if op.startswith('ds_read') else \
            'ds_write' if op.startswith('ds_write') else None
        if key:
            if run == key:
                cnt += 1
            else:
                flush()
                run, cnt = key, 1
            continue
        if op.startswith(('s_waitcnt', 's_barrier', 'buffer_', 's_cbranch', 's_branch', 'global_')) or t.startswith('.LBB'):
            flush()
            out.append(t[:90])
    flush()
    return out[:limit]


if __name__ == '__main__':
    print('\n'.join(outline(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 200)))

"""Scan gfx950 device assembly for MFMA hazards that are not covered by enough wait states.

The rules are the compiler's own (tools/mfma_hazard_rules.py reads them from LLVM's gfx950
hazard recognizer with llc): an XDL MFMA's destination D is written back NumPasses + 4 wait
states after issue (8 for the 16x16x32 forms, 10 for 16x16x4f32, 12 for 32x32x16) and its SrcC
is read late, so the hardware does not interlock
  * RAW -- a later read of D (VALU, LDS / buffer store data, v_permlane, another MFMA's A/B;
    another MFMA's C with a partial overlap: 6 / 8),
  * WAW -- a later non-MFMA write of D (VALU, an LDS or buffer load's destination),
  * WAR -- a later non-MFMA write of a SrcC register that is not D (3 / 0 / 7),
  * and, MFMA-independent: a VALU write read by an MFMA's A/B or by v_permlane16/32_swap
    (2 wait states; gfx950's swaps WRITE both operands too).
Each instruction is one wait state (`s_nop N` = N + 1).  The scan follows the kernel's control
flow: a pending window enters a label from every predecessor (fall-through and every branch to
it) with the largest remaining count, and loops are iterated to a fixpoint, so a window that
crosses a branch or a loop back edge is checked on the shortest executed path.

`--ab N` also lists (as information, not counted) non-MFMA writes to an in-flight MFMA's A/B
registers within N wait states of its issue -- a WAR class LLVM does not model (it requires 0).

    python tools/mfma_hazard_check.py file.s [...]        # hipcc --cuda-device-only -S output
    python tools/mfma_hazard_check.py --build              # every kinet_amd/csrc/*.hip, library flags
    python tools/mfma_hazard_check.py --build --filter gemm_rw_kernel --ab 8
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

# wait states per MFMA form (tools/mfma_hazard_rules.py on ROCm 7.2 llc, gfx950):
# (D -> read/write, SrcC -> write, D -> partial-overlap C of the next MFMA)
RULES = {
    '16x16x32': (8, 3, 6), '16x16x16': (8, 3, 6), '16x16x4f32': (10, 0, 8), '32x32x16': (12, 7, 10),
}
VALU_TO_MFMA_AB = 2
VALU_TO_PERMLANE = 2
REG = re.compile(r'\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)')
BRANCH = re.compile(r'^s_(c?branch\w*)\s+(\S+)')


def regs(text):
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(4) is not None:
            out.add((k, int(m.group(4))))
        else:
            out.update((k, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def rule_of(op):
    o = op.replace('_', '')
    for shape, r in RULES.items():
        if shape in o:
            return r
    return max(RULES.values())


def split_ops(ins):
    op = ins.split()[0]
    rest = ins[len(op):].strip()
    parts, depth, cur = [], 0, ''
    for ch in rest:
        if ch == '[':
            depth += 1
        elif ch == ']':
            depth -= 1
        if ch == ',' and depth == 0:
            parts.append(cur.strip())
            cur = ''
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return op, parts


def classify(ins):
    """(kind, reads, writes) of one instruction; kind in mfma / valu / permlane / lds / vmem / s."""
    op, parts = split_ops(ins)
    if op.startswith('s_'):
        return 's', set(), set()
    if op.startswith('v_mfma') or op.startswith('v_smfmac'):
        d = regs(parts[0]) if parts else set()
        a = regs(parts[1]) if len(parts) > 1 else set()
        b = regs(parts[2]) if len(parts) > 2 else set()
        c = regs(parts[3]) if len(parts) > 3 else set()
        return 'mfma', (a, b, c), d
    if op.startswith('v_permlane16_swap') or op.startswith('v_permlane32_swap'):
        r = regs(','.join(parts[:2]))
        return 'permlane', r, r
    if op.startswith('v_'):
        if op.startswith(('v_cmp', 'v_readlane', 'v_readfirstlane')):
            return 'valu', regs(','.join(parts)), set()
        w = regs(parts[0]) if parts else set()
        r = regs(','.join(parts[1:]))
        if op.startswith(('v_fmac', 'v_mac', 'v_dot2c', 'v_writelane', 'v_pk_fmac')):
            r |= w
        return 'valu', r, w
    if op.startswith('ds_'):
        if op.startswith(('ds_read', 'ds_load', 'ds_bpermute', 'ds_permute', 'ds_swizzle')) or '_rtn' in op:
            return 'lds', regs(','.join(parts[1:])), regs(parts[0]) if parts else set()
        return 'lds', regs(','.join(parts)), set()
    if op.startswith(('buffer_', 'global_', 'flat_', 'scratch_')):
        if ' lds' in ins or '_lds_' in op:
            return 'vmem', regs(','.join(parts)), set()
        if '_load' in op or ('_atomic' in op and ' sc0' in ins):
            return 'vmem', regs(','.join(parts[1:])), regs(parts[0]) if parts else set()
        return 'vmem', regs(','.join(parts)), set()
    return 'valu', regs(','.join(parts[1:])), regs(parts[0]) if parts else set()


class Pending:
    """A window still open at a point: (kind, regs, remaining wait states, producer text)."""
    __slots__ = ('kind', 'regs', 'rem', 'src', 'cpart')

    def __init__(self, kind, regs_, rem, src, cpart=0):
        self.kind, self.regs, self.rem, self.src, self.cpart = kind, frozenset(regs_), rem, src, cpart

    def key(self):
        return (self.kind, self.regs, self.src)


def step(state, ins, idx, name, report, ab_info, seen, record):
    """Check instruction `ins` against the open windows, then open its own and age them all."""
    kind, reads, writes = classify(ins)
    op = ins.split()[0]
    ws = int(ins.split()[1], 0) + 1 if op == 's_nop' else 1

    def bad(p, what, regs_hit, need):
        tag = (idx, p.src, what)
        if record and tag not in seen:
            seen.add(tag)
            report.append(f'{name}: [{idx}] {ins}  {what} {sorted(regs_hit)[:2]} of [{p.src[0]}] {p.src[1]}'
                          f' -- {need} wait state(s) missing')

    for p in state.values():
        if p.rem <= 0:
            continue
        if p.kind == 'D':
            if kind == 'mfma':
                a, b, c = reads
                if p.regs & (a | b):
                    bad(p, 'MFMA A/B reads D', p.regs & (a | b), p.rem)
                if p.regs & c and c != p.regs:
                    need = p.rem - (rule_of(p.src[1])[0] - p.cpart)
                    if need > 0:
                        bad(p, 'MFMA C overlaps D partly', p.regs & c, need)
                # the same D taken whole as C by an MFMA (accumulate chain): no wait
            else:
                if p.regs & reads:
                    bad(p, 'reads D', p.regs & reads, p.rem)
                if p.regs & writes:
                    bad(p, 'writes D', p.regs & writes, p.rem)
        elif p.kind == 'C':
            if kind != 'mfma' and p.regs & writes:
                bad(p, 'writes SrcC', p.regs & writes, p.rem)
        elif p.kind == 'W':
            if kind == 'mfma' and p.regs & (reads[0] | reads[1]):
                bad(p, 'MFMA A/B reads a fresh VALU result', p.regs & (reads[0] | reads[1]), p.rem)
            if kind == 'permlane' and p.regs & reads:
                bad(p, 'v_permlane reads a fresh VALU result', p.regs & reads, p.rem)
        elif p.kind == 'AB' and ab_info is not None and kind != 'mfma' and p.regs & writes:
            tag = (idx, p.src, 'ab')
            if record and tag not in seen:
                seen.add(tag)
                ab_info.append(f'{name}: [{idx}] {ins}  writes A/B {sorted(p.regs & writes)[:2]} of in-flight '
                               f'[{p.src[0]}] {p.src[1]} ({p.rem} wait states after issue)')

    new = {}
    for k, p in state.items():
        rg = p.regs
        if kind == 'mfma' and p.kind in ('D', 'C', 'AB'):
            # MFMAs retire in order: a later MFMA's write of a register supersedes an earlier
            # MFMA's pending result there (and lands after the earlier one's SrcC read)
            rg = rg - writes
        r = p.rem - ws
        if r > 0 and rg:
            q = Pending(p.kind, rg, r, p.src, p.cpart)
            new[q.key()] = q
    if kind == 'mfma':
        a, b, c = reads
        d_rule, c_rule, part_rule = rule_of(op)
        src = (idx, ins)
        q = Pending('D', writes, d_rule, src, cpart=d_rule - part_rule)
        new[q.key()] = q
        cc = c - writes
        if cc and c_rule:
            q = Pending('C', cc, c_rule, src)
            new[q.key()] = q
        if ab_info is not None:
            q = Pending('AB', a | b, ab_info_ws[0], src)
            new[q.key()] = q
    elif kind in ('valu', 'permlane') and writes:
        q = Pending('W', writes, VALU_TO_PERMLANE, (idx, ins))
        new[q.key()] = q
    return new


ab_info_ws = [0]


def blocks_of(lines):
    """Split a kernel's lines (labels end with ':') into basic blocks: [(label, [(idx, ins)])]."""
    blocks, cur, lab = [], [], None
    for idx, t in lines:
        if t.endswith(':'):
            if cur or lab is not None:
                blocks.append((lab, cur))
            lab, cur = t[:-1], []
            continue
        cur.append((idx, t))
        op = t.split()[0]
        if op.startswith('s_branch') or op.startswith('s_cbranch') or op in ('s_endpgm', 's_setpc_b64'):
            blocks.append((lab, cur))
            lab, cur = None, []
    if cur or lab is not None:
        blocks.append((lab, cur))
    return blocks


def scan(lines, name, report, ab_info=None):
    """lines: [(index, text)] of one kernel incl. labels.  Returns the number of violations."""
    blocks = blocks_of(lines)
    index = {lab: i for i, (lab, _) in enumerate(blocks) if lab is not None}
    succ = []
    for i, (_, ins) in enumerate(blocks):
        s = []
        last = ins[-1][1] if ins else ''
        m = BRANCH.match(last)
        op = last.split()[0] if last else ''
        if m and m.group(2) in index:
            s.append(index[m.group(2)])
        if not (op.startswith('s_branch') or op in ('s_endpgm', 's_setpc_b64')) and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    entry = [dict() for _ in blocks]
    n0 = len(report)
    seen = set()
    for it in range(64):
        changed = False
        for i, (_, ins) in enumerate(blocks):
            st = dict(entry[i])
            for idx, t in ins:
                st = step(st, t, idx, name, report, ab_info, seen, record=True)
            for j in succ[i]:
                e = entry[j]
                for k, p in st.items():
                    if k not in e or e[k].rem < p.rem:
                        e[k] = p
                        changed = True
        if not changed:
            break
    return len(report) - n0


def kernels_from_s(path):
    cur, name, idx = None, None, 0
    for ln in open(path):
        s = ln.rstrip('\n')
        m = re.match(r'^(_Z\S+|[A-Za-z_]\w*):', s)
        if m and not s.startswith('.') and not s.startswith('.L'):
            if cur is not None and name:
                yield name, cur
            name, cur, idx = m.group(1), [], 0
            continue
        t = s.split(';')[0].strip()
        if cur is None or not t:
            continue
        if t.startswith('.Lfunc_end'):
            yield name, cur
            cur, name = None, None
            continue
        if re.match(r'^\.L\w+:$', t):
            cur.append((idx, t))
            continue
        if t.startswith('.') or t.endswith(':'):
            continue
        cur.append((idx, t))
        idx += 1
    if cur is not None and name:
        yield name, cur


def build_s(out_dir, flags=(), jobs=8):
    """hipcc --cuda-device-only -S of every kinet_amd/csrc/*.hip with the library's flags."""
    import concurrent.futures as cf
    sys.path.insert(0, ROOT)
    from kinet_amd import build as kb

    def one(src):
        dst = os.path.join(out_dir, os.path.basename(src) + '.s')
        cmd = [kb.HIPCC] + kb.FLAGS + list(flags) + ['-DKINET_SRC_HASH="0"', '--cuda-device-only', '-S', src,
                                                   '-o', dst]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr[-3000:])
        return dst
    with cf.ThreadPoolExecutor(jobs) as ex:
        return list(ex.map(one, sorted(kb._sources())))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('files', nargs='*')
    ap.add_argument('--build', action='store_true', help='compile kinet_amd/csrc/*.hip to .s and scan them')
    ap.add_argument('--keep', default=None, help='with --build: directory for the .s files')
    ap.add_argument('--filter', default='')
    ap.add_argument('--max', type=int, default=40)
    ap.add_argument('--ab', type=int, default=0, help='also list writes to in-flight A/B within N wait states')
    a = ap.parse_args()
    files = list(a.files)
    tmp = None
    if a.build:
        out = a.keep or tempfile.mkdtemp(prefix='kinet_s_')
        os.makedirs(out, exist_ok=True)
        files += build_s(out)
        tmp = out
    ab_info_ws[0] = a.ab
    report, info, total, nk = [], [] if a.ab else None, 0, 0
    for f in files:
        for name, lines in kernels_from_s(f):
            if a.filter and a.filter not in name:
                continue
            if not any(t.startswith('v_mfma') for _, t in lines):
                continue
            nk += 1
            total += scan(lines, name, report, info)
    for r in report[:a.max]:
        print(r)
    if info:
        print(f'-- {len(info)} write(s) to in-flight MFMA A/B registers within {a.ab} wait states (LLVM requires 0):')
        for r in info[:a.max]:
            print('  ' + r)
    print(f'{nk} MFMA kernels scanned, {total} hazard(s) short of the compiler\'s wait states'
          + (f' (.s in {tmp})' if tmp else ''))
    return 1 if total else 0


if __name__ == '__main__':
    sys.exit(main())

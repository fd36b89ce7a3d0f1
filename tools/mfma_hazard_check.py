"""Scan gfx950 device assembly for MFMA-result reads that come too early.

An XDL MFMA's destination registers are written `passes` cycles after issue, and the hardware does
not interlock a later non-MFMA read of them: the compiler must put enough independent instructions
(or s_nop) in between -- on gfx950 NumPasses + 4 wait states for an 8- or 16-pass XDL op (12 for
v_mfma_f32_16x16x32_{bf16,f16}, 20 for the 32x32x16 forms; MI355X guides, cdna_hip_programming.md
section 5.7).  This tool walks every kernel's instruction stream linearly (each instruction = 1
wait state, `s_nop N` = N + 1; a branch target or `s_cbranch` ends the window conservatively only
for the instructions that follow in program order) and reports every non-MFMA instruction that
reads an MFMA destination register within the window.  A report is a candidate hazard to inspect,
not proof: control flow can make the linear distance shorter or longer than the executed one.

    python tools/mfma_hazard_check.py file.s [...]          # hipcc --cuda-device-only -S output
    python tools/mfma_hazard_check.py --so kinet_amd/_lib/libkinet_amd.so
"""
import argparse
import re
import subprocess
import sys

PASSES = {  # gfx950 XDL pass counts of the forms this repo emits
    '16x16x32': 4, '16x16x16': 4, '16x16x8': 8, '16x16x4': 8, '32x32x16': 8, '32x32x8': 16, '32x32x4': 16,
    '4x4x4': 2,
}
REG = re.compile(r'\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)')


def regs(text):
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(4) is not None:
            out.add((k, int(m.group(4))))
        else:
            out.update((k, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def passes_of(op):
    for shape, n in PASSES.items():
        if shape in op:
            return n
    return 16


def scan(lines, name, report):
    """lines: instruction strings of one kernel in program order."""
    pend = []   # (dst regs, remaining wait states, index, text)
    n_bad = 0
    for i, ins in enumerate(lines):
        op = ins.split()[0]
        ops = ins[len(op):]
        if op.startswith('s_nop'):
            ws = int(ins.split()[1], 0) + 1
        else:
            ws = 1
        if op.startswith('v_mfma'):
            parts = [p.strip() for p in ops.split(',')]
            dst = regs(parts[0])
            srcs = regs(','.join(parts[1:3]))    # A / B operands: reading a pending dst there is a hazard too
            srcc = regs(parts[3]) if len(parts) > 3 else set()
            for d, rem, j, t in pend:
                if d & srcs:
                    n_bad += 1
                    report.append(f'{name}: [{i}] {ins.strip()}  reads A/B {sorted(d & srcs)[:2]} of [{j}] {t.strip()}'
                                  f' with {rem} wait states missing')
                # srcC == dst of an identical-shape MFMA is the supported back-to-back chain
            pend = [(d - dst, rem, j, t) for d, rem, j, t in pend]
            pend.append((dst, passes_of(op) + 4, i, ins))
        elif not op.startswith('s_') or op.startswith('s_waitcnt'):
            rd = regs(ops)
            for d, rem, j, t in pend:
                hit = d & rd
                if hit:
                    n_bad += 1
                    report.append(f'{name}: [{i}] {ins.strip()}  reads {sorted(hit)[:2]} of [{j}] {t.strip()}'
                                  f' with {rem} wait states missing')
        pend = [(d, rem - ws, j, t) for d, rem, j, t in pend if rem - ws > 0 and d]
        if op in ('s_endpgm',):
            pend = []
    return n_bad


def kernels_from_s(path):
    cur, name = None, None
    for ln in open(path):
        s = ln.rstrip('\n')
        m = re.match(r'^(_Z\S+|[A-Za-z_]\w*):', s)
        if m and not s.startswith('.'):
            if cur is not None and name:
                yield name, cur
            name, cur = m.group(1), []
            continue
        t = s.split(';')[0].strip()
        if cur is not None and t and not t.startswith('.') and not t.endswith(':'):
            cur.append(t)
    if cur is not None and name:
        yield name, cur


def kernels_from_so(path):
    dis = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', '--no-show-raw-insn', path],
                         capture_output=True, text=True, check=True).stdout
    cur, name = None, None
    for ln in dis.splitlines():
        m = re.match(r'^[0-9a-f]+ <(.+)>:', ln)
        if m:
            if cur:
                yield name, cur
            name, cur = m.group(1), []
            continue
        t = ln.split('//')[0].strip()
        if cur is not None and t:
            cur.append(t)
    if cur:
        yield name, cur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('files', nargs='*')
    ap.add_argument('--so', action='append', default=[])
    ap.add_argument('--filter', default='')
    ap.add_argument('--max', type=int, default=40)
    a = ap.parse_args()
    report, total, nk = [], 0, 0
    srcs = [(f, kernels_from_s) for f in a.files] + [(f, kernels_from_so) for f in a.so]
    for f, fn in srcs:
        for name, lines in fn(f):
            if a.filter and a.filter not in name:
                continue
            if not any(x.startswith('v_mfma') for x in lines):
                continue
            nk += 1
            total += scan(lines, name, report)
    for r in report[:a.max]:
        print(r)
    print(f'{nk} MFMA kernels scanned, {total} candidate early reads')
    return 1 if total else 0


if __name__ == '__main__':
    sys.exit(main())

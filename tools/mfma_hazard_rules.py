"""Wait-state rules of the gfx950 MFMA hazards, read from the compiler's own hazard recognizer.

Each case is a two-instruction machine function (producer, consumer) fed to
`llc -mcpu=gfx950 -run-pass=post-RA-hazard-rec`; the `S_NOP` the pass inserts between them is
the number of wait states LLVM's GCNHazardRecognizer requires for that pair.  The table this
prints is what tools/mfma_hazard_check.py enforces on the library's assembly, so the scanner
checks the code against the same rules the compiler pads by (and reports where hand-placed
code or a scheduling decision leaves a pair short).

    python tools/mfma_hazard_rules.py            # prints the table (JSON with --json)
    python tools/mfma_hazard_rules.py --cfg-repro  # the recognizer's gap across a CFG merge

Producer / consumer classes (registers: D = MFMA destination, A/B/C = MFMA sources):
  raw_valu      D -> VALU read                 waw_valu   D -> VALU write
  war_c_valu    C (not D) -> VALU write        war_ab_valu A -> VALU write
  raw_mfma_ab   D -> next MFMA A operand       raw_mfma_c_part D -> next MFMA C, partial overlap
  raw_ds_data   D -> ds_write data             raw_vmem_data D -> buffer_store data
  raw_permlane  D -> v_permlane16_swap operand
  waw_ds        D -> ds_read destination       war_c_ds   C (not D) -> ds_read destination
  waw_vmem      D -> buffer_load destination   war_c_vmem C (not D) -> buffer_load destination
  valu_mfma_ab  VALU write -> MFMA A read      valu_permlane VALU write -> v_permlane16_swap read
"""
import argparse
import json
import os
import re
import subprocess
import tempfile

LLC = '/opt/rocm/lib/llvm/bin/llc'

# MIR opcodes of the MFMA forms the library emits, with their operand widths (A/B regs, D/C regs)
MFMA = {
    '16x16x32_bf16': ('V_MFMA_F32_16X16X32_BF16_vgprcd_e64', 4, 4),
    '16x16x32_f16': ('V_MFMA_F32_16X16X32_F16_vgprcd_e64', 4, 4),
    '16x16x16bf16_1k': ('V_MFMA_F32_16X16X16BF16_1K_vgprcd_e64', 2, 4),
    '16x16x4f32': ('V_MFMA_F32_16X16X4F32_vgprcd_e64', 1, 4),
    '32x32x16_bf16': ('V_MFMA_F32_32X32X16_BF16_vgprcd_e64', 4, 16),
}


def vr(base, n):
    return '$vgpr%d' % base if n == 1 else '$' + '_'.join('vgpr%d' % (base + i) for i in range(n))


def mfma(op, d, a, b, c):
    name, nab, ndc = MFMA[op]
    return f'{vr(d, ndc)} = {name} {vr(a, nab)}, {vr(b, nab)}, {vr(c, ndc)}, 0, 0, 0, implicit $mode, implicit $exec'


def cases():
    """(class, op, producer, consumer): D = v[0..], A = v[40..], B = v[48..], C (separate) = v[64..]."""
    out = []
    for op, (_, nab, ndc) in MFMA.items():
        p_same = mfma(op, 0, 40, 48, 0)      # D == C: the accumulate form
        p_sepc = mfma(op, 0, 40, 48, 64)     # C in other registers
        out += [
            ('raw_valu', op, p_same, '$vgpr100 = V_ADD_F32_e32 $vgpr1, $vgpr101, implicit $mode, implicit $exec'),
            ('waw_valu', op, p_same, '$vgpr1 = V_MOV_B32_e32 0, implicit $exec'),
            ('war_c_valu', op, p_sepc, '$vgpr65 = V_MOV_B32_e32 0, implicit $exec'),
            ('war_ab_valu', op, p_sepc, '$vgpr40 = V_MOV_B32_e32 0, implicit $exec'),
            ('raw_mfma_ab', op, p_same, mfma(op, 120, 0, 48, 120)),
            ('raw_ds_data', op, p_same,
             'DS_WRITE_B128_gfx9 $vgpr100, $vgpr0_vgpr1_vgpr2_vgpr3, 0, 0, implicit $exec'),
            ('raw_vmem_data', op, p_same,
             'BUFFER_STORE_DWORD_OFFEN $vgpr1, $vgpr100, $sgpr0_sgpr1_sgpr2_sgpr3, 0, 0, 0, 0, implicit $exec'),
            ('raw_permlane', op, p_same, '$vgpr1, $vgpr100 = V_PERMLANE16_SWAP_B32_e32 $vgpr1, $vgpr100, implicit $exec'),
            ('waw_ds', op, p_same, '$vgpr0_vgpr1_vgpr2_vgpr3 = DS_READ_B128_gfx9 $vgpr100, 0, 0, implicit $exec'),
            ('war_c_ds', op, p_sepc, '$vgpr64_vgpr65_vgpr66_vgpr67 = DS_READ_B128_gfx9 $vgpr100, 0, 0, implicit $exec'),
            ('waw_vmem', op, p_same,
             '$vgpr1 = BUFFER_LOAD_DWORD_OFFEN $vgpr100, $sgpr0_sgpr1_sgpr2_sgpr3, 0, 0, 0, 0, implicit $exec'),
            ('war_c_vmem', op, p_sepc,
             '$vgpr65 = BUFFER_LOAD_DWORD_OFFEN $vgpr100, $sgpr0_sgpr1_sgpr2_sgpr3, 0, 0, 0, 0, implicit $exec'),
            ('valu_mfma_ab', op, '$vgpr40 = V_MOV_B32_e32 0, implicit $exec', p_sepc),
        ]
        if ndc == 4:
            out.append(('raw_mfma_c_part', op, p_same, mfma(op, 2, 40, 48, 2).replace(vr(2, 4), '$vgpr2_vgpr3_vgpr4_vgpr5')))
    out.append(('valu_permlane', '-', '$vgpr1 = V_MOV_B32_e32 0, implicit $exec',
                '$vgpr1, $vgpr100 = V_PERMLANE16_SWAP_B32_e32 $vgpr1, $vgpr100, implicit $exec'))
    return out


def mir(cs):
    fns = []
    for i, (_, _, p, c) in enumerate(cs):
        fns.append(f"""---
name: f{i}
tracksRegLiveness: false
machineFunctionInfo:
  isEntryFunction: true
body: |
  bb.0:
    {p}
    {c}
    S_ENDPGM 0
...
""")
    return ''.join(fns)


def probe():
    cs = cases()
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, 'h.mir')
        with open(src, 'w') as f:
            f.write(mir(cs))
        r = subprocess.run([LLC, '-mtriple=amdgcn-amd-amdhsa', '-mcpu=gfx950', '-run-pass=post-RA-hazard-rec', src,
                            '-o', '-'], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr[-4000:])
    bodies = re.split(r'^name:\s+', r.stdout, flags=re.M)[1:]
    table = {}
    for body, (cls, op, _, _) in zip(bodies, cs):
        ins = [ln.strip() for ln in body.split('body:', 1)[1].splitlines() if ln.strip()
               and not ln.strip().startswith(('bb.', '...', '|'))]
        ws = 0
        for ln in ins[1:]:
            m = re.match(r'S_NOP (\d+)', ln)
            if m:
                ws += int(m.group(1)) + 1
            else:
                break
        table.setdefault(cls, {})[op] = ws
    return table


CFG_REPRO = """---
name: merge
tracksRegLiveness: false
machineFunctionInfo:
  isEntryFunction: true
body: |
  bb.0:
    successors: %bb.1, %bb.2
    $vgpr0_vgpr1_vgpr2_vgpr3 = V_MFMA_F32_16X16X32_F16_vgprcd_e64 $vgpr40_vgpr41_vgpr42_vgpr43, $vgpr48_vgpr49_vgpr50_vgpr51, $vgpr64_vgpr65_vgpr66_vgpr67, 0, 0, 0, implicit $mode, implicit $exec
    S_CBRANCH_VCCZ %bb.2, implicit $vcc
  bb.1:
    successors: %bb.3
    $vgpr126 = V_MOV_B32_e32 $vgpr125, implicit $exec
    $vgpr127 = V_MOV_B32_e32 $vgpr125, implicit $exec
    $vgpr128 = V_MOV_B32_e32 $vgpr125, implicit $exec
    $vgpr129 = V_MOV_B32_e32 $vgpr125, implicit $exec
    $vgpr130 = V_MOV_B32_e32 $vgpr125, implicit $exec
    S_BRANCH %bb.3
  bb.2:
    successors: %bb.3
    $vgpr120 = V_RCP_IFLAG_F32_e32 $vgpr121, implicit $mode, implicit $exec
  bb.3:
    S_WAITCNT 0
    $vgpr100 = V_ADD_F32_e32 $vgpr0, $vgpr101, implicit $mode, implicit $exec
    S_ENDPGM 0
...
"""


def cfg_repro():
    """An MFMA, a branch, and its result read after the merge: 8 wait states via bb.1 (5 moves +
    branch + wait), 3 via bb.2 (1 instruction).  The recognizer pads 8 - (the distance along the
    first predecessor it searches) and never re-searches bb.0 through bb.2."""
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, 'r.mir')
        with open(src, 'w') as f:
            f.write(CFG_REPRO)
        r = subprocess.run([LLC, '-mtriple=amdgcn-amd-amdhsa', '-mcpu=gfx950', '-run-pass=post-RA-hazard-rec', src,
                            '-o', '-'], capture_output=True, text=True)
    body = r.stdout.split('body:', 1)[1]
    nops = re.findall(r'S_NOP (\d+)', body)
    print(body.strip())
    print('s_nop inserted:', nops or 'none', '-- the path through bb.2 has 3 wait states, 8 are required')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--json', action='store_true')
    ap.add_argument('--cfg-repro', action='store_true')
    a = ap.parse_args()
    if a.cfg_repro:
        cfg_repro()
        return
    t = probe()
    if a.json:
        print(json.dumps(t, indent=1, sort_keys=True))
        return
    ops = list(MFMA)
    print('%-16s' % 'class' + ''.join('%17s' % o for o in ops))
    for cls, row in t.items():
        print('%-16s' % cls + ''.join('%17s' % row.get(o, row.get('-', '')) for o in ops))


if __name__ == '__main__':
    main()

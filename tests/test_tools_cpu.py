"""CPU tests of the assembly checkers under tools/: the MFMA hazard scanner
(tools/mfma_hazard_check.py) and the LDS-DMA drain check (tools/dma_drain_check.py), on small
hand-written gfx950 listings whose answer is known; and, where llc is present, the wait-state
rules read from LLVM's hazard recognizer (tools/mfma_hazard_rules.py)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import dma_drain_check as ddc  # noqa: E402
import mfma_hazard_check as mhc  # noqa: E402

MFMA = 'v_mfma_f32_16x16x32_bf16 v[0:3], v[40:43], v[48:51], v[0:3]'


def _scan(text):
    lines = [(i, t.strip()) for i, t in enumerate(text.strip().splitlines()) if t.strip()]
    report = []
    return mhc.scan(lines, 'k', report), report


def test_hazard_raw_read_too_early():
    n, _ = _scan(f"""
        {MFMA}
        v_add_f32_e32 v100, v1, v101
        s_endpgm""")
    assert n == 1


def test_hazard_padded_read_is_clean():
    n, _ = _scan(f"""
        {MFMA}
        s_nop 7
        v_add_f32_e32 v100, v1, v101
        s_endpgm""")
    assert n == 0


def test_hazard_short_path_across_a_merge():
    # 8 wait states on the long path, 2 on the short one: LLVM's recognizer pads neither
    # (tools/mfma_hazard_rules.py --cfg-repro); the scanner takes the shortest executed path
    n, _ = _scan(f"""
        {MFMA}
        s_cbranch_vccz .LBB0_2
        v_mov_b32_e32 v126, v125
        v_mov_b32_e32 v127, v125
        v_mov_b32_e32 v128, v125
        v_mov_b32_e32 v129, v125
        v_mov_b32_e32 v130, v125
        s_branch .LBB0_3
        .LBB0_2:
        v_rcp_f32_e32 v120, v121
        .LBB0_3:
        v_add_f32_e32 v100, v0, v101
        s_endpgm""")
    assert n == 1


def _drains(body):
    return ddc.drains([ln for ln in body.strip('\n').splitlines()])


LOOP = """
.LBB0_1:                                ; =>This Inner Loop Header: Depth=1
	;;#ASMSTART
	s_waitcnt vmcnt(0)
	;;#ASMEND
	s_barrier
	buffer_load_dwordx4 v1, s[0:3], 0 offen lds
	{wait}
	ds_read_b128 v[4:7], v2
	s_cbranch_scc1 .LBB0_1
	s_endpgm
"""


def test_drain_flagged_when_compiler_waits_for_this_iterations_dma():
    assert len(_drains(LOOP.format(wait='s_waitcnt vmcnt(0)'))) == 1


def test_drain_not_flagged_when_the_dma_may_stay_in_flight():
    assert _drains(LOOP.format(wait='s_waitcnt vmcnt(1)')) == []


def test_drain_not_flagged_for_the_loop_top_inline_asm_wait():
    assert _drains(LOOP.format(wait='v_mov_b32_e32 v3, v4')) == []


def test_drain_across_a_rotated_loop():
    # the DMA in a block laid out above the header, the wait behind a VGPR load in another:
    # the round-6 records-GEMM pattern (an indexed kernel-argument load inside the tile loop)
    body = """
	s_branch .LBB0_3
.LBB0_2:                                ;   in Loop: Header=BB0_3 Depth=1
	buffer_load_dwordx4 v1, s[0:3], 0 offen lds
	global_load_dword v9, v[10:11], off
	s_waitcnt vmcnt(0)
	v_add_f32_e32 v3, v9, v4
.LBB0_3:                                ; =>This Inner Loop Header: Depth=1
	;;#ASMSTART
	s_waitcnt vmcnt(0)
	;;#ASMEND
	s_barrier
	s_cbranch_scc1 .LBB0_2
	s_endpgm
"""
    assert len(_drains(body)) == 1


@pytest.mark.skipif(not os.path.exists('/opt/rocm/lib/llvm/bin/llc'), reason='llc not present')
def test_hazard_rules_match_the_scanner_table():
    import mfma_hazard_rules as mhr
    t = mhr.probe()
    raw, war_c, part = mhc.RULES['16x16x32']
    assert t['raw_valu']['16x16x32_bf16'] == raw
    assert t['war_c_valu']['16x16x32_bf16'] == war_c
    assert t['raw_mfma_c_part']['16x16x32_bf16'] == part
    assert t['raw_valu']['32x32x16_bf16'] == mhc.RULES['32x32x16'][0]
    assert t['valu_mfma_ab']['16x16x32_bf16'] == mhc.VALU_TO_MFMA_AB

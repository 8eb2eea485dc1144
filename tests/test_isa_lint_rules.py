"""The rules of tools/isa_lint.py on hand-written gfx950 disassembly (CPU only, no tools):
R1 fires only for a 12/16-B buffer store with a register soffset whose data VGPRs the very
next VALU instruction writes; R2 for every buffer store with a register soffset; a constant
soffset (the engine's form, nw_fft_dev.h store_row) is clean."""
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, 'tools'))
import isa_lint  # noqa: E402


def _asm(*lines):
    head = ['', 'Disassembly of section .text:', '', '0000000000001000 <kern>:']
    return '\n'.join(head + ['\t' + l + ' // 000000001000: DEADBEEF' for l in lines]) + '\n'


def test_register_soffset_then_overwrite_is_r1_and_r2():
    finds, n = isa_lint.lint_asm(_asm('buffer_store_dwordx4 v[4:7], v1, s[8:11], s12 offen nt',
                                      'v_mov_b32_e32 v4, 0'))
    assert n == 1
    assert sorted(f[0] for f in finds) == ['R1', 'R2']
    assert all(f[1] == 'kern' for f in finds)


def test_overwrite_of_a_later_data_register_is_r1():
    finds, _ = isa_lint.lint_asm(_asm('buffer_store_dwordx3 v[10:12], v1, s[8:11], s2 offen',
                                      'v_cndmask_b32_e32 v12, v3, v5, vcc'))
    assert sorted(f[0] for f in finds) == ['R1', 'R2']


def test_register_soffset_without_overwrite_is_r2_only():
    finds, _ = isa_lint.lint_asm(_asm('buffer_store_dwordx4 v[4:7], v1, s[8:11], s12 offen',
                                      'v_add_u32_e32 v9, v2, v3',
                                      'buffer_store_dword v5, v1, s[8:11], s13 offen',
                                      'v_mov_b32_e32 v5, 0'))
    assert [f[0] for f in finds] == ['R2', 'R2']     # a 4-B store is not the 12/16-B hazard


def test_constant_soffset_is_clean():
    finds, n = isa_lint.lint_asm(_asm('buffer_store_dwordx4 v[4:7], v1, s[8:11], 0 offen nt',
                                      'v_mov_b32_e32 v4, 0',
                                      'buffer_store_dwordx2 v[2:3], v1, s[8:11], 0 offen offset:256'))
    assert n == 2 and finds == []


def test_non_valu_successor_is_not_r1():
    finds, _ = isa_lint.lint_asm(_asm('buffer_store_dwordx4 v[4:7], v1, s[8:11], s12 offen',
                                      's_waitcnt vmcnt(0)',
                                      'v_mov_b32_e32 v4, 0'))
    assert [f[0] for f in finds] == ['R2']

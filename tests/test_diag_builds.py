"""The diagnostic compile switches still build (CPU: device-only compiles, nothing runs).

Ablation and stamp builds are how the kernels' time was split up (no stores /
no twiddles / no exchanges / no W loads / column-pass ablations, NW_STAMPS phase stamps) and
how A/B variants were measured (tools/ab.sh); a switch no build exercises would rot.  Each
source is compiled once with all of its switches on (they are independent)."""
import os
import subprocess

import pytest

from conftest import ROOT

HIPCC = '/opt/rocm/bin/hipcc'
CSRC = os.path.join(ROOT, 'ninwavelets_amd', 'csrc')
SWITCHES = {
    'nw_fused.hip': ['NW_ABL_NOWLOAD', 'NW_STAMPS', 'NW_ABL_NOSTORE', 'NW_ABL_NOTWIDDLE', 'NW_ABL_NOEXCH',
                     'NW_PAIR_PAD16=0', 'NW_TAIL_EXACT', 'NW_PACK_MAX=4', 'NW_PAIR_XD_ALL', 'NW_F64_FINE=0',
                     'NW_GROUP64=4', 'NW_TILE64_F=4', 'NW_TILE64_G=8', 'NW_WKEEP64=4', 'NW_PRIO64=0',
                     'NW_GROUP64_16K=8', 'NW_TILE64_G_16K=4'],
    'nw_large.hip': ['NW_ABL_ROWS_NOW', 'NW_B_PLAIN', 'NW_ABL_COLS_NOFFT', 'NW_ABL_COLS_NOSTORE',
                     'NW_ABL_COLS_NOTW', 'NW_ABL_COLS_STREAM', 'NW_ABL_ROWS_STREAM', 'NW_ABL_NOSTORE', 'NW_ABL_NOTWIDDLE', 'NW_ABL_NOEXCH',
                     'NW_ROWS_NO_REC', 'NW_TAIL_EXACT', 'NW_COLS64_E16'],
}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason='hipcc not available')
def test_diagnostic_switches_compile(tmp_path):
    procs = []
    for src, defs in SWITCHES.items():
        procs.append((src, subprocess.Popen(
            [HIPCC, '--offload-arch=gfx950', '-O3', '-std=c++20', '-fno-slp-vectorize', '--cuda-device-only',
             *[f'-D{d}' for d in defs], '-c', os.path.join(CSRC, src), '-o', str(tmp_path / (src + '.co'))],
            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
    for src, p in procs:
        _, err = p.communicate(timeout=600)
        assert p.returncode == 0, f'{src}: {err[-2000:]}'
        assert os.path.getsize(tmp_path / (src + '.co')) > 0

"""ISA lint of the built gfx950 code objects (CPU only: disassembly, no kernel runs).

The buffer-store data hazard (tools/isa_lint.py): with a register in a buffer store's SGPR
soffset field the compiler does not guard the next VALU write of the store's data VGPRs,
and on gfx950 that corrupted paired C3 |cwt|^2 outputs (base.py:409-425) nondeterministically
in round 3.  The product and debug libraries must have no such store (R2) and no such
overwrite (R1); the deliberately hazardous form (NW_LINT_HAZARD_SOFFSET, the offset in the
soffset field as the first buffer form had it) must trip both rules."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, 'tools'))
import isa_lint  # noqa: E402

HIPCC = '/opt/rocm/bin/hipcc'
TOOLS_OK = (os.path.exists(f'{isa_lint.LLVM}/llvm-objdump') and os.path.exists(f'{isa_lint.LLVM}/clang-offload-bundler')
            and shutil.which('objcopy') is not None)
pytestmark = pytest.mark.skipif(not TOOLS_OK, reason='llvm-objdump / clang-offload-bundler / objcopy not available')


@pytest.mark.parametrize('lib', ['libninwave.so', 'libninwave_debug.so'])
def test_built_libraries_have_no_soffset_buffer_stores(lib):
    path = os.path.join(ROOT, 'ninwavelets_amd', lib)
    if not os.path.exists(path):
        pytest.skip(f'{lib} not built')
    finds, nstores, nobj = isa_lint.lint_file(path)
    assert nobj >= 4                       # kernels, fused, two-pass and chirp-z code objects
    # the signal-pair kernel's stores (kStoreBuffer): every output kind x n = 1024 .. 4096
    assert nstores >= 100
    assert finds == [], finds[:5]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason='hipcc not available')
def test_hazardous_variant_trips_the_lint(tmp_path):
    out = tmp_path / 'hazard.co'
    subprocess.run([HIPCC, '--offload-arch=gfx950', '-O3', '-std=c++20', '-fno-slp-vectorize', '--cuda-device-only',
                    '-DNW_LINT_HAZARD_SOFFSET', '-c', os.path.join(ROOT, 'ninwavelets_amd', 'csrc', 'nw_fused.hip'),
                    '-o', str(out)], check=True, capture_output=True, timeout=600)
    finds, nstores, nobj = isa_lint.lint_file(str(out))
    assert nobj == 1 and nstores >= 100
    rules = {f[0] for f in finds}
    assert rules == {'R1', 'R2'}, rules
    # R1 is the corruption seen in round 3: a 16-B store's FIRST data VGPR overwritten next
    r1 = [f for f in finds if f[0] == 'R1']
    assert all('nw_fused_pair_kernel' in f[1] and 'buffer_store_dwordx4' in f[3] for f in r1)

"""The numpy drop-in as the reference's users run it: a child process that never imports
torch (the reference imports only numpy / scipy / cupy, /root/reference/ninwavelets/base.py:1-4),
so libninwave.so binds /opt/rocm's HIP runtime and rocFFT instead of the torch wheel's.
tests/torchfree_parity.py runs the single-signal goldens, the benchmark-length goldens and
the C3 / C4 bench shapes there (tolerances as test_gpu_parity.py)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_numpy_dropin_parity_without_torch():
    env = {k: v for k, v in os.environ.items() if k != 'NINWAVE_LIB'}
    r = subprocess.run([sys.executable, '-u', os.path.join(ROOT, 'tests', 'torchfree_parity.py')],
                       capture_output=True, text=True, timeout=600, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    d = json.loads(lines[-1])
    assert not d['torch_imported']
    assert r.returncode == 0 and not d['failures'], d
    assert d['counts']['single'] >= 100 and d['counts']['long'] >= 8 and d['counts']['bench_shapes'] == 2
    # the runtime the child bound: /opt/rocm's, not a torch wheel's bundled copy
    assert d['runtime'] and all('torch' not in p for p in d['runtime']), d['runtime']

"""The debug library (SURVEY §5 "Race detection / sanitizers": bounds asserts in debug kernels).
libninwave_debug.so is the product sources built with -DNW_DEBUG_BOUNDS (nw_dcheck.h): the
kernels check their LDS-image indices, output indices, row maps and W-support values, a
failing check is counted on the device (nothing traps), and every API call synchronises and
fails with NW_E_BOUNDS naming file:line.  Run in child processes (NINWAVE_LIB picks the
library at load time)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

DEBUG_LIB = os.path.join(ROOT, 'ninwavelets_amd', 'libninwave_debug.so')


def child(args, timeout=600):
    env = dict(os.environ, NINWAVE_LIB=DEBUG_LIB)
    return subprocess.run([sys.executable, '-u', *args], capture_output=True, text=True, timeout=timeout, env=env)


def test_debug_checks_fire():
    """A kernel whose checks fail on purpose (lanes >= 32 of one 64-lane block): the status is
    NW_E_BOUNDS with the count and the site; the next call starts clean."""
    code = ('import sys; sys.path.insert(0, %r)\n'
            'from ninwavelets_amd import _lib as L\n'
            'lib = L.lib()\n'
            'print("debug", lib.nw_debug_bounds())\n'
            'print("rc", lib.nw_debug_selftest(0))\n'
            'print("msg", lib.nw_last_error().decode())\n'
            'print("rc2", lib.nw_debug_selftest(0))\n') % ROOT
    r = child(['-c', code], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = dict(ln.split(' ', 1) for ln in r.stdout.splitlines() if ' ' in ln)
    assert out['debug'] == '1'
    assert int(out['rc']) == -7 and int(out['rc2']) == -7          # NW_E_BOUNDS, each time
    assert '32 failing check(s), first at nw_kernels.hip:' in out['msg'], out['msg']


def test_parity_suite_under_bounds_checks():
    """tests/torchfree_parity.py (every single-signal golden on both engines, the benchmark-
    length goldens, the C3 / C4 bench shapes, epoch reductions on every engine form) on the
    debug library: no check fails and the results stay within the parity tolerances."""
    r = child([os.path.join(ROOT, 'tests', 'torchfree_parity.py')])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    d = json.loads(lines[-1])
    assert d['debug_bounds'] == 1 and d['lib'] == DEBUG_LIB
    assert r.returncode == 0 and not d['failures'], d
    assert d['counts']['single'] >= 100 and d['counts']['reductions'] == 6


def test_nw_log_names_the_engine_and_kernels():
    """NW_LOG=2 (SURVEY §5 "Metrics / logging"): one line per plan, wavelet, execute and
    reduction-path decision, and per launch stage with its kernel and time (NW_TIMING)."""
    code = ('import sys; sys.path.insert(0, %r)\n'
            'import numpy as np\n'
            'import ninwavelets_amd as nw\n'
            'from ninwavelets_amd import _lib as L\n'
            'x = np.random.default_rng(0).standard_normal((3, 4096)).astype(np.float32)\n'
            'g = L.trans_grid(4.096, 1000., False)\n'
            'p = nw.Plan(4096, 8, "float32", max_batch=4, timing=True)\n'
            'p.set_wavelet("morse", [17.5, 3.], np.arange(1., 9.), g)\n'
            'p.execute(x, out_kind="power")\n'
            'p.execute(x, out_kind="power_mean")\n'
            'p.close()\n') % ROOT
    env = {k: v for k, v in os.environ.items() if k != 'NINWAVE_LIB'}
    env['NW_LOG'] = '2'
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    log = [ln for ln in r.stderr.splitlines() if ln.startswith('[ninwave] ')]
    text = '\n'.join(log)
    assert 'n 4096 nfreq 8 float32 max_batch 4: fused engine, one-pass form' in text, text
    assert 'wavelet kind 1, 8 scales (every row distinct)' in text
    assert 'execute power, 3 signals, host buffers' in text
    assert 'launch fused: nw_fused_pair_kernel' in text
    assert 'power_mean over 3 signals: fp64 block partial sums inside the transform kernel' in text
    assert any(ln.startswith('[ninwave] plan') and ' fused ' in ln and ln.endswith(' ms') for ln in log), text

"""Sanitizer build of the engine's host-only logic ("-fsanitize=address on the
CPU path").  ninwavelets_amd/csrc/nw_host.cpp -- numpy-exact grid lengths, Normal-mode
row timelines, distinct-row grouping with row hashing, balanced signal blocks and the
threaded copy-out -- is compiled with g++ -fsanitize=address,undefined together with the
driver tests/asan/host_asan.cpp; any out-of-bounds access, leak or UB aborts the run."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def host_asan(tmp_path_factory):
    gxx = shutil.which('g++')
    if gxx is None:
        pytest.skip('g++ not available')
    exe = str(tmp_path_factory.mktemp('asan') / 'host_asan')
    subprocess.run([gxx, '-std=c++20', '-O1', '-g', '-fsanitize=address,undefined', '-fno-omit-frame-pointer',
                    '-fno-sanitize-recover=all', '-pthread',
                    os.path.join(ROOT, 'ninwavelets_amd', 'csrc', 'nw_host.cpp'),
                    os.path.join(ROOT, 'tests', 'asan', 'host_asan.cpp'), '-o', exe], check=True)
    return exe


ENV = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=1', UBSAN_OPTIONS='halt_on_error=1')


def test_host_logic_under_asan(host_asan):
    r = subprocess.run([host_asan, 'self'], capture_output=True, text=True, env=ENV, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == 'ok'


def test_trans_grid_under_asan_matches_numpy(host_asan):
    """nw::host::trans_grid (the nw_trans_grid body) against numpy's arange length
    (base.py:191-194, 238-245) on random (N, sfreq, interpolate)."""
    rng = np.random.default_rng(3)
    cases = [(int(n), float(sf), int(i)) for n, sf, i in zip(rng.integers(1, 70000, 600),
                                                             rng.choice([100., 250., 500., 512., 1000., 1024.,
                                                                         2048., 600.5], 600),
                                                             rng.integers(0, 2, 600))]
    inp = ''.join(f'{n / sf!r} {sf!r} {i}\n' for n, sf, i in cases)
    r = subprocess.run([host_asan, 'grid'], input=inp, capture_output=True, text=True, env=ENV, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split('\n')
    for (n, sf, interp), ln in zip(cases, lines):
        rl = n / sf
        one = 1 / rl
        rwl = rl / 2 if interp else rl
        want = len(np.arange(0, sf / rl * rwl, one))
        lv, lf, d = ln.split()
        assert int(lv) == want and int(lf) == (2 * want if interp else want) and float(d) == one, (n, sf, interp)

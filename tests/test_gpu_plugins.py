"""User plugins through the drop-in on the GPU, against the reference's own outputs.

The reference's extension point is a user subclass of WaveletBase (or of a stock wavelet)
overriding trans_formula / formula / peak_freq (README.md:342-355), in any WaveletMode
(base.py:126-142, 221-256, 346-359).  tests/golden/make_golden_plugins.py ran four such
plugins on the reference (Reverse, a Morse subclass, Normal, Twice; tests/plugins.py) at a
power-of-two length, an MNE length (interpolating) and a short one; here the same plugin
classes built on ninwavelets_amd run their host-built table rows through the device engines
(fused complex-row kernel, chirp-z form, rocFFT) in fp64 and fp32.
Tolerances as test_gpu_parity.py: fp64 1e-12 of max|ref|, fp32 1e-5 (x2 for |.|^2)."""
import numpy as np
import pytest

from conftest import golden_names, load_golden
import plugins

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402

NAMES = golden_names('plugin_')


def test_every_plugin_mode_has_goldens():
    modes = {load_golden(n)['meta']['mode'] for n in NAMES}
    assert modes == {'Reverse', 'Normal', 'Twice'} and len(NAMES) == len(plugins.CASES)


@pytest.mark.parametrize('engine', ['auto', 'rocfft'])
@pytest.mark.parametrize('dtype', ['float64', 'float32'])
@pytest.mark.parametrize('name', NAMES)
def test_plugin_against_reference(name, dtype, engine):
    g = load_golden(name)
    m = g['meta']
    w = plugins.make(nw, m['plugin'], m['sfreq'], m['interpolate'], dtype=dtype, engine=engine)
    got = w.cwt(g['x'], g['freqs'], reuse=False)
    ref = g['out']
    tol = 1e-12 if dtype == 'float64' else 1e-5
    assert got.dtype == (np.complex128 if dtype == 'float64' else np.complex64)
    assert np.max(np.abs(got - ref)) <= tol * np.max(np.abs(ref))
    pw = w.power(g['x'], None, reuse=True)
    assert np.max(np.abs(pw - g['power'])) <= 2 * tol * np.max(g['power'])
    st = next(iter(w._plans.values())).stats()
    if engine == 'auto':
        assert st['engine'] == 'fused'
        n = m['n']
        want = 'nw_fused_kernel' if n & (n - 1) == 0 and n >= 1024 else 'nw_chirp_kernel'
        assert L.KERNEL_NAMES[st['kernel']] == want

"""User wavelet plugins: the reference's extension point (README.md:342-355 "Way to inherit":
subclass WaveletBase and override ``formula`` / ``trans_formula`` / ``peak_freq``; the mode
picks the spectrum source, base.py:126-142, 221-256, 346-359).

Test infrastructure.  The same four plugins are built on either package by ``make(pkg, name)``:
on the reference (tests/golden/make_golden_plugins.py, this container only) to generate the
fixtures, and on ninwavelets_amd (tests/test_gpu_plugins.py) to run them through the drop-in.
The formulas are plain numpy and shared, so both packages evaluate the same plugin code.

  gauss_bump  WaveletMode.Reverse, a WaveletBase subclass overriding trans_formula
  morse_sqrt  a Morse subclass overriding trans_formula (calls the stock one through super())
  paul        WaveletMode.Normal, overriding formula + peak_freq (complex time-domain wavelet)
  twice_bump  WaveletMode.Twice, overriding trans_formula (evaluated as base.py:349-355 does:
              ifft of the spectrum on the freq's own grid, conj-mirrored, then FFT'd back)
"""
from __future__ import annotations

import numpy as np


def gauss_bump_trans(self, freqs, freq=1.):
    return 2.0 * np.exp(-np.square((freqs - freq) / (0.2 * freq + 0.5)))


def morse_sqrt_trans(self, freqs, freq=1.):
    return np.sqrt(super(type(self), self).trans_formula(freqs, freq))


def paul_formula(self, timeline, freq=1.):
    return np.power(1.0 - 1j * timeline, -5.0)


def paul_peak(self, freq):
    return 0.7 + 0.002 * freq


def twice_bump_trans(self, freqs, freq=1.):
    return np.exp(-np.square(freqs - 15.0) / 20.0)


# name -> (base class name, mode name, methods)
PLUGINS = {
    'gauss_bump': ('WaveletBase', 'Reverse', {'trans_formula': gauss_bump_trans}),
    'morse_sqrt': ('Morse', None, {'trans_formula': morse_sqrt_trans}),
    'paul': ('WaveletBase', 'Normal', {'formula': paul_formula, 'peak_freq': paul_peak}),
    'twice_bump': ('WaveletBase', 'Twice', {'trans_formula': twice_bump_trans}),
}

# (plugin, n, freqs, interpolate): a power-of-two length (fused kernel, complex table rows),
# an MNE length (chirp-z form) and a short one; Twice / Normal rows are sfreq * real_wave_length
# = 1000 points, cropped or centre-padded to n (base.py:75-82)
CASES = [
    ('gauss_bump', 512, [5., 12., 30., 70.], False),
    ('gauss_bump', 1201, [3., 8., 20., 45., 90.], True),
    ('gauss_bump', 300, [10., 40.], False),
    ('morse_sqrt', 1024, [4., 16., 64.], False),
    ('morse_sqrt', 1201, [2., 9., 31., 77.], True),
    ('morse_sqrt', 300, [10., 25., 60.], False),
    ('paul', 2048, [3., 10., 40.], False),
    ('paul', 1201, [5., 20.], True),
    ('paul', 300, [8., 30.], False),
    ('twice_bump', 1024, [2., 6., 20., 50.], False),
    ('twice_bump', 1201, [4., 11., 33.], True),
    ('twice_bump', 300, [5., 25.], False),
]


def make(pkg, name: str, sfreq: float = 1000., interpolate: bool = False, **kw):
    """An instance of plugin `name` built on package `pkg` (the reference's ninwavelets or
    ninwavelets_amd): both export WaveletBase, WaveletMode and Morse.  kw: constructor
    keywords of the drop-in only (dtype, engine, ...)."""
    base_name, mode, methods = PLUGINS[name]
    base = getattr(pkg, base_name)
    mode_v = getattr(pkg.WaveletMode, mode) if mode else None

    def __init__(self, sfreq=1000., interpolate=False, **kw):
        base.__init__(self, sfreq, interpolate=interpolate, **kw)
        if mode_v is not None:
            self.mode = mode_v

    cls = type(f'Plugin_{name}', (base,), dict(methods, __init__=__init__))
    return cls(sfreq, interpolate=interpolate, **kw)


def case_name(name: str, n: int, interpolate: bool) -> str:
    return f'plugin_{name}_n{n}' + ('_interp' if interpolate else '')

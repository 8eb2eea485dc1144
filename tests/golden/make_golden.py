"""Generate golden input/output vectors by running the REFERENCE itself.

Runs only in the build container, where the read-only reference tree is
mounted at /root/reference.  It imports ``ninwavelets`` from there (with a
stub ``cupy`` module: the CPU path only touches ``cp.ndarray`` in type
annotations, base.py:12, wavelets.py:53-54, 124-125) and writes small
compressed ``.npz`` fixtures (inputs + reference outputs) next to this file.
Nothing from the reference is copied: only the numbers it computes.

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


def load_reference():
    stub = types.ModuleType('cupy')
    stub.ndarray = object
    sys.modules.setdefault('cupy', stub)
    sys.path.insert(0, REF)
    import ninwavelets  # noqa: E402  (never ninwavelets.init — it chdirs and runs setup.py)
    return ninwavelets


class FakeEpochs:
    """Duck-typed mne.Epochs: info['sfreq'], ch_names, get_data() (mneutils.py:24, 37-38)."""

    def __init__(self, data, sfreq, ch_names):
        self._data = data
        self.info = {'sfreq': sfreq}
        self.ch_names = list(ch_names)

    def get_data(self):
        return self._data


def save(name, meta, **arrays):
    path = os.path.join(OUT, name + '.npz')
    np.savez_compressed(path, meta=np.array(json.dumps(meta)), **arrays)
    print(f'{name:34s} ' + ' '.join(f'{k}{tuple(v.shape)}' for k, v in arrays.items()))


def main():
    nw = load_reference()
    rng = np.random.default_rng(0)

    def signal(n, dtype=np.float64, sfreq=1000.):
        t = np.arange(n) / sfreq
        f1, f2 = rng.uniform(3, 120, 2)
        x = np.sin(2 * np.pi * f1 * t) + 0.5 * np.sin(2 * np.pi * f2 * t + 1.0) \
            + 0.1 * rng.standard_normal(n)
        return x.astype(dtype)

    def ctor(kind, sfreq, interpolate, params):
        if kind == 'morse':
            return nw.Morse(sfreq, b=params.get('b', 17.5), r=params.get('r', 3.),
                            interpolate=interpolate)
        if kind == 'morlet':
            return nw.Morlet(sfreq, sigma=params.get('sigma', 7.),
                             gabor=params.get('gabor', False), interpolate=interpolate)
        if kind == 'shannon':
            return nw.Shannon(sfreq, interpolate=interpolate)
        if kind == 'mexican_hat':
            return nw.MexicanHat(sfreq, sigma=params.get('sigma', 7.),
                                 real_wave_length=params.get('real_wave_length', 1.),
                                 interpolate=interpolate)
        if kind == 'haar':
            return nw.Haar(sfreq, interpolate=interpolate)
        raise ValueError(kind)

    # ---- single-signal CWT cases: (name, kind, N, freqs, sfreq, interpolate, params, dtype)
    cases = [
        ('morse_n21', 'morse', 21, list(range(1, 11)), 1000., False, {}, np.float64),
        ('morse_n29', 'morse', 29, [2., 5., 11.], 1000., False, {}, np.float64),
        ('morse_n300', 'morse', 300, list(range(1, 100, 7)), 1000., False, {}, np.float64),
        ('morse_n301', 'morse', 301, list(range(1, 100, 9)), 1000., False, {}, np.float64),
        ('morse_n1024', 'morse', 1024, list(range(1, 65, 4)), 1000., False, {}, np.float64),
        ('morse_n4096', 'morse', 4096, [5., 10., 17.5, 23., 31., 40., 77., 120.], 1000., False, {}, np.float64),
        ('morse_b3r2_n512', 'morse', 512, [4., 9., 30., 60.], 1000., False, {'b': 3., 'r': 2.}, np.float64),
        ('morse_f01_n2048', 'morse', 2048, [0.1, 0.2, 0.5, 1.0], 1000., False, {}, np.float64),
        ('morse_interp_n300', 'morse', 300, list(range(1, 100, 11)), 1000., True, {}, np.float64),
        ('morse_interp_n301', 'morse', 301, list(range(1, 100, 11)), 1000., True, {}, np.float64),
        ('morse_interp_n1024', 'morse', 1024, list(range(2, 200, 25)), 1000., True, {}, np.float64),
        ('morse_f32_n1024', 'morse', 1024, list(range(1, 65, 8)), 1000., False, {}, np.float32),
        ('morse_sfreq500_n1000', 'morse', 1000, [1.5, 3., 7.25, 12.], 500., False, {}, np.float64),
        ('morlet_n300', 'morlet', 300, list(range(1, 100, 7)), 1000., False, {}, np.float64),
        ('morlet_n1024', 'morlet', 1024, list(range(1, 129, 16)), 1000., False, {}, np.float64),
        ('morlet_gabor_n1024', 'morlet', 1024, list(range(1, 129, 16)), 1000., False, {'gabor': True}, np.float64),
        ('morlet_s5_n700', 'morlet', 700, [0.5, 3., 20., 90.], 1000., False, {'sigma': 5.}, np.float64),
        ('morlet_interp_n1024', 'morlet', 1024, list(range(1, 129, 16)), 1000., True, {}, np.float64),
        ('shannon_n1024', 'shannon', 1024, [1., 10., 50., 100.], 1000., False, {}, np.float64),
        ('shannon_n300', 'shannon', 300, [3., 7.], 1000., False, {}, np.float64),
        ('shannon_interp_n512', 'shannon', 512, [3., 7.], 1000., True, {}, np.float64),
        ('mexhat_n1024', 'mexican_hat', 1024, [2., 5., 10., 20., 40., 80.], 1000., False, {}, np.float64),
        ('mexhat_n300', 'mexican_hat', 300, [2., 10., 40.], 1000., False, {}, np.float64),
        ('mexhat_n2500', 'mexican_hat', 2500, [2., 10., 40.], 1000., False, {}, np.float64),
        ('mexhat_interp_n1024', 'mexican_hat', 1024, [2., 10., 40.], 1000., True, {}, np.float64),
        ('haar_n1000', 'haar', 1000, [1., 3., 9., 27.], 1000., False, {}, np.float64),
    ]
    for name, kind, n, freqs, sfreq, interp, params, dtype in cases:
        w = ctor(kind, sfreq, interp, params)
        x = signal(n, dtype, sfreq)
        out = w.cwt(x, freqs, reuse=False)
        rows = w.fft_wavelets
        meta = dict(kind=kind, n=n, sfreq=sfreq, interpolate=interp, params=params,
                    dtype=np.dtype(dtype).name, op='cwt')
        arrays = dict(x=x, freqs=np.asarray(freqs, dtype=np.float64), out=out)
        if n <= 1024 and len(freqs) <= 16:
            # first and last wavelet rows for kernel-level checks of the spectrum evaluation
            arrays['w_first'] = np.asarray(rows[0])
            arrays['w_last'] = np.asarray(rows[-1])
        save(name, meta, **arrays)

    # ---- README example (README.md:60-82, wavelets.py:11-19): 2-D (1,300) input and 1-D
    t = np.arange(0, 0.3, 0.001)
    sin2d = np.array([np.sin(t * 60 * 2 * np.pi)])
    for kind in ('morse', 'morlet', 'shannon', 'mexican_hat'):
        w = ctor(kind, 1000, False, {})
        p2 = w.power(sin2d, range(1, 100), reuse=False)
        save(f'readme_2d_{kind}', dict(kind=kind, n=300, sfreq=1000., interpolate=False,
                                       params={}, dtype='float64', op='power'),
             x=sin2d, freqs=np.arange(1, 100, dtype=np.float64), out=p2)
    w = ctor('morse', 1000, False, {})
    p1 = w.power(sin2d[0], range(1, 100), reuse=False)
    save('readme_1d_morse_power', dict(kind='morse', n=300, sfreq=1000., interpolate=False,
                                        params={}, dtype='float64', op='power'),
         x=sin2d[0], freqs=np.arange(1, 100, dtype=np.float64), out=p1)
    a1 = w.abs(sin2d[0], range(1, 100), reuse=True)
    save('readme_1d_morse_abs', dict(kind='morse', n=300, sfreq=1000., interpolate=False,
                                      params={}, dtype='float64', op='abs'),
         x=sin2d[0], freqs=np.arange(1, 100, dtype=np.float64), out=a1)

    # ---- reuse quirk: the cache is not keyed on freqs or N (base.py:394-397)
    w = ctor('morse', 1000, False, {})
    xa, xb, xc = signal(300), signal(600), signal(200)
    oa = w.cwt(xa, [5., 10., 20., 40.])
    ob = w.cwt(xb, [1., 2.])          # freqs ignored, W centre-padded 300 -> 600
    oc = w.cwt(xc, None)              # W cropped 300 -> 200
    save('reuse_morse', dict(kind='morse', sfreq=1000., interpolate=False, params={},
                             dtype='float64', op='reuse'),
         xa=xa, xb=xb, xc=xc, freqs=np.array([5., 10., 20., 40.]), oa=oa, ob=ob, oc=oc)
    w = ctor('morse', 1000, True, {})
    oa = w.cwt(xa, [5., 10., 20., 40.])
    ob = w.cwt(xb, [1., 2.])
    save('reuse_morse_interp', dict(kind='morse', sfreq=1000., interpolate=True, params={},
                                    dtype='float64', op='reuse'),
         xa=xa, xb=xb, freqs=np.array([5., 10., 20., 40.]), oa=oa, ob=ob)

    # ---- make_example (test.py:17-27) power, 1 s at 1 kHz
    ex_t = np.arange(0, 1.0, 0.001)
    ex = (np.sin(ex_t * 60 * 2 * np.pi) + np.sin(ex_t * 160 * 2 * np.pi) * np.sin(ex_t * np.pi)
          + np.sin(np.pad(np.arange(0, 0.5, 0.001), [250, 250], 'constant') * 300 * 2 * np.pi))
    w = ctor('morse', 1000, False, {})
    pex = w.power(ex, [20., 60., 100., 160., 230., 300.], reuse=False)
    save('example_morse_power', dict(kind='morse', n=ex.shape[0], sfreq=1000., interpolate=False,
                                     params={}, dtype='float64', op='power'),
         x=ex, freqs=np.array([20., 60., 100., 160., 230., 300.]), out=pex)

    # ---- EpochsWavelet with a duck-typed epochs object (mneutils.py:9-71), sfreq 500
    E, C, N = 5, 3, 256
    data = np.stack([np.stack([signal(N, sfreq=500.) for _ in range(C)]) for _ in range(E)])
    freqs = list(np.linspace(2., 40., 6))
    for kind in ('morse', 'morlet'):
        ep = FakeEpochs(data, 500., ['a', 'b', 'c'])
        ew = nw.EpochsWavelet(ep, ctor(kind, 1000, False, {}))   # sfreq overwritten to 500
        c = ew.cwt('b', freqs)
        ew2 = nw.EpochsWavelet(ep, ctor(kind, 1000, False, {}))
        p = ew2.power('c', freqs)
        ew3 = nw.EpochsWavelet(ep, ctor(kind, 1000, False, {}))
        itc = ew3.itc('a', freqs)
        save(f'epochs_{kind}', dict(kind=kind, n=N, sfreq=500., interpolate=False, params={},
                                    dtype='float64', op='epochs', ch_names=['a', 'b', 'c']),
             data=data, freqs=np.asarray(freqs), cwt_b=c, power_c=p, itc_a=itc)


if __name__ == '__main__':
    main()

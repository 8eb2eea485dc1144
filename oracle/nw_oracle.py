"""CPU oracle for the FFT-domain CWT hot path — TEST INFRASTRUCTURE ONLY.

This module is a from-scratch numpy/scipy.fftpack restatement of the
reference's CWT arithmetic (Hiroki-Maeda/ninwavelets, reference tree at
/root/reference, cited below as ``base.py:L`` / ``wavelets.py:L`` /
``mneutils.py:L``).  It is the *checker*: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``ninwavelets_amd``) never imports, calls or falls back
to anything in ``oracle/``.

Parity pinning: the reference has no tests and no golden vectors of its own
(SURVEY.md §4).  This restatement is pinned against golden vectors produced by
importing the reference itself in the build container
(``tests/golden/make_golden.py`` → ``tests/golden/*.npz``); see
``tests/test_oracle_golden.py``.

Third-party arithmetic: the FFTs are scipy.fftpack (pocketfft; scipy 1.15.3 in
this image, unpinned by the reference's setup.py:6) and the elementwise math is
numpy 2.2.6, exactly as the reference uses them (base.py:1-4).
"""
from __future__ import annotations

import numpy as np
from scipy.fftpack import fft, ifft

# ---------------------------------------------------------------------------
# grid / padding helpers
# ---------------------------------------------------------------------------


def trans_grid(sfreq: float, real_length: float, interpolate: bool) -> np.ndarray:
    """Frequency grid nu_k of the analytic-spectrum path.

    Follows base.py:173-194 (``_setup_trans_shape``) as it is called from
    base.py:238-245: ``freq = real_length`` and
    ``real_wave_length = real_length`` (or ``real_length / 2`` when
    interpolating), i.e. ``np.arange(0, sfreq / rl * rl', 1 / rl)``.
    """
    one = 1 / real_length
    rwl = real_length / 2 if interpolate else real_length
    total = sfreq / real_length * rwl
    return np.arange(0, total, one)


def pad_to(row: np.ndarray, n: int) -> np.ndarray:
    """Crop to n, or zero-pad centred (base.py:75-82)."""
    m = row.shape[0]
    if m > n:
        return row[:n]
    side1 = (n - m) // 2
    side2 = n - m - side1
    return np.pad(row, [side1, side2], 'constant')


def alias_mask(spec: np.ndarray) -> np.ndarray:
    """Keep the first int(len/2) bins and zero the rest (base.py:107-123)."""
    half = int(spec.shape[0] / 2)
    return np.pad(spec[:half], [0, spec.shape[0] - half], 'constant')


# ---------------------------------------------------------------------------
# analytic spectra (WaveletMode.Reverse / Both)
# ---------------------------------------------------------------------------


def morse_spectrum(nu: np.ndarray, freq: float, b: float = 17.5,
                   r: float = 3.0) -> np.ndarray:
    """Generalised Morse spectrum, wavelets.py:65-74."""
    x = nu / freq
    step = np.heaviside(x, x)
    return 2. * (step * np.float_power(x, b)
                 * np.exp((b / r) * (1. - np.float_power(x, r))))


def morlet_constants(sigma: float, gabor: bool):
    """(c, k) of wavelets.py:118-122."""
    c = np.float_power(1 + np.exp(-np.square(sigma))
                       - 2 * np.exp(-3 / 4 * np.square(sigma)), -1 / 2)
    k = 0 if gabor else np.exp(-np.float_power(sigma, 2) / 2)
    return c, k


def morlet_peak(sigma: float, freq: float) -> float:
    """wavelets.py:143-144."""
    return sigma / (1. - np.exp(-sigma * freq))


def morlet_spectrum(nu: np.ndarray, freq: float, sigma: float = 7.,
                    gabor: bool = False) -> np.ndarray:
    """Morlet/Gabor spectrum, wavelets.py:132-136."""
    c, k = morlet_constants(sigma, gabor)
    x = nu / freq * morlet_peak(sigma, freq)
    return (c * np.float_power(np.pi, -1 / 4)
            * (np.exp(-np.square(sigma - x) / 2) - k * np.exp(-np.square(x) / 2)))


def shannon_spectrum(nu: np.ndarray, freq: float) -> np.ndarray:
    """Shannon spectrum, wavelets.py:256-262: 1 where nu <= 1, else 0 (freq unused)."""
    return np.where(nu <= 1., 1., 0.).astype(np.float64)


# ---------------------------------------------------------------------------
# time-domain formulas (WaveletMode.Normal) → table path
# ---------------------------------------------------------------------------


def mexican_hat_formula(tc: np.ndarray, sigma: float = 7.) -> np.ndarray:
    """wavelets.py:219-221."""
    return (1 - np.power(tc / sigma, 2)) * np.exp(-np.square(tc) / np.square(sigma) / 2)


def haar_formula(tc: np.ndarray) -> np.ndarray:
    """wavelets.py:272-280 (vectorised; same piecewise values)."""
    out = np.zeros_like(tc, dtype=np.float64)
    out[(tc > 0.) & (tc <= 1.)] = 1.
    out[(tc > -1.) & (tc <= 0.)] = -1.
    return out


def normal_mode_spectrum(formula, peak: float, freq: float, sfreq: float,
                         real_wave_length: float) -> np.ndarray:
    """FFT of a centred time-domain wavelet, base.py:249-256 with
    make_wavelet/_setup_waveletshape (base.py:346-359, 196-216)."""
    total = 1 / peak * freq * 2 * np.pi
    one = 1 / sfreq * 2 * np.pi * freq / peak
    timeline = np.arange(-total / 2, total / 2, one)
    w = formula(timeline)
    half = int((sfreq * real_wave_length - w.shape[0]) / 2)
    w = np.hstack((np.zeros(half), w, np.zeros(half)))
    spec = fft(w)
    return np.abs(spec.real) + 1j * np.abs(spec.imag)


MEXICAN_HAT_PEAK = np.sqrt(6) / np.pi / np.pi   # wavelets.py:227-228


# ---------------------------------------------------------------------------
# wavelet table + CWT
# ---------------------------------------------------------------------------


def fft_wavelets(kind: str, freqs, sfreq: float, real_length: float,
                 interpolate: bool, real_wave_length: float = 1.0, **params):
    """List of per-frequency spectra, base.py:221-279 (make_fft_wavelet(s)).

    ``real_length`` is ``N / sfreq`` as passed by cwt (base.py:395).
    """
    freqs = list(freqs)
    if len(freqs) < 2:
        raise IndexError('freqs needs at least two entries (base.py:272)')
    rows = []
    for f in freqs:
        if f == 0:
            raise ZeroDivisionError
        if kind in ('morse', 'morlet', 'shannon'):
            nu = trans_grid(sfreq, real_length, interpolate)
            if kind == 'morse':
                w = morse_spectrum(nu, f, params.get('b', 17.5), params.get('r', 3.))
            elif kind == 'morlet':
                w = morlet_spectrum(nu, f, params.get('sigma', 7.), params.get('gabor', False))
            else:
                w = shannon_spectrum(nu, f)
            if interpolate:
                w = np.hstack((w, np.zeros(len(nu))))
        elif kind == 'mexican_hat':
            sig = params.get('sigma', 7.)
            w = normal_mode_spectrum(lambda t: mexican_hat_formula(t, sig),
                                     MEXICAN_HAT_PEAK, f, sfreq, real_wave_length)
        elif kind == 'haar':
            w = normal_mode_spectrum(haar_formula, 1.0, f, sfreq, real_wave_length)
        else:
            raise ValueError(kind)
        if interpolate:
            w = alias_mask(w)
        rows.append(w)
    return rows


def cwt_from_rows(x: np.ndarray, rows, interpolate: bool) -> np.ndarray:
    """ifft(pad_to(W) * fft(x)) of base.py:378-407 (CPU branch)."""
    n = x.shape[0]
    w = np.array([pad_to(r, n) for r in rows])
    spec = fft(x)
    if interpolate:
        spec = alias_mask(spec)
    return ifft(w * spec)


def cwt(kind: str, x: np.ndarray, freqs, sfreq: float = 1000.,
        interpolate: bool = False, real_wave_length: float = 1.0, **params) -> np.ndarray:
    """Uncached CWT of one 1-D signal (the reuse=False call of base.py:378)."""
    rows = fft_wavelets(kind, freqs, sfreq, x.shape[0] / sfreq, interpolate,
                        real_wave_length, **params)
    return cwt_from_rows(x, rows, interpolate)


def power(kind: str, x: np.ndarray, freqs, **kw) -> np.ndarray:
    """abs(cwt)**2, base.py:409-425."""
    return np.abs(cwt(kind, x, freqs, **kw)) ** 2


def epochs_cwt(kind: str, waves: np.ndarray, freqs, **kw) -> np.ndarray:
    """Per-epoch map with the table built once from epoch 0 (mneutils.py:26-40)."""
    sfreq = kw.pop('sfreq', 1000.)
    interpolate = kw.pop('interpolate', False)
    rwl = kw.pop('real_wave_length', 1.0)
    rows = fft_wavelets(kind, freqs, sfreq, waves[0].shape[0] / sfreq, interpolate, rwl, **kw)
    return np.array([cwt_from_rows(w, rows, interpolate) for w in waves])


def epochs_power(kind: str, waves: np.ndarray, freqs, **kw) -> np.ndarray:
    """Epoch-mean power, mneutils.py:42-55."""
    return np.mean(np.abs(epochs_cwt(kind, waves, freqs, **kw)) ** 2, axis=0)


def epochs_itc(kind: str, waves: np.ndarray, freqs, **kw) -> np.ndarray:
    """Inter-trial coherence, mneutils.py:57-71."""
    c = epochs_cwt(kind, waves, freqs, **kw)
    with np.errstate(invalid='ignore', divide='ignore'):
        return np.abs(np.mean(c / np.abs(c), axis=0))


# ---------------------------------------------------------------------------
# synthetic inputs shared by tests and bench (BASELINE.json configs)
# ---------------------------------------------------------------------------


def make_example(length: float = 3.0) -> np.ndarray:
    """The reference demo signal of test.py:17-27 (60 Hz + 160 Hz AM + 300 Hz burst)."""
    t = np.arange(0, length, 0.001)
    return (np.sin(t * 60 * 2 * np.pi)
            + np.sin(t * 160 * 2 * np.pi) * np.sin(t * np.pi)
            + np.sin(np.pad(np.arange(0, length / 2, 0.001),
                            [int(length * 250), int(length * 250)], 'constant')
                     * 300 * 2 * np.pi))


# ---------------------------------------------------------------------------
# Baseline correction (base.py:18-68): slice AXIS 0, one scalar mean / population
# std over the whole slice, then one elementwise op.
# ---------------------------------------------------------------------------
BASELINE_OPS = ('mean', 'ratio', 'percent', 'log', 'zscore', 'zlog')


def baseline(wave: np.ndarray, sfreq: float, start: float, stop: float, op: str) -> np.ndarray:
    """Baseline(wave, sfreq, start, stop).<op>() of base.py:23-68."""
    part = wave[int(start * sfreq): int(stop * sfreq)]          # base.py:18-20, 49
    m = part.mean()                                             # 50
    ops = {
        'mean': lambda: wave - m,                               # 53-54
        'ratio': lambda: wave / m,                              # 56-57
        'percent': lambda: (wave - m) / m,                      # 59-60
        'log': lambda: np.log10(wave / m),                      # 62-63
        'zscore': lambda: (wave - m) / np.std(part),            # 65-66
        'zlog': lambda: np.log10(wave / m) / np.std(part),      # 68-69
    }
    return ops[op]()


# ---------------------------------------------------------------------------
# Time-domain wavelets, make_wavelet(s) (base.py:346-376).  Reverse mode (Morse,
# Shannon): ifft of the spectrum on arange(0, sfreq/f*rwl, 1/f) with the spectrum's
# default freq = 1, then conj-flip + stack + centre slice.  Otherwise (Morlet's Both,
# MexicanHat / Haar's Normal): the time-domain formula on the zero-mean timeline.
# ---------------------------------------------------------------------------
def morlet_formula(tc: np.ndarray, sigma: float = 7., gabor: bool = False) -> np.ndarray:
    """wavelets.py:138-141."""
    c, k = morlet_constants(sigma, gabor)
    return c * np.float_power(np.pi, -1 / 4) * np.exp(-np.square(tc) / 2) * (np.exp(sigma * 1j * tc) - k)


def make_wavelet(kind: str, freq: float, sfreq: float = 1000., real_wave_length: float = 1.,
                 **params) -> np.ndarray:
    if freq == 0:
        raise ZeroDivisionError
    if kind in ('morse', 'shannon'):
        t = np.arange(0, sfreq / freq * real_wave_length, 1 / freq)          # base.py:191-194
        spec = (morse_spectrum(t, 1., params.get('b', 17.5), params.get('r', 3.)) if kind == 'morse'
                else shannon_spectrum(t, 1.))
        w = ifft(spec)
        half = int(w.shape[0])
        both = np.hstack((np.conj(np.flip(w)), w))
        return both[half // 2: half // 2 * 3]
    sigma = params.get('sigma', 7.)
    peak = {'morlet': lambda: morlet_peak(sigma, freq), 'mexican_hat': lambda: MEXICAN_HAT_PEAK,
            'haar': lambda: 1.}[kind]()
    total = 1. / peak * freq * 2 * np.pi                                      # base.py:211-216
    one = 1 / sfreq * 2 * np.pi * freq / peak
    tl = np.arange(-total / 2, total / 2, one)
    if kind == 'morlet':
        return morlet_formula(tl, sigma, params.get('gabor', False))
    return mexican_hat_formula(tl, sigma) if kind == 'mexican_hat' else haar_formula(tl)


def make_wavelets(kind: str, freqs, **kw) -> list:
    return [make_wavelet(kind, f, **kw) for f in freqs]


# ---------------------------------------------------------------------------
# user plugins (README.md:342-355): any WaveletBase subclass, by its mode
# ---------------------------------------------------------------------------


def plugin_row(mode: str, trans_formula, formula, peak_freq, freq: float, sfreq: float,
               real_length: float, interpolate: bool, real_wave_length: float = 1.) -> np.ndarray:
    """One cached row of a user plugin: make_fft_wavelet (base.py:221-256) by the plugin's
    mode name.  Reverse / Both: the spectrum on the trans grid (base.py:238-245, ×2 zero-padded
    when interpolating); Normal / Twice / Indifferentiable: the FFT of the zero-padded
    time-domain wavelet, |Re| + i|Im| (base.py:247-256), where make_wavelet (base.py:346-359)
    takes Twice (and Reverse) through ifft(trans_formula(t)) on the freq's own grid
    (trans_formula called with its default freq, base.py:350), conj-mirrored, and the others
    through formula(timeline, freq) on _setup_waveletshape's grid (base.py:196-216)."""
    if freq == 0:
        raise ZeroDivisionError
    if mode in ('Reverse', 'Both'):
        nu = trans_grid(sfreq, real_length, interpolate)
        w = trans_formula(nu, freq)
        return np.hstack((w, np.zeros(len(nu)))) if interpolate else w
    # (Reverse returned above: base.py:238-250 reaches make_wavelet only for the other modes)
    if mode == 'Twice':
        t = np.arange(0, sfreq / freq * real_wave_length, 1 / freq)          # base.py:191-194
        w = ifft(trans_formula(t))
        half = int(w.shape[0])
        w = np.hstack((np.conj(np.flip(w)), w))[half // 2: half // 2 * 3]
    else:
        peak = peak_freq(freq)
        total = 1 / peak * freq * 2 * np.pi                                   # base.py:211-216
        one = 1 / sfreq * 2 * np.pi * freq / peak
        w = formula(np.arange(-total / 2, total / 2, one), freq)
    half = int((sfreq * real_wave_length - w.shape[0]) / 2)
    spec = fft(np.hstack((np.zeros(half), w, np.zeros(half))))
    return np.abs(spec.real) + 1j * np.abs(spec.imag)


def plugin_cwt(mode: str, trans_formula, formula, peak_freq, x: np.ndarray, freqs,
               sfreq: float = 1000., interpolate: bool = False, real_wave_length: float = 1.):
    """Uncached CWT of one signal with a user plugin (base.py:258-279 then 378-407)."""
    freqs = list(freqs)
    if len(freqs) < 2:
        raise IndexError('freqs needs at least two entries (base.py:272)')
    rows = [plugin_row(mode, trans_formula, formula, peak_freq, f, sfreq, x.shape[0] / sfreq, interpolate,
                       real_wave_length) for f in freqs]
    if interpolate:
        rows = [alias_mask(r) for r in rows]
    return cwt_from_rows(x, rows, interpolate), rows

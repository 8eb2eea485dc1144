"""Drop-in wavelet classes (reference wavelets.py).

Morse, Morlet and Shannon are *analytic* on the device: while a class keeps the
stock ``trans_formula`` its cache is the descriptor (kind, params) and the
kernels evaluate the spectrum; a subclass that overrides ``trans_formula`` is
treated as a plugin and its rows are evaluated on the host and uploaded as a
table.  MexicanHat and Haar are time-domain (WaveletMode.Normal) wavelets whose
spectrum is a host-built table (reference base.py:249-256).

The numpy ``trans_formula``/``formula`` methods are the public plugin API of the
reference (README.md:342-355); the cwt hot path does not call them for the
analytic classes.
"""
from __future__ import annotations

import numpy as np

from .base import WaveletBase, WaveletMode


class Morse(WaveletBase):
    """Generalised Morse wavelet: psi(x) = 2 H(x) x^b exp((b/r)(1 - x^r)), x = nu/f
    (wavelets.py:7-74)."""

    def __init__(self, sfreq: float = 1000, b: float = 17.5, r: float = 3,
                 real_wave_length: float = 1., interpolate: bool = False,
                 cuda: bool = False, **kw) -> None:
        super().__init__(sfreq, real_wave_length, interpolate, cuda, **kw)
        self.r: float = r
        self.b: float = b
        self.mode = WaveletMode.Reverse
        self.help = ('Generalised Morse wavelets are defined in the frequency domain; '
                     'the time-domain view is the inverse FFT of that spectrum.')

    def trans_formula(self, freqs: np.ndarray, freq: float = 1.) -> np.ndarray:
        x = freqs / freq
        step = np.heaviside(x, x)
        return 2. * (step * np.float_power(x, self.b)
                     * np.exp((self.b / self.r) * (1. - np.float_power(x, self.r))))

    def _analytic(self):
        if type(self).trans_formula is not Morse.trans_formula:
            return None
        return 'morse', [float(self.b), float(self.r)]


class Morlet(WaveletBase):
    """Morlet / Gabor wavelet (wavelets.py:77-144)."""

    def __init__(self, sfreq: float = 1000, sigma: float = 7.,
                 real_wave_length: float = 1., gabor: bool = False,
                 interpolate: bool = False, cuda: bool = False, **kw) -> None:
        super().__init__(sfreq, real_wave_length, interpolate, cuda, **kw)
        self.mode = WaveletMode.Both
        self.sigma = sigma
        self.gabor = gabor
        s2 = np.square(self.sigma)
        self.c = np.float_power(1 + np.exp(-s2) - 2 * np.exp(-3 / 4 * s2), -1 / 2)
        self.k = 0 if gabor else np.exp(-np.float_power(self.sigma, 2) / 2)

    def trans_formula(self, freqs: np.ndarray, freq: float = 1) -> np.ndarray:
        x = freqs / freq * self.peak_freq(freq)
        return (self.c * np.float_power(np.pi, -1 / 4)
                * (np.exp(-np.square(self.sigma - x) / 2) - self.k * np.exp(-np.square(x) / 2)))

    def formula(self, timeline: np.ndarray, freq: float = 1) -> np.ndarray:
        return (self.c * np.float_power(np.pi, -1 / 4) * np.exp(-np.square(timeline) / 2)
                * (np.exp(self.sigma * 1j * timeline) - self.k))

    def peak_freq(self, freq: float) -> float:
        return self.sigma / (1. - np.exp(-self.sigma * freq))

    def _time_formula_spec(self):
        if type(self).formula is not Morlet.formula or type(self).peak_freq is not Morlet.peak_freq:
            return None
        return 'morlet', [float(self.sigma), 1.0 if self.k == 0 else 0.0, float(self.c), float(self.k)]

    def _analytic(self):
        if (type(self).trans_formula is not Morlet.trans_formula
                or type(self).peak_freq is not Morlet.peak_freq):
            return None
        # c and k as the instance holds them (the kernels use these, not recomputed ones)
        return 'morlet', [float(self.sigma), 1.0 if self.k == 0 else 0.0, float(self.c), float(self.k)]


class Shannon(WaveletBase):
    """Shannon wavelet: 1 for nu <= 1 Hz, else 0; every scale identical because the
    reference ignores ``freq`` (wavelets.py:231-262)."""

    def __init__(self, sfreq: float = 1000, sigma: float = 7,
                 real_wave_length: float = 1., interpolate: bool = False,
                 cuda: bool = False, **kw) -> None:
        super().__init__(sfreq, real_wave_length, interpolate, cuda, **kw)
        self.sigma: float = sigma
        self.mode = WaveletMode.Reverse
        self.help = ''

    def trans_formula(self, tc: np.ndarray, freq: float = 1) -> np.ndarray:
        tc[...] = np.where(tc <= 1., 1., 0.)      # in place, as the reference's loop
        return tc

    def _analytic(self):
        if type(self).trans_formula is not Shannon.trans_formula:
            return None
        return 'shannon', []


class MexicanHat(WaveletBase):
    """Mexican-hat wavelet, time-domain formula -> FFT table (wavelets.py:194-228)."""

    def __init__(self, sfreq: float = 1000, sigma: float = 7,
                 real_wave_length: float = 1., interpolate: bool = False,
                 cuda: bool = False, **kw) -> None:
        super().__init__(sfreq, real_wave_length, interpolate, cuda, **kw)
        self.sigma: float = sigma
        self.mode = WaveletMode.Normal
        self.help = ''

    def formula(self, tc: np.ndarray, freq: float = 1) -> np.ndarray:
        return ((1 - np.power(tc / self.sigma, 2))
                * np.exp(-np.square(tc) / np.square(self.sigma) / 2))

    def cp_formula(self, tc: np.ndarray, freq: float = 1) -> np.ndarray:
        return self.formula(tc, freq)

    def peak_freq(self, freq: float) -> float:
        return np.sqrt(6) / np.pi / np.pi

    def _device_normal(self):
        cls = type(self)
        if cls.formula is MexicanHat.formula and cls.peak_freq is MexicanHat.peak_freq:
            return 'mexican_hat', [float(self.sigma), float(self.sfreq), float(self.real_wave_length)]
        return None

    def _time_formula_spec(self):
        spec = self._device_normal()
        return None if spec is None else ('mexican_hat', [float(self.sigma)])


class Haar(WaveletBase):
    """Haar wavelet, time-domain table path (wavelets.py:265-280)."""

    def __init__(self, sfreq: float = 1000, real_wave_length: float = 1.,
                 interpolate: bool = False, **kw) -> None:
        super().__init__(sfreq, real_wave_length, interpolate, **kw)
        self.mode = WaveletMode.Normal

    def formula(self, timeline: np.ndarray, freq: float = 1) -> np.ndarray:
        out = np.zeros_like(timeline)
        out[(timeline > 0.) & (timeline <= 1.)] = 1.
        out[(timeline > -1.) & (timeline <= 0.)] = -1.
        timeline[...] = out                      # in place, as the reference's loop
        return timeline

    def _device_normal(self):
        cls = type(self)
        if cls.formula is Haar.formula and cls.peak_freq is WaveletBase.peak_freq:
            return 'haar', [float(self.sfreq), float(self.real_wave_length)]
        return None

    def _time_formula_spec(self):
        return None if self._device_normal() is None else ('haar', [])


class MorseMNE(Morse):
    """Morse wavelets handed to mne's time-domain cwt (wavelets.py:147-191).

    Out of the hot path: kept only so the import surface matches; it needs mne,
    which this framework does not bundle."""

    def cwt(self, wave, freqs, use_fft: bool = True, mode: str = 'same', decim: float = 1):
        from mne.time_frequency import tfr     # ImportError without mne, as the reference
        return tfr.cwt(wave, list(self.make_wavelets(range(1, 100))),
                       use_fft=use_fft, mode=mode, decim=decim).mean(axis=0)

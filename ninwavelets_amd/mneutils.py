"""EpochsWavelet: CWT over the epochs of one channel (reference mneutils.py:9-71).

The reference maps ``wavelet.cwt`` over epochs in a Python loop (mneutils.py:39);
here all epochs go to the device in one batched call (``cwt_batch``) with the
same cache semantics: the wavelet table is built from the first epoch's length
unless the wavelet already holds one (``reuse=True``)."""
from __future__ import annotations

import numpy as np

from .base import WaveletBase


class EpochsWavelet:
    """Wavelet transform of mne-style epochs (anything with ``info['sfreq']``,
    ``ch_names`` and ``get_data() -> (epochs, channels, samples)``)."""

    def __init__(self, epochs, wavelet: WaveletBase) -> None:
        self.epochs = epochs
        self.wavelet = wavelet
        wavelet.sfreq = self.epochs.info['sfreq']           # mneutils.py:24

    def _waves(self, ch_name: str) -> np.ndarray:
        idx = self.epochs.ch_names.index(ch_name)
        return self.epochs.get_data()[:, idx, :]

    def cwt(self, ch_name: str, freqs) -> np.ndarray:
        """(epochs, F, N) complex (mneutils.py:26-40)."""
        return self.wavelet.cwt_batch(self._waves(ch_name), freqs, reuse=True)

    def power(self, ch_name: str, freqs) -> np.ndarray:
        """Epoch-mean of |cwt|^2, (F, N) (mneutils.py:42-55), reduced on the device:
        the (epochs, F, N) CWT is never materialised (fp64 sums in epoch order)."""
        return self.wavelet.cwt_batch(self._waves(ch_name), freqs, reuse=True, out='power_mean')

    def itc(self, ch_name: str, freqs) -> np.ndarray:
        """Inter-trial coherence |mean(cwt/|cwt|)|, (F, N) (mneutils.py:57-71), reduced
        on the device; a point where some epoch has |cwt| = 0 is NaN, as in the reference."""
        return self.wavelet.cwt_batch(self._waves(ch_name), freqs, reuse=True, out='itc')

"""ninwavelets_amd — MI355X-native drop-in for ninwavelets' FFT-domain CWT.

    from ninwavelets_amd import Morse
    power = Morse(1000, b=17.5, r=3).power(signal, range(1, 100))

Exports the reference's hot-path API (ninwavelets/__init__.py:1-3):
WaveletBase, WaveletMode, Morse, MorseMNE, Morlet, Haar, MexicanHat, Shannon,
EpochsWavelet, Baseline; plus the batched device engine (``Plan``,
``execute_multi``, ``execute_multi_device``).  Plotting is outside the accelerated
path and not provided.
"""
from .base import WaveletBase, WaveletMode, pad_to, interpolate_alias
from .wavelets import Morse, MorseMNE, Morlet, Haar, MexicanHat, Shannon
from .mneutils import EpochsWavelet
from .baseline import Baseline, baseline_of
from .engine import Plan, execute_multi, execute_multi_device
from . import _lib

__all__ = ['Baseline', 'baseline_of', 'WaveletBase', 'WaveletMode', 'Morse', 'MorseMNE', 'Morlet', 'Haar', 'MexicanHat',
           'Shannon', 'EpochsWavelet', 'Plan', 'execute_multi', 'execute_multi_device', 'pad_to', 'interpolate_alias']
__version__ = '0.1.0'

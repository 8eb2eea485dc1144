"""Baseline correction (reference base.py:18-68), computed on the GPU.

Same interface as the reference: ``Baseline(wave, sfreq, start, stop)`` slices
``wave[int(start*sfreq):int(stop*sfreq)]`` along AXIS 0 -- for an (F, N) CWT power
array that is a range of FREQUENCY rows (base.py:49), kept as is -- and its methods
``mean / ratio / percent / log / zscore / zlog`` return the corrected array.
basemean and std (one scalar each over the whole slice, np.std's population std)
are reduced on the device in fp64 (``nw_baseline``); the elementwise op runs in the
array's precision.  numpy arrays round-trip through the device; CUDA tensors stay
on it.  There is no CPU path: without a GPU every call raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


def baseline_of(wave, sfreq: float, start: float, stop: float):
    """The baseline slice itself (base.py:18-20): a view of ``wave``."""
    return wave[int(start * sfreq): int(stop * sfreq)]


def _rows(wave, sfreq, start, stop):
    """(row0, row1) of the axis-0 slice after Python's slice normalisation."""
    n0 = wave.shape[0] if len(wave.shape) else 0
    r0, r1, _ = slice(int(start * sfreq), int(stop * sfreq)).indices(n0)
    return r0, max(r0, r1)


class Baseline:
    """Baseline correction of one array (base.py:23-68) on the device."""

    def __init__(self, wave, sfreq: float, start: float, stop: float, device: int = 0) -> None:
        self.wave = wave
        self.baseline = baseline_of(wave, sfreq, start, stop)
        self.device = int(device)
        self._r0, self._r1 = _rows(wave, sfreq, start, stop)
        self._stats = None

    # -- device call -------------------------------------------------------------
    def _run(self, op: str):
        w = self.wave
        is_dev = hasattr(w, 'data_ptr') and getattr(w, 'is_cuda', False)
        if is_dev:
            import torch
            if w.dtype not in (torch.float32, torch.float64) or not w.is_contiguous():
                raise ValueError('Baseline on a device tensor needs a contiguous float32/float64 tensor')
            dt = L.NW_F32 if w.dtype == torch.float32 else L.NW_F64
            out = torch.empty_like(w)
            x_ptr, o_ptr, mem, dev = w.data_ptr(), out.data_ptr(), L.NW_MEM_DEVICE, w.device.index
            torch.cuda.synchronize(w.device)
        else:
            w = np.ascontiguousarray(w)
            if w.dtype not in (np.float32, np.float64):
                if np.iscomplexobj(w):
                    raise ValueError('Baseline is applied to real arrays (power / abs), got complex')
                w = w.astype(np.float64)
            dt = L.NW_F32 if w.dtype == np.float32 else L.NW_F64
            out = np.empty_like(w)
            x_ptr, o_ptr, mem, dev = w.ctypes.data, out.ctypes.data, L.NW_MEM_HOST, self.device
        count = int(np.prod(w.shape)) if len(w.shape) else 1
        row_len = max(1, count // w.shape[0]) if len(w.shape) and w.shape[0] else 1
        stats = (ctypes.c_double * 2)()
        L.check(L.lib().nw_baseline(dev, dt, ctypes.c_void_p(x_ptr), count, row_len, self._r0, self._r1,
                                    L.NW_BL[op], ctypes.c_void_p(o_ptr), mem, stats))
        self._stats = (stats[0], stats[1])
        return out

    @property
    def basemean(self):
        """baseline.mean() (base.py:51), reduced on the device."""
        if self._stats is None:
            self._run('mean')
        return self._stats[0]

    def mean(self):
        return self._run('mean')

    def ratio(self):
        return self._run('ratio')

    def percent(self):
        return self._run('percent')

    def log(self):
        return self._run('log')

    def zscore(self):
        return self._run('zscore')

    def zlog(self):
        return self._run('zlog')

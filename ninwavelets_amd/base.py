"""Drop-in ``WaveletBase`` / ``WaveletMode`` running the CWT on MI355X.

Mirrors the reference's L2 engine (base.py:126-443): same constructor
arguments, the same stateful, *unkeyed* wavelet cache (``reuse=True`` keeps the
first table whatever ``freqs`` or length later calls pass, base.py:394-397),
the same exceptions, the same pad/crop of the cached rows to the current
signal length and the same output dtypes (complex128 / float64 by default).

What changes is where the work runs.  The cache is a *descriptor*: for the
analytic wavelets (Morse, Morlet, Shannon) it is (kind, params, freqs, grid)
and the spectrum is evaluated inside the HIP kernels; for time-domain
(WaveletMode.Normal) wavelets and user plugins that override
``trans_formula``/``formula``, the host evaluates the rows once with the
plugin's own Python formula (the reference's plugin protocol, README.md:342-355)
and they are uploaded as a table.  fft -> multiply -> inverse fft -> |.|^2 run
in libninwave.so; there is no CPU compute path.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from enum import Enum
from functools import partial

import numpy as np
from scipy.fftpack import fft, ifft

from . import _lib as L
from .engine import REDUCTIONS, Plan, execute_multi, np_dtype
from .engine import make_wavelets as _make_wavelets_dev

# Device working-set budget per plan chunk (bytes); signals are streamed through it.
CHUNK_BYTES = int(os.environ.get('NINWAVE_CHUNK_BYTES', str(4 << 30)))
# Device bytes the plans cached by one wavelet object may hold together (nw_stats.device_bytes).
# Plans are keyed on (n, batch, device, ...): a session whose epoch lengths or batch sizes vary
# creates a plan per combination, so the least recently used ones are destroyed (their buffers
# freed) once the total exceeds this; the plans of the current call are always kept.
PLAN_CACHE_BYTES = int(os.environ.get('NINWAVE_PLAN_CACHE_BYTES', str(16 << 30)))


class WaveletMode(Enum):
    """Which spectrum source a wavelet uses (base.py:126-142)."""
    Normal = 0            # time-domain formula -> FFT table
    Both = 1              # analytic spectrum (time formula also available)
    Reverse = 2           # analytic spectrum only
    Indifferentiable = 3
    Twice = 4


def pad_to(wave_from: np.ndarray, wave_to: np.ndarray) -> np.ndarray:
    """Crop or centre-pad ``wave_from`` to ``wave_to.shape[0]`` (base.py:75-82)."""
    m, n = wave_from.shape[0], wave_to.shape[0]
    if m > n:
        return wave_from[:n]
    lo = (n - m) // 2
    return np.pad(wave_from, [lo, n - m - lo], 'constant')


def interpolate_alias(wave: np.ndarray, cuda: bool = False) -> np.ndarray:
    """Zero everything from bin int(len/2) up (base.py:107-123)."""
    keep = int(wave.shape[0] / 2)
    return np.pad(wave[:keep], [0, wave.shape[0] - keep], 'constant')


class _Cache:
    """The wavelet cache of one make_fft_wavelets call (base.py:258-279)."""

    _version = 0

    def __init__(self, kind, params, freqs, grid, table=None, row_len=None):
        _Cache._version += 1
        self.version = _Cache._version
        self.kind, self.params, self.freqs, self.grid, self.table = kind, params, freqs, grid, table
        if row_len is None and table is not None:
            row_len = np.full(table.shape[0], table.shape[1], dtype=np.int64)
        self.row_len = row_len


class WaveletBase:
    """Base class of the wavelets (base.py:145-443).

    Extra keyword arguments (not in the reference):
      dtype   -- compute dtype, 'float64' (default: the reference's arithmetic) or
                 'float32' (2x less HBM traffic; results within 1e-5 of max|ref|)
      device  -- HIP device index for single-device calls
      devices -- list of devices: batched calls shard signals over them
      engine  -- 'auto' (fused where supported), 'fused' or 'rocfft'
    ``cuda`` is accepted for compatibility; the GPU is always used.
    """

    def __init__(self, sfreq: float = 1000, real_wave_length: float = 1.,
                 interpolate: bool = True, cuda: bool = False, *, dtype='float64',
                 device: int = 0, devices=None, engine: str | None = None) -> None:
        self.mode: WaveletMode = WaveletMode.Normal
        self.sfreq: float = sfreq
        self.help: str = ''
        self.real_wave_length: float = real_wave_length
        self.interpolate = interpolate
        self.cuda = cuda
        self.dtype = np_dtype(dtype)
        self.device = device
        self.devices = list(devices) if devices else None
        self.engine = engine
        self._cache: _Cache | None = None
        self._rows = None
        self._plans: OrderedDict = OrderedDict()     # least recently used first
        self.plan_cache_bytes = PLAN_CACHE_BYTES

    # ------------------------------------------------------------------ plugin API
    def peak_freq(self, freq: float) -> float:
        return 1.

    def formula(self, timeline: np.ndarray, freq: float) -> np.ndarray:
        """Time-domain wavelet (override in plugins; base.py:281-302)."""
        return timeline

    def trans_formula(self, freqs: np.ndarray, freq: float = 1.) -> np.ndarray:
        """Frequency-domain wavelet (override in plugins; base.py:304-323)."""
        return freqs

    def cp_trans_formula(self, freqs: np.ndarray, freq: float = 1.) -> np.ndarray:
        """The reference's cupy twin (base.py:325-344); host arrays here."""
        return self.trans_formula(freqs, freq)

    def _analytic(self):
        """(kind, params) when the stock analytic spectrum applies, else None."""
        return None

    def _device_normal(self):
        """(kind, params) when the stock time-domain formula applies (the table is then
        built on the device), else None (plugin formulas: host-built table)."""
        return None

    # ------------------------------------------------------------------ grids
    def _setup_trans_shape(self, freq: float, real_wave_length: float,
                           cuda: bool = False) -> np.ndarray:
        """Frequency grid (base.py:173-194)."""
        return np.arange(0, self.sfreq / freq * real_wave_length, 1 / freq)

    def _setup_waveletshape(self, freq: float, real_length: float = 1,
                            zero_mean: bool = False) -> np.ndarray:
        """Time grid of the time-domain wavelet (base.py:196-216)."""
        p = self.peak_freq(freq)
        span = real_length / p * freq * 2 * np.pi
        step = 1 / self.sfreq * 2 * np.pi * freq / p
        return np.arange(-span / 2, span / 2, step) if zero_mean else np.arange(0, span, step)

    # ------------------------------------------------------------------ wavelets
    def _time_formula_spec(self):
        """(kind, params) when the stock time-domain formula applies (override)."""
        return None

    def _device_wavelet_spec(self):
        """(kind, params) of nw_make_wavelets for this wavelet, None for plugin formulas."""
        if self.mode in (WaveletMode.Reverse, WaveletMode.Twice):
            a = self._analytic()
            return a if a is not None and a[0] in ('morse', 'shannon') else None
        return self._time_formula_spec()

    def _device_wavelets(self, spec, freqs) -> list:
        kind, params = spec
        rows = _make_wavelets_dev(kind, params, freqs, self.sfreq, self.real_wave_length, self.device)
        return [r.real.copy() for r in rows] if kind in ('mexican_hat', 'haar') else rows

    def make_wavelet(self, freq: float) -> np.ndarray:
        """Time-domain wavelet (base.py:346-359): on the device for the stock wavelets."""
        if freq == 0:
            raise ZeroDivisionError
        spec = self._device_wavelet_spec()
        if spec is not None:
            return self._device_wavelets(spec, [freq])[0]
        if self.mode in (WaveletMode.Reverse, WaveletMode.Twice):
            w = ifft(self.trans_formula(self._setup_trans_shape(freq, self.real_wave_length)))
            half = int(w.shape[0])
            both = np.hstack((np.conj(np.flip(w)), w))
            return both[half // 2: half // 2 * 3]
        return self.formula(self._setup_waveletshape(freq, 1, zero_mean=True), freq)

    def make_wavelets(self, freqs) -> list:
        """List of time-domain wavelets (base.py:361-376): one device call for the stock
        wavelets (nw_make_wavelets), the plugin's own formula otherwise."""
        spec = self._device_wavelet_spec()
        if spec is not None:
            fr = list(freqs)
            if any(f == 0 for f in fr):
                raise ZeroDivisionError
            self.wavelets = self._device_wavelets(spec, fr)
        else:
            self.wavelets = [self.make_wavelet(f) for f in freqs]
        return self.wavelets

    def _normal_row(self, freq: float) -> np.ndarray:
        """Spectrum of the zero-padded time-domain wavelet, |Re|+i|Im| (base.py:249-256)."""
        w = self.make_wavelet(freq)
        half = int((self.sfreq * self.real_wave_length - w.shape[0]) / 2)
        spec = fft(np.hstack((np.zeros(half), w, np.zeros(half))))
        return np.abs(spec.real) + 1j * np.abs(spec.imag)

    def make_fft_wavelet(self, freq: float, real_length: float = 1.) -> np.ndarray:
        """One cached row, host-evaluated (base.py:221-256).  cwt() does not use
        this: it evaluates the analytic rows on the device."""
        if freq == 0:
            raise ZeroDivisionError
        if self.mode in (WaveletMode.Reverse, WaveletMode.Both):
            rl = real_length / 2 if self.interpolate else real_length
            t = self._setup_trans_shape(real_length, rl)
            row = self.trans_formula(t, freq)
            return np.hstack((row, np.zeros(len(t)))) if self.interpolate else row
        return self._normal_row(freq)

    def _build_cache(self, freqs, real_length: float) -> _Cache:
        self.freq_dist = freqs[1] - freqs[0]          # IndexError / TypeError as base.py:272
        fr = np.asarray(list(freqs), dtype=np.float64)
        spectral = self.mode in (WaveletMode.Reverse, WaveletMode.Both)
        analytic = self._analytic() if spectral else None
        if analytic is not None:
            if np.any(fr == 0):
                raise ZeroDivisionError
            kind, params = analytic
            cache = _Cache(kind, params, fr, L.trans_grid(real_length, self.sfreq, self.interpolate))
        elif not spectral and self._device_normal() is not None:
            if np.any(fr == 0):
                raise ZeroDivisionError                  # make_wavelet, base.py:234-235
            kind, params = self._device_normal()
            cache = _Cache(kind, params, fr, L.nw_grid(1.0, 0, 0))
        else:
            rows = [self.make_fft_wavelet(f, real_length) for f in fr]
            if self.interpolate:
                rows = [interpolate_alias(r) for r in rows]
            cache = self._table_cache(rows, fr)
        self._cache = cache
        self._rows = None
        return cache

    @staticmethod
    def _table_cache(rows, freqs) -> _Cache:
        rows = [np.asarray(r) for r in rows]
        lens = np.array([r.shape[0] for r in rows], dtype=np.int64)
        m = int(lens.max()) if len(rows) else 0
        table = np.zeros((len(rows), m), dtype=np.complex128)   # rows left-aligned
        for i, r in enumerate(rows):
            table[i, :r.shape[0]] = r
        grid = L.nw_grid(1.0, m, m)
        return _Cache('table', [], freqs, grid, table, lens)

    def make_fft_wavelets(self, freqs, real_wave_length: float = 1.) -> list:
        """Build (and return) the cached rows (base.py:258-279)."""
        self._build_cache(freqs, real_wave_length)
        return self.fft_wavelets

    @property
    def fft_wavelets(self) -> list:
        """The cached rows as the reference stores them (evaluated on the device
        for the analytic kinds)."""
        c = self._cache
        if c is None:
            raise AttributeError('fft_wavelets')
        if self._rows is None:
            if c.kind == 'table':
                self._rows = [row[:n] for row, n in zip(c.table, c.row_len)]
            else:
                plan = Plan(max(1, c.grid.len_full), len(c.freqs), 'float64', self.device,
                            interpolate=self.interpolate)   # Normal tables apply the alias mask
                plan.set_wavelet(c.kind, c.params, c.freqs, c.grid)
                rows = plan.rows()
                lens = getattr(plan, 'row_len', None)
                plan.close()
                self._rows = ([row[:n] for row, n in zip(rows, lens)] if lens is not None
                              else [row for row in rows])
        return self._rows

    @fft_wavelets.setter
    def fft_wavelets(self, rows) -> None:
        freqs = self._cache.freqs if self._cache is not None else np.arange(len(rows), dtype=np.float64)
        self._cache = self._table_cache(list(rows), freqs)
        self._rows = None

    @fft_wavelets.deleter
    def fft_wavelets(self) -> None:
        self._cache = None
        self._rows = None

    # ------------------------------------------------------------------ execution
    def _plan(self, n: int, nsig: int, device: int, scales: tuple[int, int] | None = None,
              slot: int = 0) -> Plan:
        """The cached plan for (n, batch, device) -- of the scale slice [f0, f1) when
        ``scales`` is given (scale-sharded multi-device calls).  ``slot`` is the shard
        index of a multi-device call: a plan is not reentrant, so ``devices=[0, 0]`` gets
        one plan per shard, never one plan driven from two host threads."""
        c = self._cache
        f0, f1 = scales if scales is not None else (0, len(c.freqs))
        nf = f1 - f0
        esz = self.dtype.itemsize
        per_sig = nf * n * esz * 5 + n * esz * 3
        cap = max(1, CHUNK_BYTES // per_sig)
        batch = 1
        while batch < min(nsig, cap):
            batch *= 2
        batch = min(batch, cap)
        key = (n, nf, self.dtype.str, bool(self.interpolate), device, batch, self.engine, f0, slot)
        plan = self._plans.get(key)
        if plan is None:
            plan = Plan(n, nf, self.dtype, device, batch, self.interpolate, self.engine)
            self._plans[key] = plan
        self._plans.move_to_end(key)
        if plan.wavelet_token != c.version:
            sl = slice(f0, f1)
            plan.set_wavelet(c.kind, c.params, c.freqs[sl], c.grid,
                             None if c.table is None else c.table[sl], token=c.version,
                             row_len=None if c.row_len is None else c.row_len[sl])
        return plan

    def plan_cache_device_bytes(self) -> int:
        """Device bytes held by the cached plans (sum of nw_stats.device_bytes)."""
        return sum(p.stats()['device_bytes'] for p in self._plans.values())

    def _evict_plans(self, keep: int) -> None:
        """Destroy least-recently-used plans (freeing their device buffers) while the cache
        holds more than ``plan_cache_bytes``; the ``keep`` most recent (this call's) stay."""
        sizes = {k: p.stats()['device_bytes'] for k, p in self._plans.items()}
        total = sum(sizes.values())
        while total > self.plan_cache_bytes and len(self._plans) > keep:
            k, p = self._plans.popitem(last=False)
            total -= sizes[k]
            p.close()

    def _run(self, x: np.ndarray, out_kind: str) -> np.ndarray:
        """x: (..., n) signals -> (..., F, n) on the device(s); the plan cache is trimmed
        to ``plan_cache_bytes`` after the call (its buffers grow during the call)."""
        self._used = 1
        try:
            return self._run_plans(x, out_kind)
        finally:
            if len(self._plans) > 1:
                self._evict_plans(keep=max(1, self._used))

    def _run_plans(self, x: np.ndarray, out_kind: str) -> np.ndarray:
        """Several devices shard the signals, or -- with fewer signals than devices (one
        long signal) -- the scales."""
        n = x.shape[-1]
        nsig = int(np.prod(x.shape[:-1])) if x.ndim > 1 else 1
        devs = self.devices or [self.device]
        nf = len(self._cache.freqs)
        if len(devs) > 1 and nsig < len(devs) and nf >= len(devs):
            from .dist import shard
            plans = [self._plan(n, nsig, d, shard(nf, i, len(devs)), slot=i) for i, d in enumerate(devs)]
            self._used = len(plans)
            out = execute_multi(plans, x.reshape(nsig, n), out_kind, shard='scales')
            if out_kind in REDUCTIONS:
                return out
            return out.reshape(x.shape[:-1] + out.shape[-2:])
        if len(devs) > 1 and nsig > 1:
            per = -(-nsig // len(devs))          # the largest balanced block (dist.shard)
            plans = [self._plan(n, per, d, slot=i) for i, d in enumerate(devs)]
            self._used = len(plans)
            out = execute_multi(plans, x.reshape(nsig, n), out_kind)
            if out_kind in REDUCTIONS:
                return out
            return out.reshape(x.shape[:-1] + out.shape[-2:])
        self._used = 1
        return self._plan(n, nsig, devs[0]).execute(x, out_kind=out_kind)

    def _broadcast_quirk(self, wave: np.ndarray, out_kind: str) -> np.ndarray:
        """2-D (1, N) input: the reference pads the rows to wave.shape[0] = 1 and
        broadcasts that single bin over fft(wave, axis=-1) (base.py:396-406)."""
        n = wave.shape[1]
        c = self._cache
        nf = len(c.freqs)
        odt = np.complex128 if self.dtype == np.float64 else np.complex64
        if self.interpolate:
            # interpolate_alias on a (1, N) spectrum pads BOTH axes by [0, 1] with zeros
            out = np.zeros((nf, n + 1), dtype=odt)
            return out if out_kind == 'cwt' else np.abs(out) ** (2 if out_kind == 'power' else 1)
        first = np.array([pad_to(np.asarray(r), np.zeros(1))[0] for r in self.fft_wavelets],
                         dtype=np.complex128)
        table = np.repeat(first[:, None], n, axis=1)
        saved = self._cache
        self._cache = _Cache('table', [], c.freqs, L.nw_grid(1.0, n, n), table)
        try:
            return self._run(np.ascontiguousarray(wave[0]), out_kind)
        finally:
            self._cache = saved

    def _transform(self, wave, freqs, reuse: bool, out_kind: str) -> np.ndarray:
        wave = np.asarray(wave)
        if (not reuse) or self._cache is None:
            self._build_cache(freqs, wave.shape[0] / self.sfreq)
        if wave.ndim == 1:
            return self._run(wave, out_kind)
        if wave.ndim == 2 and wave.shape[0] == 1:
            return self._broadcast_quirk(wave, out_kind)
        raise ValueError(f'cwt takes one 1-D signal (or the (1, N) form); got shape {wave.shape}. '
                         'Use cwt_batch for batches of signals.')

    def cwt(self, wave: np.ndarray, freqs, reuse: bool = True) -> np.ndarray:
        """Complex CWT (F, N) of one signal (base.py:378-407)."""
        return self._transform(wave, freqs, reuse, 'cwt')

    def power(self, wave: np.ndarray, freqs=None, reuse: bool = True) -> np.ndarray:
        """|cwt|^2 (base.py:409-425), fused on the device."""
        return self._transform(wave, freqs, reuse, 'power')

    def abs(self, wave: np.ndarray, freqs=None, reuse: bool = True) -> np.ndarray:
        """|cwt| (base.py:427-443), fused on the device."""
        return self._transform(wave, freqs, reuse, 'abs')

    def cwt_batch(self, waves: np.ndarray, freqs=None, reuse: bool = True,
                  out: str = 'cwt') -> np.ndarray:
        """Batched CWT of (..., N) signals -> (..., F, N) in one device call, or (F, N)
        for the reductions over all signals: ``power_mean``, ``itc`` (the compute
        dtype), ``power_sum`` (float64) and ``phase_sum`` (complex128).

        Equivalent to stacking ``cwt(w, freqs, reuse)`` over the leading axes
        (the per-epoch loop of mneutils.py:39): the cache is built from the
        first call's length if absent, then shared by every signal."""
        waves = np.asarray(waves)
        if waves.ndim < 1:
            raise ValueError('waves must have a trailing sample axis')
        if (not reuse) or self._cache is None:
            self._build_cache(freqs, waves.shape[-1] / self.sfreq)
        if out not in ('cwt', 'abs', 'power') + REDUCTIONS:
            raise ValueError(f"out must be one of cwt, abs, power, {', '.join(REDUCTIONS)}; got {out!r}")
        return self._run(waves, out)

    def plan_stats(self) -> list:
        """Per-plan device stage timings (nw_plan_stats)."""
        return [p.stats() for p in self._plans.values()]

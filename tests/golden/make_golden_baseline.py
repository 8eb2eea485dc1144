"""Golden vectors for the reference's Baseline correction (base.py:18-68), made by running
the REFERENCE itself (build container only; see make_golden.py for the loader).

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden_baseline.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import load_reference, save  # noqa: E402

OPS = ['mean', 'ratio', 'percent', 'log', 'zscore', 'zlog']


def main():
    nw = load_reference()
    from ninwavelets.base import Baseline, baseline_of
    rng = np.random.default_rng(7)
    t = np.arange(500) / 1000.
    x = np.sin(2 * np.pi * 11 * t) + 0.3 * np.sin(2 * np.pi * 37 * t) + 0.1 * rng.standard_normal(500)
    power = nw.Morse(1000).power(x, range(1, 40))          # (39, 500) float64
    cases = {
        # (F, N) power: the slice is along axis 0 = FREQUENCY rows 5..19 (base.py:49)
        'baseline_power': (power, 100., 0.05, 0.2),
        # one positive 1-D wave: the slice is along time
        'baseline_1d': (np.abs(x) + 0.5, 1000., 0.1, 0.3),
        # float32 data keeps float32 statistics and outputs
        'baseline_power_f32': (power.astype(np.float32), 100., 0.05, 0.2),
    }
    for name, (wave, sfreq, start, stop) in cases.items():
        b = Baseline(wave, sfreq, start, stop)
        outs = {op: np.asarray(getattr(b, op)()) for op in OPS}
        save(name, dict(sfreq=sfreq, start=start, stop=stop, dtype=str(wave.dtype), op='baseline'),
             wave=wave, baseline=np.asarray(baseline_of(wave, sfreq, start, stop)),
             basemean=np.asarray(b.basemean), std=np.asarray(np.std(b.baseline)), **outs)


if __name__ == '__main__':
    main()

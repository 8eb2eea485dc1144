"""Golden vectors for the reference's time-domain wavelets (make_wavelet(s), base.py:346-376),
made by running the REFERENCE itself (build container only; loader: make_golden.py).

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden_wavelets.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import load_reference, save  # noqa: E402

FREQS = [0.75, 2., 7.5, 30., 101.]


def main():
    nw = load_reference()
    cases = {
        'morse': nw.Morse(1000), 'morse_b': nw.Morse(500, b=10., r=2.), 'shannon': nw.Shannon(1000),
        'morlet': nw.Morlet(1000), 'morlet_gabor': nw.Morlet(1000, gabor=True),
        'mexican_hat': nw.MexicanHat(1000), 'haar': nw.Haar(1000),
    }
    for name, w in cases.items():
        rows = [np.asarray(r) for r in w.make_wavelets(FREQS)]
        lens = np.array([r.shape[0] for r in rows], dtype=np.int64)
        flat = np.concatenate([r.astype(np.complex128) for r in rows])
        save(f'wavelets_{name}', dict(case=name, sfreq=float(w.sfreq), dtype=str(rows[0].dtype), op='wavelets'),
             freqs=np.array(FREQS), lens=lens, rows=flat)


if __name__ == '__main__':
    main()

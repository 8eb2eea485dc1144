"""Golden vectors at the BENCHMARK lengths, made by running the REFERENCE itself.

The other fixtures stop at N = 4096; the benchmark configs run N = 16384 (C2 Morlet
sigma = 7, C4 Morse) and C5 runs 2^24.  This script runs the reference's
``cwt`` (base.py:378-407, with the Morse / Morlet spectra of wavelets.py:65-74,
132-136) at N = 16384, 2^17 and 2^24 in this container and stores, per case:

- the input as a seed: x = sin(2 pi f1 t) + 0.5 sin(2 pi f2 t + 1) + 0.1 N(0, 1) from
  ``np.random.default_rng(seed)`` (PCG64, stream-stable), plus sha256 of x's bytes so a
  test knows it regenerated the same signal;
- the reference output at 2048 fixed sample positions per scale (every scale's row),
  complex128;
- per scale: sum(out) and sum(|out|^2) over the WHOLE row (size-independent checks of
  every output point).

Sampling keeps the fixtures small (the full C4-length rows would be 0.8 MB per case).

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden_long.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
from make_golden import load_reference, save  # noqa: E402
from conftest import long_signal, x_digest  # noqa: E402  (the tests rebuild x the same way)

NSAMP = 2048

# (name, kind, n, freqs, seed)
LONG_CASES = [
    ('long_c2_morlet_n16384', 'morlet', 16384, [1., 64., 128.], 16384 + 2),
    ('long_c4_morse_n16384', 'morse', 16384, [1., 128., 256.], 16384 + 4),
    ('long_morse_n131072', 'morse', 1 << 17, [0.5, 40., 250.], (1 << 17) + 5),
    # C5: three of its 512 scales (linspace(0.5, 250, 512)[[0, 200, 511]])
    ('long_c5_morse_n16777216', 'morse', 1 << 24, list(np.linspace(0.5, 250, 512)[[0, 200, 511]]),
     (1 << 24) + 5),
]


def sample_positions(n: int, seed: int) -> np.ndarray:
    """NSAMP sorted sample positions: both ends, the centre, and random interior points."""
    rng = np.random.default_rng(seed + 1)
    fixed = np.array([0, 1, n // 2 - 1, n // 2, n // 2 + 1, n - 2, n - 1])
    pos = np.unique(np.concatenate([fixed, rng.choice(n, NSAMP, replace=False)]))
    return pos[:NSAMP] if pos.size > NSAMP else pos


def main():
    nw = load_reference()
    for name, kind, n, freqs, seed in LONG_CASES:
        x = long_signal(n, seed)
        w = nw.Morse(1000.) if kind == 'morse' else nw.Morlet(1000., sigma=7.)
        out = w.cwt(x, freqs, reuse=False)                 # (F, n) complex128
        pos = sample_positions(n, seed)
        meta = dict(kind=kind, n=n, sfreq=1000., interpolate=False, params={}, dtype='float64',
                    op='cwt_sampled', seed=seed, x_sha256=x_digest(x))
        save(name, meta, freqs=np.asarray(freqs, dtype=np.float64), pos=pos.astype(np.int64),
             out_at=np.ascontiguousarray(out[:, pos]), row_sum=out.sum(axis=1),
             row_energy=(np.abs(out) ** 2).sum(axis=1))


if __name__ == '__main__':
    main()

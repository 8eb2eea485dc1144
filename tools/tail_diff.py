"""The tail-threshold W support against the exact support, on the same inputs (VERDICT r05
weak #1): every output of the product library (rows cut at the last bin above 2^-72 / 2^-56 of
the row's max |W|, nw_internal.h kTailRel) against a build with -DNW_TAIL_EXACT (rows cut at
their last nonzero bin).  Cases: the C4 / C3 / C5 shapes with broadband noise, and noise-free
bin-centred tones placed in the pruned tails of C4 rows (no signal energy in those rows' main
lobes, so the cut bins carry the rows' whole signal).  Prints one line per case: the largest
|product - exact| relative to the signal's own max |y| over all rows, and the worst single row
relative to that row's own max.

    make -C ninwavelets_amd/csrc VARIANT=tailexact DEFS=-DNW_TAIL_EXACT
    python tools/tail_diff.py            # runs both libraries in child processes, compares
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cases():
    rng = np.random.default_rng(3)
    c4f = np.arange(1, 257, dtype=float)
    out = []
    for n, fr, dt, S in [(16384, c4f, 'float64', 4), (16384, c4f, 'float32', 4), (4096, c4f, 'float32', 4),
                         (1 << 20, np.linspace(0.5, 250, 64), 'float64', 1),
                         (1 << 20, np.linspace(0.5, 250, 64), 'float32', 1)]:
        t = np.arange(n) / 1000.
        x = np.sin(2 * np.pi * rng.uniform(1, 100, (S, 1)) * t) + 0.1 * rng.standard_normal((S, n))
        out.append((f'noise n={n} {dt}', n, fr, dt, x.astype(dt)))
    # tones at whole cycles per window (bin-centred: no leakage into the main lobes) at 2.5 x and
    # 4 x the peak of C4 rows f = 8, 40, 100: inside the pruned tail in both dtypes (the fp64 cut
    # sits at ~2.29 f, the fp32 one at ~2.15 f)
    n = 16384
    t = np.arange(n) / 1000.
    for dt in ('float64', 'float32'):
        sig = []
        for f in (8., 40., 100.):
            for mult in (2.5, 4.0):
                k = round(mult * f * n / 1000.)
                sig.append(np.cos(2 * np.pi * k * np.arange(n) / n))
        out.append((f'tail tones n={n} {dt}', n, c4f, dt, np.array(sig).astype(dt)))
    return out


def run(tag, outdir):
    sys.path.insert(0, ROOT)
    import ninwavelets_amd as nw
    from ninwavelets_amd import _lib as L
    for i, (name, n, fr, dt, x) in enumerate(cases()):
        p = nw.Plan(n, fr.size, dt, max_batch=x.shape[0])
        p.set_wavelet('morse', [17.5, 3.0], fr, L.trans_grid(n / 1000., 1000., False))
        np.save(os.path.join(outdir, f'{tag}_{i}.npy'), p.execute(x, out_kind='cwt'))
        p.close()


def main():
    if len(sys.argv) > 2:                      # child: python tail_diff.py run <tag> <outdir>
        run(sys.argv[2], sys.argv[3])
        return
    exact = os.path.join(ROOT, 'ninwavelets_amd', 'libninwave_tailexact.so')
    if not os.path.exists(exact):
        raise SystemExit('build the exact-support library first: '
                         'make -C ninwavelets_amd/csrc VARIANT=tailexact DEFS=-DNW_TAIL_EXACT')
    with tempfile.TemporaryDirectory(dir=os.path.join(ROOT, 'gpurun_out') if os.path.isdir(
            os.path.join(ROOT, 'gpurun_out')) else None) as td:
        for tag, lib in (('tail', os.path.join(ROOT, 'ninwavelets_amd', 'libninwave.so')), ('exact', exact)):
            env = dict(os.environ, NINWAVE_LIB=lib, PYTHONDONTWRITEBYTECODE='1')
            subprocess.run([sys.executable, os.path.abspath(__file__), 'run', tag, td], env=env, check=True)
        for i, (name, n, fr, dt, x) in enumerate(cases()):
            a = np.load(os.path.join(td, f'tail_{i}.npy')).astype(np.complex128)
            b = np.load(os.path.join(td, f'exact_{i}.npy')).astype(np.complex128)
            d = np.abs(a - b)
            mag = np.abs(b)
            sig = max(float(d[s].max() / mag[s].max()) for s in range(x.shape[0]))
            rowmax = mag.max(-1)
            row = float(np.max(np.where(rowmax > 0, d.max(-1) / np.where(rowmax > 0, rowmax, 1), 0)))
            # rows whose output the cut set to exactly zero, and how large the exact build's were
            zero = (np.abs(a).max(-1) == 0) & (rowmax > 0)
            print(json.dumps({'case': name, 'identical': bool(d.max() == 0),
                              'max_diff_over_signal_max': sig, 'worst_row_diff_over_row_max': row,
                              'rows_zeroed_by_cut': int(zero.sum()),
                              'largest_zeroed_row_max_over_signal_max':
                                  float(max((rowmax[s][zero[s]].max() / mag[s].max()) if zero[s].any() else 0.0
                                            for s in range(x.shape[0])))}), flush=True)


if __name__ == '__main__':
    main()

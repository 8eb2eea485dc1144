"""The W-row support the engines prune to, and what that cut does to the outputs.

Round 5 cut every W row at its last bin above kTailRel x the row's max |W| (2^-72 fp64, 2^-56
fp32; nw_internal.h).  Round 6 builds the two-pass engine's cut (kmax, nw_large.hip) without a
full scan for Morse / Morlet / Shannon rows (support_fast_kernel: a window around the analytic
peak, then a bisection of the falling side).  Here:
  * that support equals the full scan's, row for row, for all 512 C5 scales (fp32 and fp64),
    Morse b in {0.5, 3, 20, 63.5, 64, 100}, Morlet (both forms), Shannon, interpolate and a
    centre-padded cached row (off > 0);
  * the per-row contract (INTEGRATION.md "Contract details"): a row whose main lobe sees no
    signal energy -- noise-free, bin-centred tones at 2.5 x and 4 x the row's peak frequency,
    inside the pruned tail -- still matches the reference's cwt within the dtype's tolerance of
    the signal's own scale (max |x|): the bins the cut drops carry |W| < 2^-72 (2^-56) of the
    row's peak, so they move such a row by less than n x that of max |x|.
"""
import numpy as np
import pytest

from oracle import nw_oracle as O

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402

C5_FREQS = np.linspace(0.5, 250, 512)


def plan_for(n, freqs, dtype, kind, params, interpolate=False, real_length=None):
    p = nw.Plan(n, freqs.size, dtype, interpolate=interpolate)
    rl = (n / 1000.) if real_length is None else real_length
    p.set_wavelet(kind, params, freqs, L.trans_grid(rl, 1000., interpolate))
    return p


def check_support(p):
    fast, scan = p.row_support(), p.row_support(scan=True)
    bad = np.nonzero(fast != scan)[0]
    assert bad.size == 0, f'rows {bad[:8]}: fast {fast[bad[:8]]} scan {scan[bad[:8]]}'
    return fast


@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_c5_support_equals_the_scan(dtype):
    """All 512 C5 rows (1 x 2^24, Morse b = 17.5, r = 3, freqs linspace(0.5, 250, 512))."""
    p = plan_for(1 << 24, C5_FREQS, dtype, 'morse', [17.5, 3.0])
    try:
        k = check_support(p)
        # the cut sits past the peak (nu = f) and below the row's end: a real cut, not the row
        delta = 1000. / (1 << 24)
        assert np.all(k * delta > C5_FREQS) and np.all(k < (1 << 24) - 1)
    finally:
        p.close()


@pytest.mark.parametrize('b', [0.5, 3.0, 20.0, 63.5, 64.0, 100.0])
@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_morse_b_support_equals_the_scan(b, dtype):
    """Morse b across the multiply-chain (2b integer) and log-domain row forms, including
    b = 100, whose small-f rows overflow the reference's x^b (the scan keeps those)."""
    freqs = np.concatenate([[0.3, 0.8], np.geomspace(1.0, 480.0, 30)])
    p = plan_for(1 << 20, freqs, dtype, 'morse', [b, 3.0])
    try:
        check_support(p)
    finally:
        p.close()


@pytest.mark.parametrize('kind,params', [('morlet', [7.0, 0.0]), ('morlet', [7.0, 1.0]), ('morlet', [2.0, 0.0]),
                                         ('shannon', [])])
@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_other_kinds_support_equals_the_scan(kind, params, dtype):
    freqs = np.geomspace(0.5, 450.0, 40)
    p = plan_for(1 << 18, freqs, dtype, kind, params)
    try:
        check_support(p)
    finally:
        p.close()


@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_support_interpolate_and_padded_rows(dtype):
    """interpolate (bins >= n/2 masked) and a cached row shorter than n (centre-padded:
    the row starts at off = (n - len_full) // 2, base.py:75-82)."""
    freqs = np.geomspace(0.5, 450.0, 24)
    for kw in ({'interpolate': True}, {'real_length': (1 << 19) / 1000.}, {'real_length': 300.0}):
        p = plan_for(1 << 20, freqs, dtype, 'morse', [17.5, 3.0], **kw)
        try:
            check_support(p)
        finally:
            p.close()


TONE_ROWS = (8.0, 40.0, 100.0)


def tail_tones(n, sfreq=1000.):
    """cos tones at whole cycles per window (no leakage) at 2.5 x and 4 x each row's peak."""
    out = []
    for f in TONE_ROWS:
        for mult in (2.5, 4.0):
            k = round(mult * f * n / sfreq)
            out.append(np.cos(2 * np.pi * k * np.arange(n) / n))
    return np.array(out)


@pytest.mark.parametrize('dtype,tol', [('float64', 1e-12), ('float32', 1e-5)])
@pytest.mark.parametrize('n', [16384, 1 << 18])
def test_tail_tones_against_the_reference(dtype, tol, n):
    """The per-row contract where the cut matters most: the whole of the signal sits in the
    rows' pruned tails.  One-pass engine (n = 16384, the C4 length) and two-pass (2^18)."""
    x = tail_tones(n)
    freqs = np.array(TONE_ROWS)
    w = nw.Morse(1000, dtype=dtype)
    got = w.cwt_batch(x, freqs).astype(np.complex128)
    for s in range(x.shape[0]):
        ref = O.cwt('morse', x[s], freqs)
        scale = np.max(np.abs(x[s]))
        err = np.max(np.abs(got[s] - ref), axis=-1)       # per row
        assert np.all(err <= tol * scale), (s, err / scale)
        # the row the tone was placed beyond: in exact arithmetic the reference's output there is
        # |W_f(nu_tone)| / 2 (a bin-centred cos), far below the tolerance -- what the reference
        # prints for that row is its own FFT rounding (6e-12 of max |x| at 2^18 in fp64)
        r = s // 2
        nu = np.array([round((2.5 if s % 2 == 0 else 4.0) * TONE_ROWS[r] * n / 1000.) * 1000. / n])
        assert 0.5 * abs(O.morse_spectrum(nu, TONE_ROWS[r])[0]) <= 1e-3 * tol * scale

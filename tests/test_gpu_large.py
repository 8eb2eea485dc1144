"""GPU parity of the two-pass fused engine for long signals (nw_large.hip: fp32 and fp64,
power-of-two 2^15 <= n <= 2^24) against the fp64 CPU oracle and the rocFFT engine.

Tolerance (fp32 compute vs the fp64 oracle): max|out - ref| <= 1e-5 * max|ref|
up to n = 2^16 and 3e-5 above (fp32 FFT round-off grows with log n; the C5 case at 2^24
keeps 1e-4 in test_gpu_parity.py); |.|^2 outputs twice that.  fp64 compute: 1e-12 (as every
fp64 parity test), |.|^2 2e-12.
"""
import numpy as np
import pytest

from oracle import nw_oracle as O

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402

CLASSES = {'morse': nw.Morse, 'morlet': nw.Morlet, 'shannon': nw.Shannon, 'mexican_hat': nw.MexicanHat}


def rel_err(got, ref):
    return np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-300)


def tol(n):
    return 1e-5 if n <= (1 << 16) else 3e-5


def synth(S, n, seed, sfreq=1000.):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sfreq
    fc = rng.uniform(1, 100, (S, 1))
    ph = rng.uniform(0, 2 * np.pi, (S, 1))
    return (np.sin(2 * np.pi * fc * t + ph) + 0.1 * rng.standard_normal((S, n))).astype(np.float32)


def large_ran(w):
    st = w.plan_stats()
    return any(s['engine'] == 'fused' and s['launches_rows'] > 0 for s in st)


@pytest.mark.parametrize('n', [1 << 15, 1 << 16, 1 << 17, 1 << 18, 1 << 19, 1 << 20, 1 << 21])
@pytest.mark.parametrize('kind', ['morse', 'morlet', 'shannon'])
def test_large_cwt_against_oracle(kind, n):
    """Every N1 x N2 split (N1 = 32 with N2 = 1024 .. 16384, then N2 = 16384 with N1 = 64 ..
    128) for the analytic kinds; scales from below the bin spacing's reach to 400 Hz."""
    x = synth(1, n, seed=n % 1000 + len(kind))[0]
    freqs = np.array([0.5, 3.0, 17.0, 60.0, 250.0, 400.0])
    w = CLASSES[kind](1000, dtype='float32')
    got = w.cwt(x, freqs)
    assert large_ran(w)
    ref = O.cwt(kind, x.astype(np.float64), freqs)
    assert got.shape == (freqs.size, n) and got.dtype == np.complex64
    assert rel_err(got, ref) <= tol(n), rel_err(got, ref)


@pytest.mark.parametrize('n', [1 << 16, 1 << 22])
def test_large_power_abs_and_batch(n):
    """|.|^2 and |.| from the column pass's epilogue, a batch of signals (one Xt per
    signal), and the batch equal to the per-signal call."""
    S = 3 if n <= (1 << 16) else 2
    x = synth(S, n, seed=7)
    freqs = np.array([1.0, 8.0, 45.0, 130.0])
    w = nw.Morse(1000, dtype='float32')
    c = w.cwt_batch(x, freqs)
    p = w.cwt_batch(x, freqs, out='power')
    a = w.cwt_batch(x, freqs, out='abs')
    assert large_ran(w)
    assert c.shape == (S, 4, n)
    for s in range(S):
        ref = O.cwt('morse', x[s].astype(np.float64), freqs)
        assert rel_err(c[s], ref) <= 2 * tol(n), (s, rel_err(c[s], ref))
        assert rel_err(p[s], np.abs(ref) ** 2) <= 4 * tol(n)
        assert rel_err(a[s], np.abs(ref)) <= 2 * tol(n)
    assert rel_err(c[S - 1], w.cwt(x[S - 1], freqs)) == 0.0


def test_large_interpolate_and_table_kind():
    """interpolate=True (the X mask and the zero upper half of W, base.py:107-123, 400-401)
    and a device-built MexicanHat table (complex rows, the NW_TABLE path of the row pass)."""
    n = 1 << 17
    x = synth(1, n, seed=11)[0]
    freqs = np.array([2.0, 20.0, 90.0])
    w = nw.Morse(1000, dtype='float32', interpolate=True)
    got = w.cwt(x, freqs)
    assert large_ran(w)
    ref = O.cwt('morse', x.astype(np.float64), freqs, interpolate=True)
    assert rel_err(got, ref) <= tol(n)
    m = nw.MexicanHat(1000, dtype='float32')
    got = m.cwt(x, freqs)
    assert large_ran(m)
    ref = O.cwt('mexican_hat', x.astype(np.float64), freqs)
    assert rel_err(got, ref) <= tol(n), rel_err(got, ref)


def test_large_engine_agrees_with_rocfft_and_reductions():
    """The two-pass engine against the rocFFT engine on a 2^20 batch, and the epoch
    reductions (the fused pass writes |y|^2 per chunk, k_accumulate sums it)."""
    n = 1 << 20
    x = synth(2, n, seed=5)
    freqs = np.linspace(0.5, 250, 12)
    a = nw.Morse(1000, dtype='float32', engine='rocfft').cwt_batch(x, freqs)
    w = nw.Morse(1000, dtype='float32')
    b = w.cwt_batch(x, freqs)
    assert large_ran(w)
    assert rel_err(b, a) <= 3e-5, rel_err(b, a)
    pm = w.cwt_batch(x, freqs, out='power_mean')
    assert rel_err(pm, np.mean(np.abs(a.astype(np.complex128)) ** 2, axis=0)) <= 1e-4


def test_large_support_pruning_edges():
    """Rows whose support ends inside the first element block (f = 0.1 Hz at 2^18: the
    Morse row is zero past bin ~ 700) and a scale whose support covers every bin."""
    n = 1 << 18
    x = synth(1, n, seed=13)[0]
    freqs = np.array([0.1, 0.2, 499.0])
    w = nw.Morse(1000, dtype='float32')
    got = w.cwt(x, freqs)
    ref = O.cwt('morse', x.astype(np.float64), freqs)
    for i in range(freqs.size):
        assert rel_err(got[i], ref[i]) <= tol(n), (freqs[i], rel_err(got[i], ref[i]))


# ------------------------------------------------------------------ fp64 (the reference's dtype)
@pytest.mark.parametrize('n', [1 << 15, 1 << 16, 1 << 18, 1 << 19, 1 << 21])
@pytest.mark.parametrize('kind', ['morse', 'morlet', 'shannon'])
def test_large_fp64_against_oracle(kind, n):
    """The fp64 two-pass form (N2 <= 8192 on chip, N1 = 32 .. 256 here; pass-0 column
    twiddles from two exact tables) for the analytic kinds at the default compute dtype."""
    x = synth(1, n, seed=n % 997 + len(kind))[0].astype(np.float64)
    freqs = np.array([0.5, 3.0, 17.0, 60.0, 250.0, 400.0])
    w = CLASSES[kind](1000)
    got = w.cwt(x, freqs)
    assert large_ran(w)
    ref = O.cwt(kind, x, freqs)
    assert got.shape == (freqs.size, n) and got.dtype == np.complex128
    assert rel_err(got, ref) <= 1e-12, rel_err(got, ref)


def test_large_fp64_outputs_batch_table_and_rocfft_agreement():
    """fp64: |.|^2 / |.| epilogues, a 2-signal batch, interpolate, a MexicanHat table (complex
    rows) and agreement with the rocFFT engine."""
    n = 1 << 17
    x = synth(2, n, seed=17).astype(np.float64)
    freqs = np.array([1.0, 8.0, 45.0, 130.0])
    w = nw.Morse(1000)
    c = w.cwt_batch(x, freqs)
    p = w.cwt_batch(x, freqs, out='power')
    a = w.cwt_batch(x, freqs, out='abs')
    assert large_ran(w)
    for s in range(2):
        ref = O.cwt('morse', x[s], freqs)
        assert rel_err(c[s], ref) <= 1e-12
        assert rel_err(p[s], np.abs(ref) ** 2) <= 2e-12
        assert rel_err(a[s], np.abs(ref)) <= 1e-12
    r = nw.Morse(1000, engine='rocfft').cwt_batch(x, freqs)
    assert rel_err(c, r) <= 1e-12
    pm = w.cwt_batch(x, freqs, out='power_mean')            # epoch reduction over the batch
    assert rel_err(pm, np.mean(np.abs(c) ** 2, axis=0)) <= 1e-13
    itc = w.cwt_batch(x, freqs, out='itc')
    assert np.max(np.abs(itc - np.abs(np.mean(c / np.abs(c), axis=0)))) <= 1e-12
    wi = nw.Morse(1000, interpolate=True)
    assert rel_err(wi.cwt(x[0], freqs), O.cwt('morse', x[0], freqs, interpolate=True)) <= 1e-12
    assert large_ran(wi)
    m = nw.MexicanHat(1000)
    assert rel_err(m.cwt(x[1], freqs), O.cwt('mexican_hat', x[1], freqs)) <= 1e-12
    assert large_ran(m)


@pytest.mark.parametrize('out', ['cwt', 'power', 'abs'])
@pytest.mark.parametrize('kind', ['morse', 'mexican_hat'])
def test_fused_fp64_16384_one_pass(kind, out):
    """fp64 at n = 16384: the one-pass fused kernel with 1024 threads (E = 16, W re-read
    per signal), real (Morse) and complex (MexicanHat table) rows, against the oracle."""
    n, S = 16384, 3
    x = synth(S, n, seed=29).astype(np.float64)
    freqs = np.array([0.7, 5.0, 33.0, 260.0])
    w = CLASSES[kind](1000)
    got = w.cwt_batch(x, freqs, out=out)
    st = w.plan_stats()
    assert any(s['engine'] == 'fused' and s['launches_fused'] > 0 and s['launches_rows'] == 0 for s in st)
    for s in range(S):
        ref = O.cwt(kind, x[s], freqs)
        ref = {'cwt': ref, 'power': np.abs(ref) ** 2, 'abs': np.abs(ref)}[out]
        assert rel_err(got[s], ref) <= (2e-12 if out == 'power' else 1e-12), (s, rel_err(got[s], ref))


@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_large_scale_chunks_are_exact(dtype, monkeypatch):
    """The two-pass form runs its scales in chunks sized to the B budget (8 GiB: one chunk at
    this length); chunks of 2 scales (NW_LARGE_FCHUNK, diagnostics) give the same bits."""
    n = 1 << 15
    x = synth(2, n, seed=21).astype(dtype)
    freqs = np.array([1.0, 5.0, 17.0, 60.0, 140.0])
    whole = nw.Morse(1000, dtype=dtype).cwt_batch(x, freqs)
    monkeypatch.setenv('NW_LARGE_FCHUNK', '2')
    w = nw.Morse(1000, dtype=dtype)
    chunked = w.cwt_batch(x, freqs)
    assert large_ran(w)
    st = next(iter(w._plans.values())).stats()
    assert st['launches_rows'] == 2 * 3                   # per signal, ceil(5 / 2) row-pass launches
    np.testing.assert_array_equal(chunked, whole)


@pytest.mark.parametrize('b', [0.5, 3.0, 20.0, 63.5, 64.0, 100.0])
@pytest.mark.parametrize('n', [1 << 15, 1 << 16])
def test_large_fp64_morse_b_forms(b, n):
    """The fp64 row pass's Morse forms across their dispatch boundary (nw_large.hip
    morse_fast_of): r = 3 with 2b a whole number below 128 takes the x^b multiply chain
    (b = 0.5: the sqrt alone, b = 3 / 20: whole powers, b = 63.5: the longest chain), b = 64
    and above the log-domain form.  b = 100 with f = 0.5 / 0.8 Hz puts x^b past the fp64 range
    (x = nu / f up to 2000): the reference's 2 * (x^b * exp(...)) is inf * 0 = NaN there, so
    those whole rows are NaN (ifft) and the checked form must give the same NaN rows
    (wavelets.py:65-74).  fp64 1e-12 of each finite row's max."""
    x = synth(1, n, seed=int(b * 10) + n % 97)[0].astype(np.float64)
    freqs = np.array([0.5, 0.8, 3.0, 17.0, 60.0, 250.0])
    w = nw.Morse(1000, b=b, r=3.0)
    got = w.cwt(x, freqs)
    assert large_ran(w)
    with np.errstate(all='ignore'):
        ref = O.cwt('morse', x, freqs, b=b, r=3.0)
    nan_rows = np.isnan(ref).any(axis=1)
    assert nan_rows.any() == (b == 100.0)
    for f in range(freqs.size):
        if nan_rows[f]:
            assert np.isnan(got[f]).all(), (b, freqs[f])
        else:
            assert np.isfinite(got[f]).all() and rel_err(got[f], ref[f]) <= 1e-12, (b, freqs[f])


@pytest.mark.parametrize('n', [4096, 1 << 15])
def test_morse_overflow_rows_fp32(n):
    """fp32 compute (one-pass table at n = 4096, the two-pass rows' checked instantiation at
    2^15) keeps the reference's NaN rows where x^b overflows fp64 (b = 100, f <= 0.8 Hz) and
    matches the finite rows at the fp32 tolerance."""
    x = synth(1, n, seed=n % 89)[0]
    freqs = np.array([0.5, 0.8, 3.0, 60.0])
    got = nw.Morse(1000, b=100.0, r=3.0, dtype='float32').cwt(x, freqs)
    with np.errstate(all='ignore'):
        ref = O.cwt('morse', x.astype(np.float64), freqs, b=100.0, r=3.0)
    for f in range(freqs.size):
        if np.isnan(ref[f]).any():
            assert np.isnan(got[f]).all(), freqs[f]
        else:
            assert rel_err(got[f], ref[f]) <= tol(n), freqs[f]


@pytest.mark.parametrize('grid', ['full', 'half'])
def test_large_fp64_morse_rows_each_scale(grid):
    """The fp64 b = 17.5 row pass's two evaluators, every row on its own scale: rows that
    start at bin 0 (the plan's grid spans n: WDesc::off = 0) take the exponential factor by
    the product recurrence of nw_large.hip RowW<double>::Rec, rows of a shorter grid
    (real_length n / 2: pad_to centres them, off = n / 4) the per-bin exp.  24 scales from
    C5's range (bin strides in x from ~0.1 to ~70) against y = ifft(pad_to(W) * fft(x)) of
    the oracle's rows; 1e-12 of each row's own max (the parity contract is per signal)."""
    torch = pytest.importorskip('torch')
    from ninwavelets_amd import _lib as L
    n = 1 << 20
    freqs = np.linspace(0.5, 250, 24)
    rl = n / 1000. if grid == 'full' else n / 2000.
    x = synth(1, n, seed=5)[0].astype(np.float64)
    p = nw.Plan(n, freqs.size, 'float64', max_batch=1)
    p.set_wavelet('morse', [17.5, 3.0], freqs, L.trans_grid(rl, 1000., False))
    xt = torch.from_numpy(x[None]).cuda()
    ot = torch.empty((1, freqs.size, n), dtype=torch.complex128, device='cuda')
    p.execute(xt, ot, out_kind='cwt')
    p.sync()
    st = p.stats()
    assert st['engine'] == 'fused' and st['launches_rows'] > 0, st
    got = ot[0].cpu().numpy()
    p.close()
    rows = O.fft_wavelets('morse', freqs, 1000., rl, False)
    assert (rows[0].shape[0] == n) == (grid == 'full')
    ref = O.cwt_from_rows(x, rows, False)
    for f in range(freqs.size):
        assert rel_err(got[f], ref[f]) <= 1e-12, (grid, freqs[f], rel_err(got[f], ref[f]))

"""GPU parity of the chirp-z fused form (nw_chirp.hip): the lengths the power-of-two
kernels do not take (any n with 2n - 1 <= 16384 in fp32, <= 8192 in fp64, other than the
power-of-two n >= 1024) -- e.g. MNE epochs of 1201 or 4097 samples -- now run as two
on-chip FFTs per (scale, signal) row instead of rocFFT, of the smallest power of two M >= 1024
that is wrap-free for the row (M >= n + K - 1, K = the W row's support; at most
2^ceil(log2(2n - 1))).

Tolerances against the fp64 oracle (numpy + scipy.fftpack, the reference's arithmetic):
fp64 1e-12 of max|ref| (|.|^2 twice that), fp32 2e-5 (the chirp factors and two M-point
FFTs add round-off over the power-of-two kernels' 1e-5; |.|^2 twice that), plus the 1e-30
floor for outputs below fp32 range (test_gpu_parity.py).
"""
import numpy as np
import pytest

from oracle import nw_oracle as O

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402


def synth(S, n, seed, sfreq=1000.):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sfreq
    fc = rng.uniform(1, 100, (S, 1))
    ph = rng.uniform(0, 2 * np.pi, (S, 1))
    return (np.sin(2 * np.pi * fc * t + ph) + 0.1 * rng.standard_normal((S, n))).astype(np.float32)


def within(got, ref, dtype, out):
    t = (1e-12 if dtype == 'float64' else 2e-5) * (2 if out == 'power' else 1)
    floor = 1e-30 if dtype == 'float32' else 0.0
    return np.max(np.abs(got - ref), initial=0.0) <= t * np.max(np.abs(ref), initial=0.0) + floor


def oracle(kind, x, freqs, out, **kw):
    y = np.stack([O.cwt(kind, xi.astype(np.float64), freqs, **kw) for xi in x])
    return y if out == 'cwt' else (np.abs(y) if out == 'abs' else np.abs(y) ** 2)


def chirp_plan(n, F, dtype, kind, params, freqs, max_batch=4, interpolate=False, engine=None):
    g = L.trans_grid(n / 1000., 1000., interpolate)
    p = nw.Plan(n, F, dtype, max_batch=max_batch, interpolate=interpolate, engine=engine)
    p.set_wavelet(kind, list(params), np.asarray(freqs, dtype=np.float64), g)
    return p


F32_N = [1, 2, 3, 5, 21, 300, 301, 512, 1000, 1021, 1201, 2049, 3001, 4097, 8191]
F64_N = [1, 3, 21, 300, 301, 1000, 1201, 2049, 4095]


@pytest.mark.parametrize('dtype,n', [('float32', n) for n in F32_N] + [('float64', n) for n in F64_N])
def test_chirp_lengths_against_oracle(dtype, n):
    freqs = np.array([1.5, 7., 30., 120.])
    S = 3
    x = synth(S, n, 51 + n).astype(dtype)
    p = chirp_plan(n, len(freqs), dtype, 'morse', (17.5, 3.), freqs)
    for out in ('cwt', 'abs', 'power'):
        got = p.execute(x, out_kind=out)
        ref = oracle('morse', x, freqs, out)
        assert within(got, ref, dtype, out), (out, np.max(np.abs(got - ref)) / np.max(np.abs(ref)))
    st = p.stats()
    assert st['engine'] == 'fused' and st['launches_fused'] == 3 * 1 and st['launches_multiply'] == 0


@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_chirp_kinds_interpolate_and_chunks(dtype):
    """Morlet, Shannon, MexicanHat (complex table rows), interpolate, several chunks
    with a ragged last one, against the oracle and the rocFFT engine."""
    n, S = 1201, 11
    x = synth(S, n, 52).astype(dtype)
    freqs = np.array([2., 9., 40., 90., 200.])
    for kind, params, kw in (('morlet', (7., 0.), {'sigma': 7., 'gabor': False}), ('shannon', (), {})):
        for interp in (False, True):
            p = chirp_plan(n, len(freqs), dtype, kind, params, freqs, max_batch=4, interpolate=interp)
            got = p.execute(x, out_kind='cwt')
            ref = oracle(kind, x, freqs, 'cwt', interpolate=interp, **kw)
            assert within(got, ref, dtype, 'cwt'), (kind, interp)
            r = chirp_plan(n, len(freqs), dtype, kind, params, freqs, max_batch=4, interpolate=interp,
                           engine='rocfft').execute(x, out_kind='cwt')
            assert within(got, r.astype(np.complex128), dtype, 'cwt')
    w = nw.MexicanHat(1000, dtype=dtype)
    got = w.cwt(x[0].astype(np.float64 if dtype == 'float64' else np.float32), list(freqs))
    ref = O.cwt('mexican_hat', x[0].astype(np.float64), list(freqs))
    assert within(got, ref, dtype, 'cwt')


@pytest.mark.parametrize('out', ['power_mean', 'itc'])
def test_chirp_epoch_reductions(out):
    n, S = 1201, 9
    x = synth(S, n, 53)
    freqs = np.array([3., 11., 60.])
    p = chirp_plan(n, 3, 'float32', 'morse', (17.5, 3.), freqs, max_batch=4)
    c = oracle('morse', x, freqs, 'cwt')
    ref = np.mean(np.abs(c) ** 2, axis=0) if out == 'power_mean' else np.abs(np.mean(c / np.abs(c), axis=0))
    got = p.execute(x, out_kind=out)
    assert np.max(np.abs(got - ref)) <= 4e-5 * np.max(np.abs(ref))


def test_no_chirp_flag_keeps_rocfft():
    g = L.trans_grid(1.201, 1000., False)
    import ctypes
    h = ctypes.c_void_p()
    L.check(L.lib().nw_plan_create(ctypes.byref(h), 0, 1201, 1, 2, L.NW_F32, L.NW_NO_CHIRP))
    st = L.nw_stats()
    L.check(L.lib().nw_plan_stats(h, ctypes.byref(st)))
    assert st.engine == L.NW_ENGINE_ROCFFT
    L.check(L.lib().nw_plan_destroy(h))
    assert g.len_full >= 1201


@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_chirp_rows_of_different_transform_sizes(dtype):
    """Band-limited rows run at the smallest wrap-free M >= n + K - 1 (K = the W row's
    support): interleaved low / high scales at n = 1201 fall into M = 2048 and 4096
    launches of one execute; the full-M rows (K ~ n) and all-zero rows are covered too."""
    n, S = 1201, 5
    x = synth(S, n, 54).astype(dtype)
    freqs = np.array([2., 300., 5., 450., 100., 20000.])   # 20 kHz: support beyond n/2
    p = chirp_plan(n, len(freqs), dtype, 'morse', (17.5, 3.), freqs, max_batch=4)
    for out in ('cwt', 'power'):
        got = p.execute(x, out_kind=out)
        ref = oracle('morse', x, freqs, out)
        assert within(got, ref, dtype, out), out
    tab = np.zeros((3, n), dtype=np.complex128)          # an all-zero table row among others
    tab[1, :40] = 1.0 + 0.5j
    tab[2] = np.exp(-np.arange(n) / 50.)
    g = L.nw_grid(1.0, n, n)
    q = nw.Plan(n, 3, dtype, max_batch=4)
    q.set_wavelet('table', [], np.array([1., 2., 3.]), g, table=tab)
    got = q.execute(x, out_kind='cwt')
    ref = np.stack([O.cwt_from_rows(xi.astype(np.float64), list(tab), False) for xi in x])
    assert within(got, ref, dtype, 'cwt')


@pytest.mark.parametrize('dtype,n', [('float32', 10001), ('float32', 14001), ('float64', 5001)])
def test_chirp_tentative_lengths(dtype, n):
    """2n - 1 beyond the largest on-chip transform: the auto engine takes the chirp-z form
    when every row's support K fits (n + K - 1 <= 16384 fp32 / 8192 fp64), and falls back
    to the rocFFT engine for a wavelet with a wide row -- re-armed by the next wavelet."""
    S = 2
    x = synth(S, n, 55).astype(dtype)
    narrow = np.array([2., 5., 11.])
    p = chirp_plan(n, 3, dtype, 'morse', (17.5, 3.), narrow, max_batch=2)
    got = p.execute(x, out_kind='cwt')
    assert p.stats()['engine'] == 'fused'
    assert within(got, oracle('morse', x, narrow, 'cwt'), dtype, 'cwt')
    wide = np.array([2., 5., 400.])                  # 400 Hz: support ~ n
    g = L.trans_grid(n / 1000., 1000., False)
    p.set_wavelet('morse', [17.5, 3.], wide, g)
    for out in ('power', 'cwt', 'abs'):
        # hybrid: the 2 and 5 Hz rows on chip, the 400 Hz row through the rocFFT path
        got = p.execute(x, out_kind=out)
        assert p.stats()['engine'] == 'fused'
        assert within(got, oracle('morse', x, wide, out), dtype, out), out
    allwide = np.array([300., 400.])                 # no row fits: the whole wavelet on rocFFT
    p2 = chirp_plan(n, 2, dtype, 'morse', (17.5, 3.), allwide, max_batch=2)
    got = p2.execute(x, out_kind='power')
    assert p2.stats()['engine'] == 'rocfft'
    assert within(got, oracle('morse', x, allwide, 'power'), dtype, 'power')
    p.set_wavelet('morse', [17.5, 3.], narrow, g)
    got = p.execute(x, out_kind='abs')
    assert p.stats()['engine'] == 'fused'
    assert within(got, oracle('morse', x, narrow, 'abs'), dtype, 'abs')


@pytest.mark.parametrize('dtype,n', [('float32', 10001), ('float64', 4097)])
def test_chirp_hybrid_reductions_and_repeated_rows(dtype, n):
    """Hybrid rows (some on chip, the wide ones via rocFFT) under the epoch reductions and
    under repeated rows (the distinct-row view): against the oracle."""
    S = 5
    x = synth(S, n, 77).astype(dtype)
    freqs = np.array([3., 420., 3., 420., 40.])       # repeated: U = 3 > F/2, no dedup view
    p = chirp_plan(n, len(freqs), dtype, 'morse', (17.5, 3.), freqs, max_batch=2)
    ref = oracle('morse', x, freqs, 'cwt')
    pm = p.execute(x, out_kind='power_mean')
    assert p.stats()['engine'] == 'fused'
    assert within(pm, np.mean(np.abs(ref) ** 2, axis=0), dtype, 'power')
    itc = p.execute(x, out_kind='itc')
    t = 1e-10 if dtype == 'float64' else 1e-3
    assert np.max(np.abs(itc - np.abs(np.mean(ref / np.abs(ref), axis=0)))) <= t
    rep = np.array([3., 420., 3., 420.])              # U = 2 <= F/2: the distinct-row view
    p2 = chirp_plan(n, len(rep), dtype, 'morse', (17.5, 3.), rep, max_batch=2)
    got = p2.execute(x, out_kind='cwt')
    assert p2.stats()['unique_rows'] == 2 and p2.stats()['engine'] == 'fused'
    assert within(got, oracle('morse', x, rep, 'cwt'), dtype, 'cwt')


@pytest.mark.parametrize('dtype,n', [('float64', 1201), ('float64', 701), ('float32', 1201), ('float32', 4097)])
def test_chirp_fused_epoch_partials(dtype, n):
    """Epoch reductions on the chirp-z form (MNE lengths, mneutils.py:42-71): the kernel
    read-modify-writes one fp64 partial row per block of 8 signals (signal order) instead of
    writing every signal's row.  power_sum equals the sum of the same plan's per-signal power
    output (fp64: the same values, regrouped fp64 additions: 1e-13; fp32: 1e-6); chunk-size
    independent;
    ITC against the same plan's materialised cwt; both against the oracle.  fp64 phases run
    fused only where every row's transform is M <= 2048 (N = 701, 1201 at the C3 scale list)."""
    S, freqs = 19, np.arange(1, 257, dtype=np.float64)
    x = synth(S, n, seed=n + 17).astype(dtype)
    g = L.trans_grid(n / 1000., 1000., False)
    plan = nw.Plan(n, 256, dtype, max_batch=8)
    plan.set_wavelet('morse', [17.5, 3.], freqs, g)
    pw = plan.execute(x, out_kind='power').astype(np.float64)
    assert L.KERNEL_NAMES[plan.stats()['kernel']] == 'nw_chirp_kernel'
    ps = plan.execute(x, out_kind='power_sum')
    # fp32: the partial-sum instantiation (E = 16, 2 waves/SIMD) is scheduled apart from the
    # power output's (3 waves/SIMD; E = 32 at M = 8192), which moves fp32 values of y by a few
    # ulp: held to the fp32 contract
    np.testing.assert_allclose(ps, pw.sum(axis=0), rtol=1e-13 if dtype == 'float64' else 1e-5)
    other = nw.Plan(n, 256, dtype, max_batch=3)
    other.set_wavelet('morse', [17.5, 3.], freqs, g)
    np.testing.assert_allclose(other.execute(x, out_kind='power_sum'), ps, rtol=1e-13)
    c = plan.execute(x, out_kind='cwt').astype(np.complex128)
    itc = plan.execute(x, out_kind='itc')
    ref_itc = np.abs(np.mean(c / np.abs(c), axis=0))
    assert np.max(np.abs(itc - ref_itc)) <= (1e-13 if dtype == 'float64' else 1e-5)
    np.testing.assert_allclose(other.execute(x, out_kind='phase_sum'), plan.execute(x, out_kind='phase_sum'),
                               rtol=1e-13, atol=1e-13 * S)
    o = oracle('morse', x, freqs[::51], 'cwt')
    pm = plan.execute(x, out_kind='power_mean')
    assert within(pm[::51], np.mean(np.abs(o) ** 2, axis=0), dtype, 'power')
    t_itc = 1e-10 if dtype == 'float64' else 1e-4
    assert np.max(np.abs(itc[::51] - np.abs(np.mean(o / np.abs(o), axis=0)))) <= t_itc


@pytest.mark.parametrize('dtype', ['float64', 'float32'])
def test_chirp_table_rows_epoch_reductions(dtype):
    """Epoch reductions of complex table rows (MexicanHat: base.py:249-256, WaveletMode.Normal)
    at an MNE length on the chirp-z form (mneutils.py:42-71).  Table rows take the per-signal
    chunk path (their partial-sum kernels are not scratch-free), so power_sum equals the sum of
    the same plan's power output and ITC the materialised cwt's, both against the oracle."""
    n, S = 1201, 11
    freqs = np.arange(1, 100, 7, dtype=np.float64)
    x = synth(S, n, seed=4242).astype(dtype)
    w = nw.MexicanHat(1000, dtype=dtype)
    pm = w.cwt_batch(x, freqs, out='power_mean')
    assert w._plans and all(pl.stats()['engine'] == 'fused' for pl in w._plans.values())
    c = w.cwt_batch(x, freqs).astype(np.complex128)
    assert L.KERNEL_NAMES[next(iter(w._plans.values())).stats()['kernel']] == 'nw_chirp_kernel'
    np.testing.assert_allclose(pm, np.mean(np.abs(c) ** 2, axis=0), rtol=1e-12 if dtype == 'float64' else 1e-5)
    itc = w.cwt_batch(x, freqs, out='itc')
    assert np.max(np.abs(itc - np.abs(np.mean(c / np.abs(c), axis=0)))) <= (1e-12 if dtype == 'float64' else 1e-5)
    o = oracle('mexican_hat', x, freqs, 'cwt')
    assert within(pm, np.mean(np.abs(o) ** 2, axis=0), dtype, 'power')

"""GPU parity: the HIP path (through the C ABI) against the reference's own outputs
(golden vectors made by tests/golden/make_golden.py) and against the CPU oracle.

Tolerances (north_star: "within a stated fp64/fp32 tolerance"):
  fp64 compute:  max|out - ref| <= 1e-12 * max|ref|
  fp32 compute:  max|out - ref| <= 1e-5  * max|ref| + 1e-30  (2e-5 for |.|^2 outputs);
                 the 1e-30 floor covers cases whose reference output is itself below
                 fp32 range (e.g. N=21, 1 Hz: |ref| ~ 1e-260)
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden
from oracle import nw_oracle as O

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402

TOL = {'float64': 1e-12, 'float32': 1e-5}
ENGINES = ['rocfft', 'auto']
SINGLE = [n for n in golden_names() if not n.startswith(('readme_2d', 'reuse', 'epochs', 'baseline', 'wavelets', 'long',
                                                          'plugin'))]
CLASSES = {'morse': nw.Morse, 'morlet': nw.Morlet, 'shannon': nw.Shannon,
           'mexican_hat': nw.MexicanHat, 'haar': nw.Haar}


def make(kind, sfreq, interpolate, params, dtype, engine):
    p = dict(params)
    return CLASSES[kind](sfreq, interpolate=interpolate, dtype=dtype, engine=engine, **p)


def rel_err(got, ref):
    scale = max(np.max(np.abs(ref)), 1e-300)
    return np.max(np.abs(got - ref)) / scale


def close(got, ref, rtol, dtype):
    floor = 1e-30 if dtype == 'float32' else 0.0
    return np.max(np.abs(got - ref), initial=0.0) <= rtol * np.max(np.abs(ref), initial=0.0) + floor


def tol(dtype, op):
    return TOL[dtype] * (2 if op == 'power' else 1)


@pytest.mark.parametrize('engine', ENGINES)
@pytest.mark.parametrize('dtype', ['float64', 'float32'])
@pytest.mark.parametrize('name', SINGLE)
def test_single_signal_golden(name, dtype, engine):
    """Every single-signal reference golden through the drop-in class API."""
    g = load_golden(name)
    m = g['meta']
    w = make(m['kind'], m['sfreq'], m['interpolate'], m['params'], dtype, engine)
    fn = {'cwt': w.cwt, 'power': w.power, 'abs': w.abs}[m['op']]
    got = fn(g['x'], g['freqs'])
    ref = g['out']
    assert got.shape == ref.shape
    if dtype == 'float64':
        assert got.dtype == ref.dtype
    t = tol(dtype, m['op'])
    if m['dtype'] == 'float32':      # the reference ran its forward FFT in single precision
        t = max(t, 1e-5)
    assert close(got, ref, t, dtype), (name, rel_err(got, ref))


@pytest.mark.parametrize('name', [n for n in SINGLE if 'w_first' in load_golden(n)])
def test_device_wavelet_rows_match_reference(name):
    """The cached rows evaluated by the kernels equal the reference's fft_wavelets."""
    g = load_golden(name)
    m = g['meta']
    w = make(m['kind'], m['sfreq'], m['interpolate'], m['params'], 'float64', None)
    rows = w.make_fft_wavelets(g['freqs'], m['n'] / m['sfreq'])
    for got, ref in ((rows[0], g['w_first']), (rows[-1], g['w_last'])):
        assert got.shape == ref.shape
        assert np.max(np.abs(got - ref)) <= 1e-13 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize('dtype', ['float64', 'float32'])
@pytest.mark.parametrize('kind', ['morse', 'morlet', 'shannon', 'mexican_hat'])
def test_readme_2d_quirk(kind, dtype):
    """README example with a (1, 300) array: the single cached bin broadcasts."""
    g = load_golden(f'readme_2d_{kind}')
    w = make(kind, 1000, False, {}, dtype, None)
    got = w.power(g['x'], range(1, 100))
    assert got.shape == g['out'].shape
    assert close(got, g['out'], tol(dtype, 'power'), dtype)


@pytest.mark.parametrize('engine', ENGINES)
def test_reuse_cache_is_unkeyed(engine):
    g = load_golden('reuse_morse')
    w = nw.Morse(1000, engine=engine)
    assert rel_err(w.cwt(g['xa'], g['freqs']), g['oa']) <= 1e-12
    assert rel_err(w.cwt(g['xb'], [1., 2.]), g['ob']) <= 1e-12     # freqs ignored, rows padded
    assert rel_err(w.cwt(g['xc'], None), g['oc']) <= 1e-12         # rows cropped
    g = load_golden('reuse_morse_interp')
    w = nw.Morse(1000, interpolate=True, engine=engine)
    assert rel_err(w.cwt(g['xa'], g['freqs']), g['oa']) <= 1e-12
    assert rel_err(w.cwt(g['xb'], [1., 2.]), g['ob']) <= 1e-12


class FakeEpochs:
    def __init__(self, data, sfreq, ch_names):
        self._d, self.info, self.ch_names = data, {'sfreq': sfreq}, list(ch_names)

    def get_data(self):
        return self._d


@pytest.mark.parametrize('dtype', ['float64', 'float32'])
@pytest.mark.parametrize('kind', ['morse', 'morlet'])
def test_epochs_wavelet(kind, dtype):
    g = load_golden(f'epochs_{kind}')
    ep = FakeEpochs(g['data'], g['meta']['sfreq'], g['meta']['ch_names'])
    t = TOL[dtype]
    c = nw.EpochsWavelet(ep, CLASSES[kind](1000, dtype=dtype)).cwt('b', list(g['freqs']))
    assert c.shape == g['cwt_b'].shape and rel_err(c, g['cwt_b']) <= t
    p = nw.EpochsWavelet(ep, CLASSES[kind](1000, dtype=dtype)).power('c', list(g['freqs']))
    assert rel_err(p, g['power_c']) <= 2 * t
    itc = nw.EpochsWavelet(ep, CLASSES[kind](1000, dtype=dtype)).itc('a', list(g['freqs']))
    # ITC is a mean of unit phasors (values in [0, 1]): the contract is absolute.
    # fp64: 1e-10.  fp32: 2e-5 where every epoch's |cwt| >= 0.1 x its scale row's max (the
    # phase of y is then set to ~1e-6 by y's fp32 error); 1e-3 everywhere (near |y| = 0 the
    # fp32 phase is arbitrary and moves the mean by up to 2/E per such epoch)
    if dtype == 'float64':
        assert np.max(np.abs(itc - g['itc_a'])) <= 1e-10
    else:
        ca = np.abs(nw.EpochsWavelet(ep, CLASSES[kind](1000, dtype='float64')).cwt('a', list(g['freqs'])))
        good = ca.min(axis=0) >= 0.1 * ca.max(axis=(0, 2))[:, None]
        assert good.sum() > 0.2 * good.size
        err = np.abs(itc - g['itc_a'])
        assert np.max(err[good]) <= 2e-5 and np.max(err) <= 1e-3, (np.max(err[good]), np.max(err))


# ------------------------------------------------------------------ larger sizes
def synth(S, n, seed, dtype=np.float32, sfreq=1000.):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sfreq
    fc = rng.uniform(1, 100, (S, 1))
    ph = rng.uniform(0, 2 * np.pi, (S, 1))
    return (np.sin(2 * np.pi * fc * t + ph) + 0.1 * rng.standard_normal((S, n))).astype(dtype)


@pytest.mark.parametrize('engine', ENGINES)
@pytest.mark.parametrize('kind,n,F,dtype', [
    ('morlet', 16384, 128, 'float32'),     # C2 shape (fewer signals)
    ('morse', 4096, 256, 'float32'),       # C3 shape
    ('morse', 16384, 256, 'float32'),      # C4 shape
    ('morse', 16384, 64, 'float64'),
    ('shannon', 8192, 16, 'float32'),
])
def test_batch_against_oracle_sampled(kind, n, F, dtype, engine):
    S = 8
    x = synth(S, n, seed=n + F)
    freqs = np.arange(1, F + 1, dtype=np.float64)
    w = CLASSES[kind](1000, dtype=dtype, engine=engine)
    out = w.cwt_batch(x, freqs)
    assert out.shape == (S, F, n)
    rng = np.random.default_rng(1)
    for s in rng.choice(S, 3, replace=False):
        fsel = np.sort(rng.choice(F, 6, replace=False))
        ref = O.cwt(kind, x[s].astype(np.float64), freqs[fsel])
        assert rel_err(out[s, fsel], ref) <= TOL[dtype] * 3, (s, rel_err(out[s, fsel], ref))


@pytest.mark.parametrize('engine', ENGINES)
def test_power_abs_consistent_and_linear(engine):
    S, n, F = 16, 4096, 64
    x = synth(S, n, 5).astype(np.float64)
    y = synth(S, n, 6).astype(np.float64)
    freqs = np.linspace(0.5, 200, F)
    w = nw.Morse(1000, engine=engine)
    cx = w.cwt_batch(x, freqs)
    cy = w.cwt_batch(y, freqs)
    cxy = w.cwt_batch(2.0 * x - 3.0 * y, freqs)
    assert rel_err(cxy, 2.0 * cx - 3.0 * cy) <= 1e-12
    assert rel_err(w.cwt_batch(x, freqs, out='power'), np.abs(cx) ** 2) <= 1e-13
    assert rel_err(w.cwt_batch(x, freqs, out='abs'), np.abs(cx)) <= 1e-13
    # the batch equals the per-signal drop-in call
    assert rel_err(cx[3], w.cwt(x[3], freqs)) <= 1e-14


def test_engines_agree_fp32():
    x = synth(32, 16384, 9)
    freqs = np.arange(1, 65, dtype=np.float64)
    a = nw.Morse(1000, dtype='float32', engine='rocfft').cwt_batch(x, freqs, out='power')
    b = nw.Morse(1000, dtype='float32').cwt_batch(x, freqs, out='power')
    assert rel_err(b, a) <= 2e-5


def test_empty_and_ragged_inputs():
    w = nw.Morse(1000)
    out = w.cwt_batch(np.zeros((0, 256)), [1., 2., 3.])
    assert out.shape == (0, 3, 256)
    for n in (1, 2, 3, 5, 127, 1000, 1021):
        x = synth(1, n, n)[0].astype(np.float64)
        ref = O.cwt('morse', x, [2., 7., 30.])
        got = nw.Morse(1000).cwt(x, [2., 7., 30.])
        assert rel_err(got, ref) <= 1e-12, n


def test_device_tensors_and_streams():
    torch = pytest.importorskip('torch')
    n, F, S = 16384, 32, 8
    x = synth(S, n, 11)
    plan = nw.Plan(n, F, 'float32', device=0, max_batch=S)
    g = nw._lib.trans_grid(n / 1000., 1000., False)
    plan.set_wavelet('morse', [17.5, 3.], np.arange(1, F + 1, dtype=np.float64), g)
    host = plan.execute(x, out_kind='cwt')
    xt = torch.from_numpy(x).cuda()
    ot = torch.empty((S, F, n), dtype=torch.complex64, device='cuda')
    plan.execute(xt, ot, out_kind='cwt')
    plan.sync()
    np.testing.assert_array_equal(ot.cpu().numpy(), host)


def test_multi_plan_sharding_is_exact():
    n, F, S = 4096, 16, 10
    x = synth(S, n, 12)
    g = nw._lib.trans_grid(n / 1000., 1000., False)
    freqs = np.arange(1, F + 1, dtype=np.float64)
    plans = []
    for _ in range(2):                               # two shards on device 0
        p = nw.Plan(n, F, 'float32', device=0, max_batch=8)
        p.set_wavelet('morse', [17.5, 3.], freqs, g)
        plans.append(p)
    single = plans[0].execute(x, out_kind='power')
    sharded = nw.execute_multi(plans, x, out_kind='power')
    np.testing.assert_array_equal(sharded, single)


# ------------------------------------------------------------------ epoch reductions
def _plan(n, F, dtype, freqs, engine=None, max_batch=8, kind='morse', params=(17.5, 3.)):
    g = nw._lib.trans_grid(n / 1000., 1000., False)
    p = nw.Plan(n, F, dtype, max_batch=max_batch, engine=None if engine == 'auto' else engine)
    p.set_wavelet(kind, list(params), freqs, g)
    return p


@pytest.mark.parametrize('engine', ENGINES)
@pytest.mark.parametrize('dtype', ['float64', 'float32'])
def test_epoch_reductions_match_materialised(dtype, engine):
    """power_mean / itc (mneutils.py:42-71) reduced on the device over 3 chunks against the
    reference formulas on the oracle's CWT of the same signals: power 2e-12 (fp64) / 2e-5
    (fp32) of max, ITC |d| <= 1e-10 (fp64) or INTEGRATION.md's fp32 contract (2e-5 where
    every epoch's |cwt| >= 0.1 of its row's max, 1e-3 everywhere); the fp64 sum kinds are the
    un-normalised partials of the same accumulators (power_mean = power_sum / S, itc =
    |phase_sum| / S, one rounding to the compute dtype), and the materialised CWT of the same
    plan reduces to the same values within the contract."""
    n, F, S = 4096, 24, 21
    x = synth(S, n, 21).astype(dtype)
    freqs = np.linspace(2., 120., F)
    plan = _plan(n, F, dtype, freqs, engine)
    o = np.stack([O.cwt('morse', x[s].astype(np.float64), freqs) for s in range(S)])
    ref_p = np.mean(np.abs(o) ** 2, axis=0)
    mag = np.abs(o)
    ref_i = np.abs(np.mean(o / mag, axis=0))
    good = np.all(mag >= 0.1 * mag.max(axis=-1, keepdims=True), axis=0)
    f64 = dtype == 'float64'
    pm = plan.execute(x, out_kind='power_mean')
    itc = plan.execute(x, out_kind='itc')
    assert pm.shape == (F, n) and pm.dtype == np.dtype(dtype) and itc.dtype == np.dtype(dtype)
    ps = plan.execute(x, out_kind='power_sum')
    ph = plan.execute(x, out_kind='phase_sum')
    assert ps.dtype == np.float64 and ph.dtype == np.complex128
    one = 1e-15 if f64 else 1.2e-7                    # one rounding to the compute dtype
    assert rel_err(pm, ps / S) <= one
    assert np.max(np.abs(itc - np.abs(ph) / S)) <= one
    c = plan.execute(x, out_kind='cwt').astype(np.complex128)
    for p_, i_ in ((pm, itc), (np.mean(np.abs(c) ** 2, axis=0), np.abs(np.mean(c / np.abs(c), axis=0)))):
        assert rel_err(p_, ref_p) <= (2e-12 if f64 else 2e-5)
        d = np.abs(i_.astype(np.float64) - ref_i)
        if f64:
            assert d.max() <= 1e-10
        else:
            dg = d[good].max() if good.any() else 0.0
            assert dg <= 2e-5 and d.max() <= 1e-3, (dg, d.max())


@pytest.mark.parametrize('engine', ENGINES)
@pytest.mark.parametrize('dtype', ['float64', 'float32'])
def test_itc_is_nan_where_an_epoch_is_zero(dtype, engine):
    """An all-zero epoch has cwt == 0 exactly, so cwt/|cwt| is 0/0 = NaN in the reference
    (mneutils.py:68) and the mean stays NaN; power ignores nothing."""
    n, F, S = 1024, 8, 5
    x = synth(S, n, 3).astype(dtype)
    x[2] = 0
    freqs = np.arange(1., F + 1)
    plan = _plan(n, F, dtype, freqs, engine)
    assert np.all(np.isnan(plan.execute(x, out_kind='itc')))
    c = plan.execute(x, out_kind='cwt').astype(np.complex128)
    assert np.all(c[2] == 0)
    pm = plan.execute(x, out_kind='power_mean')
    assert np.all(np.isfinite(pm)) and rel_err(pm, np.mean(np.abs(c) ** 2, axis=0)) <= 2e-6


def test_epoch_reductions_empty_is_nan():
    plan = _plan(256, 3, 'float64', np.array([1., 2., 3.]))
    out = plan.execute(np.zeros((0, 256)), out_kind='power_mean')
    assert out.shape == (3, 256) and np.all(np.isnan(out))     # 0/0, like np.mean over nothing


def test_epoch_reductions_device_tensors_and_multi_plan():
    torch = pytest.importorskip('torch')
    n, F, S = 16384, 32, 12
    x = synth(S, n, 13)
    freqs = np.arange(1., F + 1)
    plan = _plan(n, F, 'float32', freqs)
    host = plan.execute(x, out_kind='power_mean')
    xt = torch.from_numpy(x).cuda()
    ot = torch.empty((F, n), dtype=torch.float32, device='cuda')
    plan.execute(xt, ot, out_kind='power_mean')
    plan.sync()
    np.testing.assert_array_equal(ot.cpu().numpy(), host)     # same sums, same order
    plans = [_plan(n, F, 'float32', freqs, max_batch=4) for _ in range(2)]
    for kind in ('power_mean', 'itc'):
        single = plan.execute(x, out_kind=kind)
        sharded = nw.execute_multi(plans, x, out_kind=kind)
        assert sharded.shape == (F, n)
        assert np.max(np.abs(sharded - single)) <= 1e-6 * max(1.0, np.max(np.abs(single)))


def test_epochs_wavelet_power_matches_per_epoch_reference():
    """EpochsWavelet.power/itc (device reductions) against the reference formulas on the
    oracle's per-epoch CWTs (mneutils.py:39, 53-55, 67-71)."""
    E, n, freqs = 7, 2048, [3., 9., 27., 81.]
    data = synth(E * 2, n, 31).astype(np.float64).reshape(E, 2, n)
    ep = FakeEpochs(data, 1000., ['a', 'b'])
    ref = np.array([O.cwt('morse', data[e, 1], freqs) for e in range(E)])
    pw = nw.EpochsWavelet(ep, nw.Morse(1000)).power('b', freqs)
    assert rel_err(pw, np.mean(np.abs(ref) ** 2, axis=0)) <= 1e-12
    itc = nw.EpochsWavelet(ep, nw.Morse(1000)).itc('b', freqs)
    assert np.max(np.abs(itc - np.abs(np.mean(ref / np.abs(ref), axis=0)))) <= 1e-10


# ------------------------------------------------------------------ C5 scale (N = 2^24)
@pytest.mark.parametrize('kind,dtype', [('morse', 'float32'), ('shannon', 'float64'), ('morse', 'float64')])
def test_c5_scale_single_signal(kind, dtype):
    """One 2^24-sample signal at three of C5's 512 scales against the fp64 oracle, on the
    auto engine: the two-pass form (nw_large.hip; Shannon's one distinct row through it and
    k_expand_rows).  Tolerance at this length: 1e-4 (fp32), 1e-12 (fp64)."""
    n = 1 << 24
    freqs = np.linspace(0.5, 250, 512)[[0, 200, 511]]
    x = synth(1, n, 3)[0].astype(dtype)
    w = CLASSES[kind](1000, dtype=dtype)
    out = w.cwt(x, freqs)
    st = next(iter(w._plans.values())).stats()
    assert st['engine'] == 'fused' and st['launches_rows'] > 0
    ref = O.cwt(kind, x.astype(np.float64), freqs)
    assert out.shape == (3, n)
    assert rel_err(out, ref) <= (1e-4 if dtype == 'float32' else 1e-12), rel_err(out, ref)


def test_c5_all_512_scales_into_hbm():
    """The whole C5 fp32 output (512 x 2^24 complex64 = 68.7 GB) written into one device
    buffer (no Y staging buffer), sampled rows against the oracle."""
    torch = pytest.importorskip('torch')
    n, F = 1 << 24, 512
    freqs = np.linspace(0.5, 250, F)
    x = synth(1, n, 3)[0]
    plan = _plan(n, F, 'float32', freqs, max_batch=1)
    xt = torch.from_numpy(x).cuda()
    ot = torch.empty((1, F, n), dtype=torch.complex64, device='cuda')
    plan.execute(xt, ot, out_kind='cwt')
    plan.sync()
    sel = [0, 255, 511]
    got = ot[0, sel].cpu().numpy()
    del ot
    torch.cuda.empty_cache()
    ref = O.cwt('morse', x.astype(np.float64), freqs[sel])
    assert rel_err(got, ref) <= 1e-4, rel_err(got, ref)



# ------------------------------------------------------------------ Baseline (§8f rank 2)
@pytest.mark.parametrize('name', golden_names('baseline'))
def test_baseline_against_reference(name):
    """nw_baseline (device fp64 statistics + elementwise op) against the reference's
    Baseline outputs (base.py:18-68); axis 0 of an (F, N) power array is frequency.
    Tolerance: 1e-13 relative (fp64), 2e-6 (fp32 data: numpy's float32 pairwise mean vs
    the device's fp64 mean rounded to fp32)."""
    g = load_golden(name)
    m = g['meta']
    t = 1e-13 if m['dtype'] == 'float64' else 2e-6
    b = nw.Baseline(g['wave'], m['sfreq'], m['start'], m['stop'])
    assert b.baseline.shape == g['baseline'].shape
    assert abs(b.basemean - float(g['basemean'])) <= t * abs(float(g['basemean']))
    for op in O.BASELINE_OPS:
        got = getattr(b, op)()
        assert got.dtype == g[op].dtype and got.shape == g[op].shape, op
        assert rel_err(got, g[op]) <= t, (op, rel_err(got, g[op]))


def test_baseline_device_tensor_and_edges():
    torch = pytest.importorskip('torch')
    rng = np.random.default_rng(3)
    w = rng.uniform(0.5, 2.0, (64, 4096))
    ref = O.baseline(w, 100., 0.1, 0.3, 'zlog')
    wt = torch.from_numpy(w).cuda()
    got = nw.Baseline(wt, 100., 0.1, 0.3).zlog()
    assert got.is_cuda and rel_err(got.cpu().numpy(), ref) <= 1e-13
    # negative start: a Python slice from the end, as in the reference
    assert rel_err(nw.Baseline(w, 100., -0.2, 0.6).mean(), O.baseline(w, 100., -0.2, 0.6, 'mean')) <= 1e-13
    # empty baseline: mean of nothing is NaN
    with np.errstate(all='ignore'):
        assert np.all(np.isnan(nw.Baseline(w, 100., 0.3, 0.1).ratio()))


# ------------------------------------------------------------------ Normal-mode tables on device
@pytest.mark.parametrize('interpolate', [False, True])
@pytest.mark.parametrize('kind', ['mexican_hat', 'haar'])
def test_device_normal_table_equals_host_table(kind, interpolate):
    """MexicanHat / Haar rows built on the device (time rows + rocFFT + |Re|+i|Im|,
    base.py:249-256) equal the host-built rows of a plugin subclass with the same
    formula (ragged lengths included), and so do the CWTs through them."""
    base = CLASSES[kind]

    class HostBuilt(base):
        def formula(self, tc, freq=1):
            return base.formula(self, tc, freq)

    freqs = np.array([0.5, 3., 7.5, 20., 47., 101.])
    dev, host = base(1000, interpolate=interpolate), HostBuilt(1000, interpolate=interpolate)
    assert dev._device_normal() is not None and host._device_normal() is None
    rd = dev.make_fft_wavelets(freqs, 2.048)
    rh = host.make_fft_wavelets(freqs, 2.048)
    assert [r.shape for r in rd] == [r.shape for r in rh]
    for a, b in zip(rd, rh):
        assert np.max(np.abs(a - b)) <= 1e-13 * max(1.0, np.max(np.abs(b)))
    x = synth(1, 2048, 17)[0].astype(np.float64)
    assert rel_err(dev.cwt(x, freqs), host.cwt(x, freqs)) <= 1e-13


# ------------------------------------------------------------------ time-domain wavelets (§8f rank 4)
WAVELET_CASES = {'morse': (nw.Morse, dict(sfreq=1000)), 'morse_b': (nw.Morse, dict(sfreq=500, b=10., r=2.)),
                 'shannon': (nw.Shannon, dict(sfreq=1000)), 'morlet': (nw.Morlet, dict(sfreq=1000)),
                 'morlet_gabor': (nw.Morlet, dict(sfreq=1000, gabor=True)),
                 'mexican_hat': (nw.MexicanHat, dict(sfreq=1000)), 'haar': (nw.Haar, dict(sfreq=1000))}


@pytest.mark.parametrize('name', golden_names('wavelets'))
def test_make_wavelets_against_reference(name):
    """make_wavelets (base.py:346-376) on the device (nw_make_wavelets: spectrum + rocFFT
    inverse + conj-flip slice, or the time-domain formula) against the reference's rows:
    same ragged lengths and dtypes, values within 1e-13 of each row's peak."""
    g = load_golden(name)
    cls, kw = WAVELET_CASES[g['meta']['case']]
    w = cls(**kw)
    assert w._device_wavelet_spec() is not None
    rows = w.make_wavelets(list(g['freqs']))
    ref = np.split(g['rows'], np.cumsum(g['lens'])[:-1])
    assert [r.shape for r in rows] == [r.shape for r in ref]
    assert str(rows[0].dtype) == g['meta']['dtype']
    for got, want in zip(rows, ref):
        assert np.max(np.abs(got - want)) <= 1e-13 * max(1e-300, np.max(np.abs(want)))
    single = w.make_wavelet(float(g['freqs'][2]))
    np.testing.assert_array_equal(single, rows[2])

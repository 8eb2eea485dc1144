"""GPU parity at the shapes the bench lines time (BASELINE.json configs C2-C5).

- C3 as benchmarked: Morse POWER (and abs) at N = 4096, F = 256 (freqs 1..256), fp32, chunks
  of >= 2 signals so ``nw_fused_pair_kernel`` runs with every pass-0 pruning variant
  (reference: base.py:409-443 power/abs over base.py:378-407 cwt);
- the same at N = 16384 (``nw_fused_kernel``, E = 32), power;
- Shannon fp32 at N = 2^24 with 16 scales (the repeated-row path: one computed row and
  ``k_expand_rows``; wavelets.py:256-262);
- the reference's own outputs at the benchmark lengths (tests/golden/long_*.npz, made by
  tests/golden/make_golden_long.py): N = 16384 (C2 Morlet, C4 Morse), 2^17 and 2^24 (C5).

Tolerances as in test_gpu_parity.py: fp64 1e-12 of max|ref|; fp32 1e-5 (x2 for |.|^2) at
N <= 16384, 1e-4 at N >= 2^17.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, long_signal, x_digest
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


def plan_for(n, freqs, dtype, max_batch, kind='morse', params=(17.5, 3.), **kw):
    g = L.trans_grid(n / 1000., 1000., False)
    p = nw.Plan(n, len(freqs), dtype, max_batch=max_batch, **kw)
    p.set_wavelet(kind, list(params), np.asarray(freqs, dtype=np.float64), g)
    return p


def max_err(got, ref):
    return np.max(np.abs(got - ref)) / np.max(np.abs(ref))


@pytest.mark.parametrize('n,kernel', [(4096, 'nw_fused_pair_kernel'), (16384, 'nw_fused_kernel')])
@pytest.mark.parametrize('out_kind', ['power', 'abs'])
def test_bench_shape_power_abs_against_oracle(n, kernel, out_kind):
    """Every one of the 256 scales of 4 signals (C3 / C4 scale list) in chunks of 2 and 4
    signals, against the oracle's |cwt|^2 / |cwt|; the kernel that ran is the bench's."""
    S, freqs = 4, np.arange(1, 257, dtype=np.float64)
    x = synth(S, n, seed=n + 7)
    ref = np.stack([O.cwt('morse', x[s].astype(np.float64), freqs) for s in range(S)])
    ref = np.abs(ref) ** 2 if out_kind == 'power' else np.abs(ref)
    for chunk in (2, 4):
        plan = plan_for(n, freqs, 'float32', chunk)
        got = plan.execute(x, out_kind=out_kind)
        st = plan.stats()
        assert st['engine'] == 'fused' and L.KERNEL_NAMES[st['kernel']] == kernel, st
        assert got.shape == (S, 256, n) and got.dtype == np.float32
        err = max_err(got, ref)
        assert err <= (2e-5 if out_kind == 'power' else 1e-5), (chunk, err)
        # each row against its own scale: the pruned (low-f) rows are tiny next to the max
        for f in (0, 1, 3, 10, 40, 100, 255):
            r = ref[:, f]
            assert np.max(np.abs(got[:, f] - r)) <= 3e-5 * np.max(np.abs(r)) + 1e-30, (chunk, f)


def test_c3_power_cwt_consistent_on_pair_kernel():
    """C3's power output equals |cwt|^2 of the same kernel family's complex output."""
    n, S, freqs = 4096, 8, np.arange(1, 257, dtype=np.float64)
    x = synth(S, n, seed=99)
    plan = plan_for(n, freqs, 'float32', 8)
    c = plan.execute(x, out_kind='cwt').astype(np.complex128)
    p = plan.execute(x, out_kind='power')
    assert max_err(p, np.abs(c) ** 2) <= 4e-7


def test_c5_shannon_fp32_16_scales():
    """C5's Shannon line at 2^24 (fp32): 16 scales; Shannon ignores the freq, so one row is
    computed and copied 15 times; every row against the oracle (tolerance 1e-4 at 2^24)."""
    n, F = 1 << 24, 16
    freqs = np.linspace(0.5, 250, 512)[::32]
    x = synth(1, n, seed=5)[0]
    w = nw.Shannon(1000, dtype='float32')
    out = w.cwt(x, freqs)
    assert out.shape == (F, n) and out.dtype == np.complex64
    ref = O.cwt('shannon', x.astype(np.float64), freqs[:2])[0]
    for f in range(F):
        assert max_err(out[f], ref) <= 1e-4, f
    assert all(np.array_equal(out[f], out[0]) for f in range(1, F))


LONG = golden_names('long_')


@pytest.mark.parametrize('dtype', ['float64', 'float32'])
@pytest.mark.parametrize('name', LONG)
def test_reference_outputs_at_benchmark_lengths(name, dtype):
    """The drop-in cwt against the reference run at the benchmark lengths: the 2048 sampled
    points of every scale, and each row's sum and energy (every output point)."""
    g = load_golden(name)
    m = g['meta']
    n = m['n']
    x = long_signal(n, m['seed'])
    assert x_digest(x) == m['x_sha256']
    cls = {'morse': nw.Morse, 'morlet': nw.Morlet}[m['kind']]
    out = cls(m['sfreq'], dtype=dtype).cwt(x.astype(dtype), g['freqs'])
    assert out.shape == (len(g['freqs']), n)
    tol = 1e-12 if dtype == 'float64' else (1e-5 if n <= 16384 else 1e-4)
    ref = g['out_at']
    assert max_err(out[:, g['pos']], ref) <= tol
    o = out.astype(np.complex128)
    # per-row sum: n point errors of size <= tol * rms(row) add like a random walk (tol *
    # sqrt(n) * rms = tol * sqrt(row_energy)), plus a relative error of the sum itself (a
    # uniform scale error of the row); the bound does not grow with n beyond sqrt(n)
    s_bound = tol * (np.sqrt(g['row_energy']) + np.abs(g['row_sum']))
    assert np.all(np.abs(o.sum(axis=1) - g['row_sum']) <= s_bound)
    np.testing.assert_allclose((np.abs(o) ** 2).sum(axis=1), g['row_energy'], rtol=4 * tol)


@pytest.mark.parametrize('n', [1201, 4097])
def test_mne_lengths_power_all_scales(n):
    """MNE epoch lengths (tmin..tmax inclusive) at the C3 scale list: the chirp-z form, Morse
    power at all 256 scales of 4 signals in chunks of 2 (tolerance 2e-5 x2 for |.|^2, as
    test_gpu_chirp.py)."""
    S, freqs = 4, np.arange(1, 257, dtype=np.float64)
    x = synth(S, n, seed=n)
    ref = np.abs(np.stack([O.cwt('morse', x[s].astype(np.float64), freqs) for s in range(S)])) ** 2
    plan = plan_for(n, freqs, 'float32', 2)
    got = plan.execute(x, out_kind='power')
    assert L.KERNEL_NAMES[plan.stats()['kernel']] == 'nw_chirp_kernel'
    assert max_err(got, ref) <= 4e-5


@pytest.mark.parametrize('out_kind', ['power', 'abs'])
def test_c2_morlet_outputs_all_scales(out_kind):
    """C2's wavelet (Morlet sigma = 7) at N = 16384, freqs 1..128, |.| and |.|^2 outputs."""
    S, n, freqs = 2, 16384, np.arange(1, 129, dtype=np.float64)
    x = synth(S, n, seed=77)
    ref = np.stack([O.cwt('morlet', x[s].astype(np.float64), freqs) for s in range(S)])
    ref = np.abs(ref) ** 2 if out_kind == 'power' else np.abs(ref)
    plan = plan_for(n, freqs, 'float32', 2, kind='morlet', params=(7.0, 0.0))
    got = plan.execute(x, out_kind=out_kind)
    assert max_err(got, ref) <= (2e-5 if out_kind == 'power' else 1e-5)


@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_interpolate_at_n16384(dtype):
    """interpolate=True (base.py:107-123: the wavelet and X above int(N/2) zeroed) at C4's
    length through the drop-in class, against the oracle."""
    n, freqs = 16384, np.array([1., 17., 90., 256., 400.])
    x = synth(1, n, seed=5)[0].astype(np.float64)
    ref = O.cwt('morse', x, freqs, interpolate=True)
    got = nw.Morse(1000, interpolate=True, dtype=dtype).cwt(x.astype(dtype), freqs)
    assert max_err(got, ref) <= (1e-12 if dtype == 'float64' else 1e-5)


def oracle_stack(x, freqs):
    """O.cwt of every signal (fp64, the reference's arithmetic), (S, F, n) complex128."""
    return np.stack([O.cwt('morse', x[s].astype(np.float64), freqs) for s in range(x.shape[0])])


def itc_within_contract(got, o):
    """INTEGRATION.md's fp32 ITC contract against the oracle's ITC of the same signals:
    |d| <= 2e-5 wherever every epoch's |cwt| is >= 0.1 of its scale row's max, <= 1e-3
    everywhere.  Returns (worst well-conditioned |d|, worst |d|)."""
    mag = np.abs(o)
    ref = np.abs(np.mean(o / mag, axis=0))
    d = np.abs(got.astype(np.float64) - ref)
    good = np.all(mag >= 0.1 * mag.max(axis=-1, keepdims=True), axis=0)
    return float(d[good].max()) if good.any() else 0.0, float(d.max())


@pytest.mark.parametrize('n', [1024, 2048, 4096, 8192, 16384])
def test_power_mean_fused_partials(n):
    """fp32 epoch power sums at the fused sizes: the kernel sums |y|^2 over each block of 8
    signals in fp64 (kOutPSum: the signal-pair kernel at n <= 4096, nw_fused_kernel above)
    and the accumulator adds the fp64 partials.  Every point against the oracle's mean power
    of the same signals (2e-5 of max: |y|^2 of the fp32 contract's 1e-5), the mean equal to
    the plan's own sum / S (one fp32 rounding), ragged chunks (37 signals in chunks of 16 ->
    16, 16, 5) and chunk-size independence (the same fp64 additions of the same fp32 values,
    regrouped: 1e-13).  The per-signal power output runs another kernel, so it is held to the
    oracle too, not to the sums (their fp32 roundings differ by code generation)."""
    S, freqs = 37, np.arange(1, 257, dtype=np.float64)
    x = synth(S, n, seed=n + 3)
    plan = plan_for(n, freqs, 'float32', 16)
    pm = plan.execute(x, out_kind='power_mean')
    pair = n <= 4096                     # the signal-pair kernel
    assert L.KERNEL_NAMES[plan.stats()['kernel']] == ('nw_fused_pair_kernel' if pair else 'nw_fused_kernel')
    assert pm.shape == (256, n) and pm.dtype == np.float32
    ps = plan.execute(x, out_kind='power_sum')
    assert ps.dtype == np.float64
    assert np.max(np.abs(pm - ps / S) / (ps / S + 1e-30 * ps.max() / S)) <= 1.2e-7
    other = plan_for(n, freqs, 'float32', 5)                  # chunks 5, 5, ... , 2
    np.testing.assert_allclose(other.execute(x, out_kind='power_sum'), ps, rtol=1e-13)
    orc = np.zeros((256, n))
    for s in range(S):                                        # the oracle's mean power, row by row
        orc += np.abs(O.cwt('morse', x[s].astype(np.float64), freqs)) ** 2
    orc /= S
    assert max_err(pm, orc) <= 2e-5
    pw = plan.execute(x[:4], out_kind='power')                # the per-signal output, same contract
    o4 = np.abs(oracle_stack(x[:4], freqs[::17])) ** 2
    assert max_err(pw[:, ::17], o4) <= 2e-5


@pytest.mark.parametrize('n', [1024, 4096, 8192])
def test_itc_fused_partials(n):
    """ITC (mneutils.py:62-71) at the fused sizes: the kernel sums y / |y| (fp64, k_accumulate's
    formula) over each block of 8 signals.  Every point against the oracle's ITC of the same
    signals under INTEGRATION.md's fp32 contract (2e-5 where every epoch's |cwt| >= 0.1 of its
    row's max, 1e-3 everywhere), ITC = |phase_sum| / S of the same plan, and chunk-size
    independent (phase_sum 1e-13)."""
    S, freqs = 21, np.arange(1, 257, dtype=np.float64)
    x = synth(S, n, seed=n + 11)
    plan = plan_for(n, freqs, 'float32', 8)
    itc = plan.execute(x, out_kind='itc')
    assert L.KERNEL_NAMES[plan.stats()['kernel']] == 'nw_fused_kernel'
    assert itc.shape == (256, n) and itc.dtype == np.float32
    ph = plan.execute(x, out_kind='phase_sum')
    assert ph.dtype == np.complex128
    assert np.max(np.abs(itc - np.abs(ph) / S)) <= 1.2e-7
    other = plan_for(n, freqs, 'float32', 3)
    np.testing.assert_allclose(other.execute(x, out_kind='phase_sum'), ph, rtol=1e-13, atol=1e-13 * S)
    for f0 in range(0, 256, 64):                              # the oracle in slices of 64 scales
        good, worst = itc_within_contract(itc[f0:f0 + 64], oracle_stack(x, freqs[f0:f0 + 64]))
        assert good <= 2e-5 and worst <= 1e-3, (f0, good, worst)


@pytest.mark.parametrize('n', [1024, 2048, 4096, 8192, 16384])
def test_fp64_fused_epoch_partials(n):
    """fp64 (the drop-in's default dtype, the reference's complex128) epoch reductions
    (mneutils.py:42-71): the kernel sums |y|^2 (ITC: y / hypot(y), the accumulator's formula)
    over each block of 8 signals in fp64 -- at n <= 4096 on the output kernel's E = 16, at
    n = 8192 on an E = 16 instantiation beside the E = 32 output kernel; n = 16384 keeps the
    chunk path.  power_sum equals the sum of the same plan's per-signal power output (1e-13
    where the same kernel computes both, else 1e-12); chunk-size independent; ITC against the
    same plan's materialised cwt; both against the oracle (fp64 contract: 1e-12 of max, ITC
    1e-10 absolute)."""
    same = n <= 4096
    S, freqs = 21, np.arange(1, 257, dtype=np.float64)
    x = synth(S, n, seed=n + 5).astype(np.float64)
    plan = plan_for(n, freqs, 'float64', 8)
    pw = plan.execute(x, out_kind='power')
    c = plan.execute(x, out_kind='cwt')
    ps = plan.execute(x, out_kind='power_sum')
    assert L.KERNEL_NAMES[plan.stats()['kernel']] == 'nw_fused_kernel'
    np.testing.assert_allclose(ps, pw.sum(axis=0), rtol=1e-13 if same else 1e-12)
    pm = plan.execute(x, out_kind='power_mean')
    assert pm.dtype == np.float64 and pm.shape == (256, n)
    np.testing.assert_allclose(pm, pw.mean(axis=0), rtol=1e-13 if same else 1e-12)
    other = plan_for(n, freqs, 'float64', 3)                  # chunks 3, 3, ..., 3
    np.testing.assert_allclose(other.execute(x, out_kind='power_sum'), ps, rtol=1e-13)
    itc = plan.execute(x, out_kind='itc')
    ref_itc = np.abs(np.mean(c / np.abs(c), axis=0))
    assert np.max(np.abs(itc - ref_itc)) <= (1e-13 if same else 1e-10)
    ph = other.execute(x, out_kind='phase_sum')
    np.testing.assert_allclose(ph, plan.execute(x, out_kind='phase_sum'), rtol=1e-13, atol=1e-13 * S)
    o = np.stack([O.cwt('morse', x[s], freqs[::51]) for s in range(S)])
    assert max_err(pm[::51], np.mean(np.abs(o) ** 2, axis=0)) <= 1e-12
    assert np.max(np.abs(itc[::51] - np.abs(np.mean(o / np.abs(o), axis=0)))) <= 1e-10

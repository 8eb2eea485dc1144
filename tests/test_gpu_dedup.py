"""GPU parity of repeated-row execution (nw_plan dedup, include/ninwave.h NW_NO_DEDUP).

When at most half of the F wavelet rows are distinct -- Shannon's spectrum ignores the
frequency (reference wavelets.py:256-262), or a freq list repeats values -- the engines
compute the distinct rows once and k_expand_rows copies them to every repeating scale.
A row's output depends only on its W row and the signal, so the result must equal the
row-by-row computation BIT FOR BIT (assert_array_equal against a NW_NO_DEDUP plan on the
same engine), and the oracle within the usual tolerances (fp64 1e-12, fp32 1e-5 of
max|ref|, |.|^2 twice that).
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


def rel_err(got, ref):
    return np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-300)


def plan_pair(n, F, dtype, kind, params, freqs, engine, max_batch=4, interpolate=False):
    g = L.trans_grid(n / 1000., 1000., interpolate)
    out = []
    for dedup in (True, False):
        p = nw.Plan(n, F, dtype, max_batch=max_batch, engine=engine, interpolate=interpolate, dedup=dedup)
        p.set_wavelet(kind, list(params), np.asarray(freqs, dtype=np.float64), g)
        out.append(p)
    return out


# (n, engine): rocFFT engine (odd n too), the one-pass fused kernel, the two-pass form
CASES = [(1000, 'rocfft'), (301, 'rocfft'), (1000, None), (301, None), (4096, 'fused'), (16384, 'fused'),
         (1 << 15, 'fused')]   # None: the auto engine, i.e. the chirp-z form at 1000 and 301


@pytest.mark.parametrize('n,engine', CASES)
@pytest.mark.parametrize('dtype', ['float32', 'float64'])
@pytest.mark.parametrize('out', ['cwt', 'abs', 'power'])
def test_shannon_rows_computed_once_bit_exact(n, engine, dtype, out):
    F, S = 12, 5                                   # 2 chunks of max_batch 4 (+ a ragged one)
    x = synth(S, n, 31).astype(dtype)
    freqs = np.linspace(1., 60., F)
    a, b = plan_pair(n, F, dtype, 'shannon', [], freqs, engine)
    ya = a.execute(x, out_kind=out)
    yb = b.execute(x, out_kind=out)
    sa, sb = a.stats(), b.stats()
    assert sa['unique_rows'] == 1 and sa['launches_expand'] >= 2
    assert sb['unique_rows'] == F and sb['launches_expand'] == 0
    np.testing.assert_array_equal(ya, yb)
    for f in range(1, F):                           # every scale row is the same row
        np.testing.assert_array_equal(ya[:, f], ya[:, 0])
    ref = np.stack([O.cwt('shannon', x[s].astype(np.float64), freqs) for s in range(S)])
    if out == 'abs':
        ref = np.abs(ref)
    elif out == 'power':
        ref = np.abs(ref) ** 2
    t = (1e-12 if dtype == 'float64' else 3e-5) * (2 if out == 'power' else 1)
    assert rel_err(ya, ref) <= t


@pytest.mark.parametrize('n,engine', [(2048, 'rocfft'), (2048, 'fused'), (1 << 15, 'fused')])
@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_repeated_freqs_morse_and_morlet(n, engine, dtype):
    """Repeated freqs: 3 distinct rows among 8, scattered; bit-exact against the
    row-by-row plan and close to the oracle."""
    freqs = np.array([5., 40., 5., 5., 120., 40., 5., 120.])
    F, S = len(freqs), 3
    x = synth(S, n, 32).astype(dtype)
    for kind, params in (('morse', (17.5, 3.)), ('morlet', (7., 0.))):
        a, b = plan_pair(n, F, dtype, kind, params, freqs, engine)
        ya = a.execute(x, out_kind='cwt')
        yb = b.execute(x, out_kind='cwt')
        assert a.stats()['unique_rows'] == 3
        np.testing.assert_array_equal(ya, yb)
        kw = {'b': params[0], 'r': params[1]} if kind == 'morse' else {'sigma': params[0], 'gabor': False}
        ref = np.stack([O.cwt(kind, x[s].astype(np.float64), freqs, **kw) for s in range(S)])
        assert rel_err(ya, ref) <= (1e-12 if dtype == 'float64' else 3e-5)


def test_few_repeats_keep_row_by_row():
    """More than half the rows distinct: no dedup (the copies would cost more)."""
    n = 4096
    freqs = np.array([5., 5., 6., 7.])             # 3 distinct of 4
    a, _ = plan_pair(n, 4, 'float32', 'morse', (17.5, 3.), freqs, None)
    x = synth(2, n, 33)
    a.execute(x, out_kind='power')
    st = a.stats()
    assert st['unique_rows'] == 4 and st['launches_expand'] == 0


@pytest.mark.parametrize('engine', ['rocfft', 'fused'])
@pytest.mark.parametrize('out', ['power_mean', 'itc', 'power_sum', 'phase_sum'])
def test_reductions_with_repeated_rows(engine, out):
    n, F, S = 2048, 6, 9
    x = synth(S, n, 34)
    freqs = np.full(F, 10.)
    a, b = plan_pair(n, F, 'float32', 'shannon', [], freqs, engine)
    np.testing.assert_array_equal(a.execute(x, out_kind=out), b.execute(x, out_kind=out))
    a2, b2 = plan_pair(n, F, 'float32', 'morse', (17.5, 3.), freqs, engine)
    np.testing.assert_array_equal(a2.execute(x, out_kind=out), b2.execute(x, out_kind=out))


def test_table_rows_repeat_by_content():
    """User table rows (NW_TABLE) are compared by contents: rows 0, 2, 3 equal, 1 and 4
    equal -> 2 distinct of 5 (row_len ragged in one case)."""
    n, S = 1024, 3
    rng = np.random.default_rng(5)
    r0 = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    r1 = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    table = np.stack([r0, r1, r0, r0, r1])
    g = L.nw_grid(1.0, n, n)
    x = synth(S, n, 35)
    for dtype in ('float32', 'float64'):
        outs = []
        for dedup in (True, False):
            p = nw.Plan(n, 5, dtype, max_batch=2, engine='rocfft', dedup=dedup)
            p.set_wavelet('table', [], np.arange(1., 6.), g, table=table)
            outs.append((p.execute(x.astype(dtype), out_kind='cwt'), p.stats()['unique_rows']))
        assert outs[0][1] == 2 and outs[1][1] == 5
        np.testing.assert_array_equal(outs[0][0], outs[1][0])
    # ragged: same contents, different row_len -> different rows (3 distinct of 7)
    table7 = np.stack([r0, r1, r0, r0, r1, r0, r0])
    outs = []
    for dedup in (True, False):
        p = nw.Plan(n, 7, 'float32', max_batch=2, engine='rocfft', dedup=dedup)
        p.set_wavelet('table', [], np.arange(1., 8.), g, table=table7, row_len=[n, n, n, n - 8, n, n, n])
        outs.append((p.execute(x, out_kind='cwt'), p.stats()['unique_rows']))
    assert outs[0][1] == 3 and outs[1][1] == 7
    np.testing.assert_array_equal(outs[0][0], outs[1][0])


def test_device_tensor_output_with_repeated_rows():
    torch = pytest.importorskip('torch')
    n, F, S = 16384, 16, 4
    x = synth(S, n, 36)
    a, b = plan_pair(n, F, 'float32', 'shannon', [], np.arange(1., F + 1), 'fused', max_batch=S)
    xt = torch.from_numpy(x).cuda()
    oa = torch.empty((S, F, n), dtype=torch.complex64, device='cuda')
    ob = torch.empty_like(oa)
    a.execute(xt, oa, out_kind='cwt')
    b.execute(xt, ob, out_kind='cwt')
    a.sync()
    b.sync()
    assert torch.equal(oa, ob)


def test_class_api_shannon_and_repeats_match_oracle():
    """The drop-in classes take the dedup path by default."""
    n = 1000
    x = synth(1, n, 37)[0].astype(np.float64)
    freqs = [3., 3., 3., 3.]
    got = nw.Shannon(1000).cwt(x, freqs)
    ref = O.cwt('shannon', x, freqs)
    assert rel_err(got, ref) <= 1e-12
    got = nw.Morse(1000).cwt(x, freqs)
    ref = O.cwt('morse', x, freqs)
    assert rel_err(got, ref) <= 1e-12

"""GPU parity of scale-sharded execution (nw_execute_multi_scales): plans that
each hold a contiguous slice of the scale list, one host thread each, write their rows of
the (S, F, n) / (F, n) output.  A scale row depends only on its W row and the signal, so
the result must equal the single-plan result BIT FOR BIT; the slices run here on device 0
(a one-GPU box), the same code path as one device per slice.
"""
import numpy as np
import pytest

from oracle import nw_oracle as O

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402
from ninwavelets_amd.dist import shard  # noqa: E402


def synth(S, n, seed, sfreq=1000.):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sfreq
    fc = rng.uniform(1, 100, (S, 1))
    ph = rng.uniform(0, 2 * np.pi, (S, 1))
    return (np.sin(2 * np.pi * fc * t + ph) + 0.1 * rng.standard_normal((S, n))).astype(np.float32)


def plans_for(n, freqs, dtype, engine, kind, params, world, max_batch=2):
    g = L.trans_grid(n / 1000., 1000., False)
    out = []
    for r in range(world):
        f0, f1 = shard(len(freqs), r, world)
        p = nw.Plan(n, f1 - f0, dtype, max_batch=max_batch, engine=engine)
        p.set_wavelet(kind, list(params), freqs[f0:f1], g)
        out.append(p)
    return out


@pytest.mark.parametrize('n,engine', [(1000, 'rocfft'), (1000, None), (4096, None), (1 << 15, None)])
@pytest.mark.parametrize('dtype', ['float32', 'float64'])
@pytest.mark.parametrize('world', [2, 3])
def test_scale_slices_equal_single_plan(n, engine, dtype, world):
    freqs = np.linspace(2., 150., 10)
    S = 3
    x = synth(S, n, 41).astype(dtype)
    single = plans_for(n, freqs, dtype, engine, 'morse', (17.5, 3.), 1, max_batch=4)[0]
    split = plans_for(n, freqs, dtype, engine, 'morse', (17.5, 3.), world)
    for out in ('cwt', 'power', 'power_mean', 'itc', 'power_sum', 'phase_sum'):
        ref = single.execute(x, out_kind=out)
        got = nw.execute_multi(split, x, out_kind=out, shard='scales')
        assert got.shape == ref.shape and got.dtype == ref.dtype, out
        np.testing.assert_array_equal(got, ref, err_msg=out)
    one = nw.execute_multi(split, x[:1], out_kind='cwt', shard='scales')     # one signal: C5's case
    np.testing.assert_array_equal(one, single.execute(x[:1], out_kind='cwt'))


def test_scale_slices_validate_plans():
    a = nw.Plan(1024, 3, 'float32')
    b = nw.Plan(2048, 3, 'float32')
    g = L.trans_grid(1.024, 1000., False)
    a.set_wavelet('morse', [17.5, 3.], np.array([1., 2., 3.]), g)
    b.set_wavelet('morse', [17.5, 3.], np.array([4., 5., 6.]), L.trans_grid(2.048, 1000., False))
    with pytest.raises(ValueError):
        nw.execute_multi([a, b], synth(1, 1024, 1), shard='scales')


def test_class_api_one_signal_on_several_devices_shards_scales():
    """devices=[0, 0]: one signal is split by scales (two plans, two host threads) and
    matches the single-device call bit for bit, and the oracle within 1e-12 (fp64)."""
    x = synth(1, 4096, 42)[0].astype(np.float64)
    freqs = np.arange(1., 41.)
    w2 = nw.Morse(1000, devices=[0, 0])
    got = w2.cwt(x, freqs)
    ref = nw.Morse(1000).cwt(x, freqs)
    np.testing.assert_array_equal(got, ref)
    assert len(w2._plans) == 2
    o = O.cwt('morse', x, freqs)
    assert np.max(np.abs(got - o)) <= 1e-12 * np.max(np.abs(o))
    np.testing.assert_array_equal(nw.MexicanHat(1000, devices=[0, 0]).power(x, freqs[:8]),
                                  nw.MexicanHat(1000).power(x, freqs[:8]))

"""GPU tests of the multi-plan paths and the torch stream contract (the batching
they shard is the per-epoch loop of the reference, /root/reference/ninwavelets/mneutils.py:39).
Several plans on device 0 stand in for several GPUs on the 1-GPU lease: every plan has its
own stream and host thread, exactly as on 8 devices.  Sharded results must equal the single
plan bit for bit (the same kernels run on the same signals)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402

torch = pytest.importorskip('torch')


def synth(S, n, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 1000.
    fc = rng.uniform(1, 100, (S, 1))
    return (np.sin(2 * np.pi * fc * t) + 0.1 * rng.standard_normal((S, n))).astype(np.float32)


def plan_for(n, freqs, dtype='float32', max_batch=8):
    g = L.trans_grid(n / 1000., 1000., False)
    p = nw.Plan(n, len(freqs), dtype, device=0, max_batch=max_batch)
    p.set_wavelet('morse', [17.5, 3.], np.asarray(freqs, dtype=np.float64), g)
    return p


@pytest.mark.parametrize('n,out_kind', [(4096, 'power'), (16384, 'cwt'), (1201, 'cwt')])
def test_execute_multi_device_is_exact(n, out_kind):
    """nw_execute_multi_device: per-plan device inputs / outputs (uneven shards) equal one plan."""
    freqs = np.arange(1., 33.)
    x = synth(11, n, n)
    single = plan_for(n, freqs).execute(x, out_kind=out_kind)
    cuts = [0, 5, 8, 11]
    plans = [plan_for(n, freqs, max_batch=4) for _ in range(3)]
    xs = [torch.from_numpy(x[a:b]).cuda() for a, b in zip(cuts, cuts[1:])]
    odt = torch.complex64 if out_kind == 'cwt' else torch.float32
    outs = [torch.empty((b - a, len(freqs), n), dtype=odt, device='cuda') for a, b in zip(cuts, cuts[1:])]
    nw.execute_multi_device(plans, xs, outs, out_kind=out_kind)
    got = np.concatenate([o.cpu().numpy() for o in outs])
    np.testing.assert_array_equal(got, single)


def test_execute_multi_device_reductions():
    n, freqs = 4096, np.arange(2., 26.)
    x = synth(9, n, 3)
    ref = plan_for(n, freqs).execute(x, out_kind='power_mean')
    plans = [plan_for(n, freqs, max_batch=4) for _ in range(2)]
    xs = [torch.from_numpy(x[:4]).cuda(), torch.from_numpy(x[4:]).cuda()]
    outs = [torch.empty((len(freqs), n), dtype=torch.float32, device='cuda'), None]
    got = nw.execute_multi_device(plans, xs, outs, out_kind='power_mean').cpu().numpy()
    assert np.max(np.abs(got - ref)) <= 1e-6 * np.max(np.abs(ref))


def test_repeated_plan_is_rejected():
    p = plan_for(1024, np.arange(1., 5.))
    with pytest.raises(Exception):
        nw.execute_multi([p, p], synth(4, 1024, 1), out_kind='cwt')


@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_batch_on_repeated_devices_is_exact(dtype):
    """devices=[0, 0] with a batch: one plan per shard (plans are not reentrant), and the
    result equals the single-device call bit for bit (advisor finding, round 1)."""
    n, freqs = 4096, np.arange(1., 17.)
    x = synth(4, n, 8).astype(dtype)
    one = nw.Morse(1000, dtype=dtype).cwt_batch(x, freqs)
    two = nw.Morse(1000, dtype=dtype, devices=[0, 0]).cwt_batch(x, freqs)
    np.testing.assert_array_equal(two, one)


def test_scale_shards_never_empty():
    """5 scales over 4 plans (one signal): balanced slices 2/1/1/1, no empty plan."""
    n, freqs = 4096, [3., 7., 11., 19., 40.]
    x = synth(1, n, 4)[0].astype(np.float64)
    one = nw.Morse(1000).cwt(x, freqs)
    four = nw.Morse(1000, devices=[0, 0, 0, 0]).cwt(x, freqs)
    np.testing.assert_array_equal(four, one)


def test_torch_stream_ordering_without_sync():
    """Input produced by a torch kernel just before the call and output consumed by a torch
    kernel right after it, with no explicit synchronisation: the plan orders itself against
    torch's current stream on both sides ('Device tensors and streams')."""
    n, S, freqs = 16384, 16, np.arange(1., 65.)
    plan = plan_for(n, freqs, max_batch=S)
    g = torch.Generator(device='cuda')
    g.manual_seed(5)
    for _ in range(3):
        x = torch.randn((S, n), generator=g, device='cuda', dtype=torch.float32) * 3.0   # torch kernels
        out = torch.empty((S, len(freqs), n), dtype=torch.float32, device='cuda')
        plan.execute(x, out, out_kind='power')
        s = out.sum(dim=(1, 2))                                   # torch kernel on the output, no sync
        ref = plan.execute(x.cpu().numpy(), out_kind='power')    # host path (synchronous)
        np.testing.assert_allclose(s.cpu().numpy(), ref.astype(np.float64).sum(axis=(1, 2)), rtol=1e-4)
        del x, out                                                # memory back to the caching allocator

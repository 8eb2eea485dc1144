"""The drop-in classes' plan cache is bounded by the device bytes its plans hold
(nw_stats.device_bytes): plans are keyed on (n, batch, device, ...), so a session of varying
epoch lengths and batch sizes would otherwise keep every plan's buffers alive.  Evicted plans
are destroyed (their HBM freed); results are unchanged (reference: base.py:378-407 returns a
new array per call, whatever came before)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402


def synth(S, n, seed):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((S, n)).astype(np.float32)


def test_plan_cache_stays_under_its_byte_cap():
    freqs = np.arange(1, 33, dtype=np.float64)
    w = nw.Morse(1000, dtype='float32')
    cap = 8 << 20
    w.plan_cache_bytes = cap
    seen, evicted = 0, False
    for n in (1024, 2048, 1201):
        for S in (1, 2, 3, 5, 9, 17):
            x = synth(S, n, seed=n + S)
            got = w.cwt_batch(x, freqs)
            seen += 1
            held = w.plan_cache_device_bytes()
            # the current call's plan always stays; everything older only within the cap
            assert held <= cap or len(w._plans) == 1, (n, S, held, len(w._plans))
            evicted |= len(w._plans) < seen
            fresh = nw.Morse(1000, dtype='float32')
            fresh._cache = w._cache                   # the same (unkeyed) wavelet cache
            np.testing.assert_array_equal(got, fresh.cwt_batch(x, freqs))
            for p in fresh._plans.values():
                p.close()
    assert evicted
    # a plan's device bytes cover at least its input, spectrum and output chunk buffers
    st = next(iter(w._plans.values())).stats()
    assert st['device_bytes'] >= 17 * 1201 * 4


def test_default_cap_keeps_plans_of_a_session():
    freqs = np.arange(1, 9, dtype=np.float64)
    w = nw.Morlet(1000, dtype='float64')
    for S in (1, 4, 16):
        w.cwt_batch(synth(S, 2048, S).astype(np.float64), freqs)
    assert len(w._plans) == 3 and w.plan_cache_device_bytes() <= w.plan_cache_bytes


def test_pooled_host_results_are_independent_arrays():
    """Large host results come from the page-locked pool (engine.HOST_POOL, written by DMA
    directly): each call still returns its own array, as the reference's new array per call
    (base.py:378-407), equal to a result written into a caller-provided pageable array."""
    import gc
    from ninwavelets_amd import engine
    freqs = np.arange(1, 65, dtype=np.float64)
    w = nw.Morse(1000, dtype='float32')
    x1, x2 = synth(64, 4096, 1), synth(64, 4096, 2)        # 64 x 64 x 4096 complex64 = 128 MiB
    a = w.cwt_batch(x1, freqs)
    b = w.cwt_batch(x2, freqs)
    assert a.nbytes >= engine.HOST_POOL.min_bytes
    assert engine.HOST_POOL.held >= a.nbytes + b.nbytes   # both page-locked, both alive
    assert a.ctypes.data != b.ctypes.data
    plan = next(iter(w._plans.values()))
    ref = np.empty_like(a)                                  # pageable: the staged copy-out
    plan.execute(x1, out=ref)
    np.testing.assert_array_equal(a, ref)
    plan.execute(x2, out=ref)
    np.testing.assert_array_equal(b, ref)
    pa = a.ctypes.data
    del a
    gc.collect()
    c = w.cwt_batch(x2, freqs)                              # reuses the dropped buffer
    assert c.ctypes.data == pa
    np.testing.assert_array_equal(c, b)

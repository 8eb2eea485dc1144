"""CPU-only checks of the boundary and the host logic (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden_names, load_golden
from oracle import nw_oracle as O

import ninwavelets_amd as nw
from ninwavelets_amd import _lib as L


def header_functions():
    text = open(os.path.join(ROOT, 'include', 'ninwave.h')).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(nw_[a-z_]+)\s*\(', text)))


def test_library_exports_every_header_symbol():
    lib = L.lib()
    names = header_functions()
    assert len(names) >= 14
    for name in names:
        assert hasattr(lib, name), name
    # and the ctypes table binds exactly the header's functions
    assert sorted(n for n, _, _ in L.SIGNATURES) == names


def test_version_and_no_device_here():
    assert L.lib().nw_version().startswith(b'ninwave')
    if not os.path.exists('/dev/kfd'):
        assert L.device_count() == 0


@pytest.mark.skipif(os.path.exists('/dev/kfd'), reason='a GPU is present')
def test_no_cpu_fallback_without_gpu():
    with pytest.raises(L.NinwaveError):
        nw.Plan(256, 4, 'float32')
    with pytest.raises(L.NinwaveError):
        nw.Morse(1000).cwt(np.zeros(256), [1., 2.])


@pytest.mark.parametrize('interp', [False, True])
@pytest.mark.parametrize('sfreq', [1000., 500., 256., 1024., 333.3, 44100.])
def test_trans_grid_matches_numpy_arange(sfreq, interp):
    """nw_trans_grid restates _setup_trans_shape + hstack + interpolate_alias
    (base.py:173-194, 238-246, 274-276) bit for bit, including the N+1 lengths."""
    for n in list(range(1, 700)) + [1023, 1024, 4096, 4097, 16384, 1 << 20, 1 << 24]:
        rl = n / sfreq
        g = L.trans_grid(rl, sfreq, interp)
        t = O.trans_grid(sfreq, rl, interp)
        assert g.len_valid == t.shape[0], (n, sfreq)
        assert g.len_full == (2 * t.shape[0] if interp else t.shape[0])
        assert g.delta == 1 / rl
        if t.shape[0] > 1:
            assert t[1] == g.delta and t[-1] == (t.shape[0] - 1) * g.delta


def test_trans_grid_arbitrary_real_length():
    for rl in [1.0, 0.5, 2.5, 1e-3, 7.123]:
        g = L.trans_grid(rl, 1000., False)
        assert g.len_full == O.trans_grid(1000., rl, False).shape[0]


def test_trans_grid_rejects_bad_args():
    with pytest.raises(ValueError):
        L.trans_grid(0.0, 1000., False)
    with pytest.raises(ValueError):
        L.trans_grid(1.0, -1., False)


def test_fused_support_table():
    # every length up to 2n - 1 <= 16384 (fp32) / 8192 (fp64) has a fused form (the chirp-z
    # form for non-powers of two and n < 1024); longer odd lengths stay on the rocFFT engine
    for n in (1, 2, 3, 300, 512, 1201, 4097, 8192):
        assert L.fused_supported(n, L.NW_F32) is True, n
    for n in (1, 300, 512, 4095):
        assert L.fused_supported(n, L.NW_F64) is True, n
    assert L.fused_supported(8193, L.NW_F32) is False
    assert L.fused_supported(4097, L.NW_F64) is False
    assert L.fused_supported(20001, L.NW_F32) is False
    for dt in (L.NW_F32, L.NW_F64):
        for lg in range(10, 25):                             # one pass to 2^14, two passes above
            assert L.fused_supported(1 << lg, dt) is True, (lg, dt)
        assert L.fused_supported(1 << 25, dt) is False


# ---------------------------------------------------------------- host-side errors
def test_errors_match_reference_before_any_device_call():
    m = nw.Morse(1000)
    with pytest.raises(IndexError):
        m.cwt(np.zeros(64), [5.])                   # freqs[1] (base.py:272)
    with pytest.raises(ZeroDivisionError):
        nw.Morse(1000).cwt(np.zeros(64), [0., 1.])  # base.py:234-235
    with pytest.raises(TypeError):
        nw.Morse(1000).cwt(np.zeros(64), None)       # None[1]
    with pytest.raises(ZeroDivisionError):
        nw.MexicanHat(1000).cwt(np.zeros(64), [0., 1.])


# ---------------------------------------------------------------- host table builds
@pytest.mark.parametrize('name', [n for n in golden_names() if n.startswith(('mexhat', 'haar'))])
def test_normal_mode_table_rows_match_reference(name):
    g = load_golden(name)
    if 'w_first' not in g:
        pytest.skip('no rows stored')
    m = g['meta']
    base = nw.MexicanHat if m['kind'] == 'mexican_hat' else nw.Haar

    class HostBuilt(base):            # a plugin formula (same values): the host table path
        def formula(self, tc, freq=1):
            return base.formula(self, tc, freq)

    w = HostBuilt(m['sfreq'], interpolate=m['interpolate'])
    assert w._device_normal() is None and base(1000)._device_normal() is not None
    cache = w._build_cache(g['freqs'], m['n'] / m['sfreq'])
    np.testing.assert_array_equal(cache.table[0][:cache.row_len[0]], g['w_first'])
    np.testing.assert_array_equal(cache.table[-1][:cache.row_len[-1]], g['w_last'])


def test_plugin_subclass_becomes_table():
    class Sq(nw.Morse):
        def trans_formula(self, freqs, freq=1.):
            return np.exp(-(freqs - freq) ** 2)

    w = Sq(1000)
    c = w._build_cache([5., 10., 20.], 256 / 1000)
    assert c.kind == 'table' and c.table.shape == (3, 256)
    t = np.arange(0, 1000 / (256 / 1000) * (256 / 1000), 1 / (256 / 1000))
    np.testing.assert_array_equal(c.table[1].real, np.exp(-(t - 10.) ** 2))
    assert nw.Morse(1000)._build_cache([5., 10.], 0.256).kind == 'morse'


def test_reference_api_surface():
    for name in ['WaveletBase', 'WaveletMode', 'Morse', 'MorseMNE', 'Morlet', 'Haar',
                 'MexicanHat', 'Shannon', 'EpochsWavelet']:
        assert hasattr(nw, name)
    m = nw.Morse(1000, b=17.5, r=3)
    assert (m.b, m.r, m.mode, m.sfreq, m.interpolate) == (17.5, 3, nw.WaveletMode.Reverse, 1000, False)
    assert nw.Morlet().mode == nw.WaveletMode.Both
    assert nw.MexicanHat().mode == nw.WaveletMode.Normal
    assert nw.WaveletBase().interpolate is True
    # the numpy plugin formulas equal the oracle's restatement
    nu = np.linspace(0, 500, 1001)
    np.testing.assert_array_equal(nw.Morse().trans_formula(nu, 40.), O.morse_spectrum(nu, 40.))
    np.testing.assert_array_equal(nw.Morlet().trans_formula(nu, 40.), O.morlet_spectrum(nu, 40.))


def test_nw_log_levels():
    """NW_LOG: errors are reported on stderr at level >= 1, silent at 0; the
    environment sets the default, nw_set_log_level overrides it."""
    import subprocess
    import sys
    code = ('import ctypes, sys; sys.path.insert(0, %r)\n'
            'from ninwavelets_amd import _lib as L\n'
            'p = ctypes.c_void_p()\n'
            'prev = L.set_log_level(0); L.set_log_level(prev); print("level", prev, flush=True)\n'
            'L.set_log_level(int(sys.argv[1]))\n'
            'rc = L.lib().nw_plan_create(ctypes.byref(p), 0, 0, 1, 1, 1, 0)\n'
            'print("rc", rc, flush=True)\n') % ROOT
    for env_level, set_level, expect in (('1', 1, True), ('0', 0, False), ('1', 0, False), ('0', 2, True)):
        env = dict(os.environ, NW_LOG=env_level)
        r = subprocess.run([sys.executable, '-c', code, str(set_level)], capture_output=True, text=True, env=env,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        assert f'level {env_level}' in r.stdout and f'rc {L.NW_E_INVALID}' in r.stdout
        logged = [ln for ln in r.stderr.splitlines() if ln.startswith('[ninwave] error')]
        assert bool(logged) == expect, r.stderr
        if expect:
            assert 'n, max_batch, nfreq must be >= 1' in logged[0]


def test_debug_library_builds_and_exports():
    """libninwave_debug.so (kernel bounds checks) exports the same header; the product library
    reports no checks and refuses the self-test."""
    import subprocess
    import sys
    dbg = os.path.join(ROOT, 'ninwavelets_amd', 'libninwave_debug.so')
    assert os.path.exists(dbg), 'make -C ninwavelets_amd/csrc debug'
    code = ('import sys; sys.path.insert(0, %r)\n'
            'from ninwavelets_amd import _lib as L\n'
            'lib = L.lib()\n'
            'print(lib.nw_debug_bounds(), lib.nw_debug_selftest(0) if not sys.argv[1:] else "-")\n') % ROOT
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, NINWAVE_LIB=dbg))
    assert r.returncode == 0, r.stderr
    bounds, _ = r.stdout.split()
    assert bounds == '1'
    lib = ctypes.CDLL(dbg)
    for name in header_functions():
        assert hasattr(lib, name), name
    assert L.lib().nw_debug_bounds() == 0
    assert L.lib().nw_debug_selftest(0) == L.NW_E_STATE


def test_plan_cache_evicts_least_recently_used():
    """WaveletBase._evict_plans (no GPU: stand-in plans report their device bytes): the least
    recently used plans are closed until the cache fits plan_cache_bytes; the current call's
    plans stay even when they alone exceed it."""
    from collections import OrderedDict

    class FakePlan:
        def __init__(self, b):
            self.b, self.closed = b, False

        def stats(self):
            return {'device_bytes': self.b}

        def close(self):
            self.closed = True

    w = nw.Morse(1000)
    plans = [FakePlan(b) for b in (10, 20, 30, 40)]
    w._plans = OrderedDict((i, p) for i, p in enumerate(plans))
    w.plan_cache_bytes = 75
    w._evict_plans(keep=1)
    assert list(w._plans) == [2, 3] and plans[0].closed and plans[1].closed and not plans[2].closed
    w.plan_cache_bytes = 5
    w._evict_plans(keep=1)
    assert list(w._plans) == [3] and not plans[3].closed
    w._plans = OrderedDict((i, p) for i, p in enumerate([FakePlan(50), FakePlan(50)]))
    w._evict_plans(keep=2)                      # a two-device call keeps both of its plans
    assert len(w._plans) == 2


@pytest.mark.parametrize('name', golden_names('plugin_'))
def test_plugin_rows_are_the_references(name):
    """User plugins (README.md:342-355) on the drop-in: the cached rows the host evaluates with
    the plugin's own formula equal the reference's make_fft_wavelets rows bit for bit
    (base.py:221-279; Reverse, Morse-subclass, Normal and Twice plugins, tests/plugins.py)."""
    import plugins
    g = load_golden(name)
    m = g['meta']
    w = plugins.make(nw, m['plugin'], m['sfreq'], m['interpolate'])
    rows = w.make_fft_wavelets(list(g['freqs']), m['n'] / m['sfreq'])
    np.testing.assert_array_equal(rows[0], g['w_first'])
    np.testing.assert_array_equal(rows[-1], g['w_last'])
    assert w._cache.kind == 'table'           # plugins take the host-table path


def test_host_pool_recycles_and_caps():
    """engine.HostPool (page-locked result arrays) with stand-in allocators, no GPU: a dropped
    result's buffer serves the next result of its size; results the caller keeps are never
    shared; past the cap results fall back to ordinary arrays; small results never pool."""
    import gc
    from ninwavelets_amd.engine import HostPool
    store, freed = {}, []

    def alloc(nb):
        b = np.zeros(nb, dtype=np.uint8)
        store[b.ctypes.data] = b
        return b.ctypes.data

    advised = []
    pool = HostPool(cap=3 * 4096, min_bytes=1024, keep_free=1, alloc=alloc, free=freed.append,
                    advise=advised.append)
    a = pool.empty((64, 8), np.float64)                  # 4096 B: pooled
    assert a.ctypes.data in store and pool.held == 4096
    a[:] = 1.0
    b = pool.empty((64, 8), np.float64)
    assert b.ctypes.data != a.ctypes.data                # both alive: distinct buffers
    pa = a.ctypes.data
    v = a[3:]                                           # a view keeps the buffer
    del a
    gc.collect()
    c = pool.empty((512,), np.float64)
    assert c.ctypes.data != pa
    del v
    gc.collect()
    d = pool.empty((8, 64), np.float64)                  # same size: the released buffer
    assert d.ctypes.data == pa and pool.held == 3 * 4096
    e = pool.empty((64, 8), np.float64)                  # over the cap: an ordinary array
    assert e.ctypes.data not in store and e.shape == (64, 8)
    assert len(advised) == 1 and advised[0] is e          # our own fresh array: huge-page advice
    s = pool.empty((10,), np.float64)                    # below min_bytes
    assert s.ctypes.data not in store and len(advised) == 1
    del b, c, d
    gc.collect()
    assert pool.free_bytes() == 4096 and len(freed) == 2  # keep_free = 1 per size


def test_host_pool_release_never_takes_the_lock():
    """A pooled array held by a reference cycle may be collected by a GC that runs anywhere --
    inside the pool's own locked region included (an allocation there can trigger it).  Its
    finalizer must not wait for the lock (the old release path deadlocked there); the buffer
    is filed at the next take."""
    import gc
    import threading
    from ninwavelets_amd.engine import HostPool
    store = {}

    def alloc(nb):
        b = np.zeros(nb, dtype=np.uint8)
        store[b.ctypes.data] = b
        return b.ctypes.data

    pool = HostPool(cap=4 * 4096, min_bytes=1024, keep_free=2, alloc=alloc, free=lambda p: None,
                    advise=lambda a: None)

    class Cycle:
        pass

    c = Cycle()
    c.me, c.arr = c, pool.empty((512,), np.float64)
    ptr = c.arr.ctypes.data
    del c
    done = threading.Event()

    def collect_under_lock():
        with pool._lock:
            gc.collect()              # runs the finalizer of the cycle's pooled array
        done.set()

    gc.disable()
    try:
        th = threading.Thread(target=collect_under_lock, daemon=True)
        th.start()
        th.join(timeout=20)
    finally:
        gc.enable()
    assert done.is_set(), 'the finalizer blocked on the pool lock'
    again = pool.empty((512,), np.float64)                # filed at this take: the same buffer
    assert again.ctypes.data == ptr and pool.held == 4096


def test_default_pool_cap_shares_the_node():
    from ninwavelets_amd.engine import default_pool_cap
    assert default_pool_cap(1 << 40, 1) == 8 << 30                 # 8 GiB per process
    assert default_pool_cap(1 << 40, 8) == 1 << 30                 # eight ranks of a node: 8 GiB in all
    assert default_pool_cap(16 << 30, 1) == 2 << 30                # at most 1/8 of the host's RAM


def test_pool_cap_counts_node_local_ranks_only():
    """A multi-node launch without LOCAL_WORLD_SIZE: the pool is shared by this node's ranks
    (the launcher's node-local count), never divided by the global WORLD_SIZE."""
    from ninwavelets_amd.engine import local_rank_count
    assert local_rank_count({'WORLD_SIZE': '64', 'RANK': '9'}) == 1
    assert local_rank_count({'WORLD_SIZE': '64', 'LOCAL_WORLD_SIZE': '8'}) == 8
    assert local_rank_count({'WORLD_SIZE': '64', 'SLURM_NTASKS_PER_NODE': '8(x8)'}) == 8
    assert local_rank_count({'WORLD_SIZE': '64', 'OMPI_COMM_WORLD_LOCAL_SIZE': '4'}) == 4
    assert local_rank_count({'LOCAL_WORLD_SIZE': 'x', 'MPI_LOCALNRANKS': '2'}) == 2


def test_pool_trim_frees_idle_buffers():
    from ninwavelets_amd.engine import HostPool
    freed = []
    nxt = iter(range(1, 100))
    pool = HostPool(cap=1 << 20, min_bytes=1024, keep_free=2, alloc=lambda n: next(nxt) * 4096,
                    free=freed.append, advise=lambda a: None)
    a, b = pool.empty((512,), np.float64), pool.empty((256,), np.float64)
    kept = pool.empty((512,), np.float64)
    assert pool.held == 4096 + 2048 + 4096
    del a, b
    assert pool.trim() == 4096 + 2048 and len(freed) == 2
    assert pool.held == 4096 and pool.free_bytes() == 0          # the live result stays
    del kept
    assert pool.trim() == 4096 and pool.held == 0


def test_pool_advice_skipped_without_the_symbol(monkeypatch):
    """An older diagnostic library without nw_host_advise: over-cap results stay plain arrays."""
    from ninwavelets_amd import engine

    class OldLib:
        pass
    monkeypatch.setattr(engine.L, 'lib', lambda: OldLib())
    engine.HostPool._nw_advise(np.empty(16))                   # no AttributeError

"""GPU parity of the numpy drop-in in a process that never imports torch (run by
tests/test_gpu_torchfree.py as a child process; not collected by pytest itself).

The reference imports only numpy / scipy / cupy (/root/reference/ninwavelets/base.py:1-4), so
its users load libninwave.so against /opt/rocm's HIP runtime and rocFFT, not the copies
bundled in the torch wheel that the rest of the GPU suite binds.  This script checks, under
that runtime:
  1. every single-signal reference golden (tests/golden/*.npz), fp64 and fp32, both engines;
  2. the reference's outputs at the benchmark lengths (tests/golden/long_*.npz), fp64 and fp32;
  3. the C3 / C4 bench shapes: Morse power at N = 4096 (nw_fused_pair_kernel) and N = 16384
     (nw_fused_kernel), all 256 scales of 4 signals, against the oracle;
  4. epoch power_mean / itc on each engine form against the same plan's per-signal outputs.
With NINWAVE_LIB naming the debug library (tests/test_gpu_debug.py) the same run exercises
the kernel bounds checks: a failing check is an NW_E_BOUNDS error in the case that hit it.
Tolerances are tests/test_gpu_parity.py's (fp64 1e-12, fp32 1e-5 of max|ref|, x2 for |.|^2,
1e-4 for fp32 at N >= 2^17).  Prints one JSON summary line; exits 1 on any failure.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from goldens import golden_names, load_golden, long_signal, x_digest  # noqa: E402
from oracle import nw_oracle as O  # noqa: E402

import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402

CLASSES = {'morse': nw.Morse, 'morlet': nw.Morlet, 'shannon': nw.Shannon,
           'mexican_hat': nw.MexicanHat, 'haar': nw.Haar}
TOL = {'float64': 1e-12, 'float32': 1e-5}
failures, counts = [], {'single': 0, 'long': 0, 'bench_shapes': 0, 'reductions': 0}


def close(got, ref, rtol, dtype):
    floor = 1e-30 if dtype == 'float32' else 0.0
    return np.max(np.abs(got - ref), initial=0.0) <= rtol * np.max(np.abs(ref), initial=0.0) + floor


def rel(got, ref):
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-300))


def single_goldens():
    names = [n for n in golden_names()
             if not n.startswith(('readme_2d', 'reuse', 'epochs', 'baseline', 'wavelets', 'long', 'plugin'))]
    for name in names:
        g = load_golden(name)
        m = g['meta']
        for dtype in ('float64', 'float32'):
            for engine in ('rocfft', 'auto'):
                w = CLASSES[m['kind']](m['sfreq'], interpolate=m['interpolate'], dtype=dtype, engine=engine,
                                       **dict(m['params']))
                got = {'cwt': w.cwt, 'power': w.power, 'abs': w.abs}[m['op']](g['x'], g['freqs'])
                t = TOL[dtype] * (2 if m['op'] == 'power' else 1)
                if m['dtype'] == 'float32':
                    t = max(t, 1e-5)
                counts['single'] += 1
                if got.shape != g['out'].shape or not close(got, g['out'], t, dtype):
                    failures.append(('single', name, dtype, engine, rel(got, g['out'])))


def long_goldens():
    for name in golden_names('long_'):
        g = load_golden(name)
        m = g['meta']
        n = m['n']
        x = long_signal(n, m['seed'])
        assert x_digest(x) == m['x_sha256']
        for dtype in ('float64', 'float32'):
            cls = {'morse': nw.Morse, 'morlet': nw.Morlet}[m['kind']]
            out = cls(m['sfreq'], dtype=dtype).cwt(x.astype(dtype), g['freqs'])
            tol = 1e-12 if dtype == 'float64' else (1e-5 if n <= 16384 else 1e-4)
            counts['long'] += 1
            err = rel(out[:, g['pos']], g['out_at'])
            o = out.astype(np.complex128)
            e_row = (np.abs(o) ** 2).sum(axis=1)
            ok = err <= tol and np.allclose(e_row, g['row_energy'], rtol=4 * tol, atol=0)
            ok = ok and np.all(np.abs(o.sum(axis=1) - g['row_sum']) <=
                               tol * (np.sqrt(g['row_energy']) + np.abs(g['row_sum'])))
            if not ok:
                failures.append(('long', name, dtype, err))
            del out, o


def bench_shapes():
    rng = np.random.default_rng(11)
    freqs = np.arange(1, 257, dtype=np.float64)
    for n, kernel in ((4096, 'nw_fused_pair_kernel'), (16384, 'nw_fused_kernel')):
        t = np.arange(n) / 1000.
        x = (np.sin(2 * np.pi * rng.uniform(1, 100, (4, 1)) * t) + 0.1 * rng.standard_normal((4, n))).astype(np.float32)
        ref = np.abs(np.stack([O.cwt('morse', x[s].astype(np.float64), freqs) for s in range(4)])) ** 2
        g = L.trans_grid(n / 1000., 1000., False)
        plan = nw.Plan(n, 256, 'float32', max_batch=2)
        plan.set_wavelet('morse', [17.5, 3.], freqs, g)
        got = plan.execute(x, out_kind='power')
        ran = L.KERNEL_NAMES[plan.stats()['kernel']]
        counts['bench_shapes'] += 1
        if ran != kernel or rel(got, ref) > 2e-5:
            failures.append(('bench_shape', n, ran, rel(got, ref)))
        plan.close()


def reductions():
    """Epoch reductions on every engine form (fused partials incl. the pair kernel, chirp-z
    partials, the two-pass chunk path): power_mean / itc against the same plan's per-signal
    power / cwt (mneutils.py:42-71)."""
    rng = np.random.default_rng(5)
    freqs = np.arange(1, 257, 16, dtype=np.float64)
    for n, dtype in ((1201, 'float32'), (1201, 'float64'), (4096, 'float32'), (4096, 'float64'),
                     (16384, 'float32'), (32768, 'float32')):
        x = rng.standard_normal((11, n)).astype(dtype)
        g = L.trans_grid(n / 1000., 1000., False)
        plan = nw.Plan(n, len(freqs), dtype, max_batch=4)
        plan.set_wavelet('morse', [17.5, 3.], freqs, g)
        pw = plan.execute(x, out_kind='power').astype(np.float64)
        y = plan.execute(x, out_kind='cwt').astype(np.complex128)
        pm = plan.execute(x, out_kind='power_mean')
        itc = plan.execute(x, out_kind='itc')
        plan.close()
        f32 = dtype == 'float32'
        counts['reductions'] += 1
        e_pm = rel(pm, pw.mean(axis=0))
        e_itc = np.max(np.abs(itc - np.abs(np.mean(y / np.abs(y), axis=0))))
        if e_pm > (1e-5 if f32 else 1e-12) or e_itc > (1e-4 if f32 else 1e-10):
            failures.append(('reduction', n, dtype, e_pm, e_itc))


def hip_runtime_path():
    with open('/proc/self/maps') as f:
        libs = sorted({ln.split()[-1] for ln in f if 'libamdhip64' in ln or 'librocfft' in ln})
    return libs


single_goldens()
long_goldens()
bench_shapes()
reductions()
summary = {'torch_imported': 'torch' in sys.modules, 'runtime': hip_runtime_path(), 'counts': counts,
           'lib': L.LIB_PATH, 'debug_bounds': int(L.lib().nw_debug_bounds()),
           'failures': [list(map(str, f)) for f in failures]}
print(json.dumps(summary), flush=True)
sys.exit(1 if failures or summary['torch_imported'] else 0)

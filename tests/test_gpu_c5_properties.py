"""C5 at its full size through size-independent properties (every row of every scale chunk).

The C5 parity tests against the oracle (test_gpu_parity.py) check a few of the 512 rows of the
2^24-sample signal, since one fp64 oracle row costs seconds.  Here every row of the two-pass
engine's output (nw_large.hip: 8 scale chunks of 64 in fp32, 32 in fp64) is checked against the
transform's own structure.  y = ifft(W_f * fft(x)) (base.py:378-407) is a circular convolution
per scale, so shifting the signal shifts every row:

    cwt(roll(x, s))[f] == roll(cwt(x)[f], s)      for every scale f,

and the row energies sum_n |y_f|^2 agree.  A wrong scale chunk, row offset, column block or
batch stride breaks either on some row by O(1).  The two signals run as one batch (per-signal Xt
and chunk loop).  Measured on the GPU (round 5): fp32 1.1e-6 of the signal's max, the worst row
2.5e-6 of its own max, energies 3.0e-7 relative; fp64 2.3e-15 / 7.5e-15 / 6.6e-16.  Bounds, ~10x
above that (and far inside the parity contract, fp32 1e-4 at 2^24 / fp64 1e-12): fp32 2e-5 /
1e-4 / 1e-5, fp64 1e-13 / 1e-12 / 1e-13.  The comparison arithmetic runs in torch on the device.
Since a wrong W row would shift with the signal, 16 rows spread over the chunks also check their
energy against Parseval with the oracle's own rows and numpy's fft (measured 1.3e-6 / 5.6e-15;
bounds fp32 1e-5, fp64 1e-13).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402
from oracle import nw_oracle as O  # noqa: E402

N = 1 << 24
SHIFT = 1234567


@pytest.mark.parametrize('dtype,nfreq', [('float32', 512), ('float64', 256)])
def test_c5_every_row_shift_equivariant(dtype, nfreq):
    torch = pytest.importorskip('torch')
    dev = torch.device('cuda', 0)
    f64 = dtype == 'float64'
    freqs = np.linspace(0.5, 250, nfreq)
    rdt = torch.float64 if f64 else torch.float32
    cdt = torch.complex128 if f64 else torch.complex64
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    t = torch.arange(N, device=dev, dtype=torch.float64) / 1000.
    x = (torch.sin(2 * np.pi * 37.0 * t) + 0.5 * torch.sin(2 * np.pi * 3.3 * t + 1.0)
         + 0.1 * torch.randn(N, device=dev, dtype=torch.float64, generator=g)).to(rdt)
    xs = torch.stack([x, torch.roll(x, SHIFT)]).contiguous()
    x_host = x.to(torch.float64).cpu().numpy()
    del t
    plan = nw.Plan(N, nfreq, dtype, max_batch=2)
    plan.set_wavelet('morse', [17.5, 3.0], freqs, L.trans_grid(N / 1000., 1000., False))
    out = torch.empty((2, nfreq, N), dtype=cdt, device=dev)
    plan.execute(xs, out, out_kind='cwt')
    plan.sync()
    st = plan.stats()
    assert st['engine'] == 'fused' and st['launches_rows'] > 0, st
    d = torch.empty(nfreq, dtype=torch.float64, device=dev)
    m = torch.empty(nfreq, dtype=torch.float64, device=dev)
    e0 = torch.empty(nfreq, dtype=torch.float64, device=dev)
    e1 = torch.empty(nfreq, dtype=torch.float64, device=dev)
    for f in range(nfreq):
        a, b = out[0, f], out[1, f]
        d[f] = (torch.roll(a, SHIFT) - b).abs().amax().to(torch.float64)
        m[f] = a.abs().amax().to(torch.float64)
        e0[f] = (a.abs().to(torch.float64) ** 2).sum()
        e1[f] = (b.abs().to(torch.float64) ** 2).sum()
    plan.close()
    del out, xs
    torch.cuda.empty_cache()
    d, m, e0, e1 = (v.cpu().numpy() for v in (d, m, e0, e1))
    assert np.all(np.isfinite(m)) and np.all(m > 0)
    sig_tol, row_tol, e_tol = (1e-13, 1e-12, 1e-13) if f64 else (2e-5, 1e-4, 1e-5)
    print(f'{dtype}: signal {d.max() / m.max():.3g}, worst row {(d / m).max():.3g}, '
          f'energy {np.max(np.abs(e1 - e0) / e0):.3g}')
    assert d.max() <= sig_tol * m.max(), (d.max() / m.max())
    worst = int(np.argmax(d / m))
    assert d[worst] <= row_tol * m[worst], (freqs[worst], d[worst] / m[worst])
    np.testing.assert_allclose(e1, e0, rtol=e_tol)
    # 16 rows across the 8 scale chunks against Parseval with the oracle's rows (base.py:221-279)
    # and numpy's fft: sum_n |y_f|^2 = (1/N) sum_k |W_f[k] X[k]|^2
    sel = list(range(0, nfreq, nfreq // 16))
    X = np.fft.fft(x_host)
    rows = O.fft_wavelets('morse', freqs[sel], 1000., N / 1000., False)
    ref = np.array([np.sum(np.abs(O.pad_to(r, N) * X) ** 2) / N for r in rows])
    print(f'{dtype}: Parseval against the oracle rows {np.max(np.abs(e0[sel] - ref) / ref):.3g}')
    np.testing.assert_allclose(e0[sel], ref, rtol=1e-13 if f64 else 1e-5)

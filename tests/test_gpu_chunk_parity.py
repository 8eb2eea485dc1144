"""GPU parity at the chunk sizes the bench times (every row of every launch it times).

The bench launches ``nw_fused_kernel`` on 512-signal chunks (C4, fp32 and fp64) and
``nw_fused_pair_kernel`` on 1024-signal chunks (C3 power), bench.py DEFAULT_CHUNK.  Such a
launch walks several XCD-tile "G-rounds" (nw_fused.hip: signal groups padded to
``nsg_pad``, ``kTileG`` groups per XCD round) and writes outputs far beyond 4 GiB, so the
small-batch parity tests (<= 37 signals: G-round 0 only) do not cover it.  Here the bench's
exact plans run S = chunk + 37 signals (one full chunk, then a ragged tail) and:

- every point of every (signal, scale) row against y = ifft(W_f * X) (base.py:378-407),
  W_f the oracle's cached row (base.py:221-279) and X = np.fft.fft(x), the inverse taken in
  complex128 on the device: the parity contract per signal, and each row on its own scale;
- every row's energy sum_n |y|^2 (or sum_n of the power output, base.py:409-425) against
  (1/N) sum_k |W_f X|^2 from numpy (Parseval);
- sampled signals in every G-round and XCD slot of the chunk and in the tail against the
  oracle's full cwt / power (oracle/nw_oracle.py), at the parity tolerances of
  test_gpu_parity.py (fp64 1e-12, fp32 1e-5 of max|ref|, x2 for |.|^2).

The device-side inverse FFT / sums (torch on the GPU) are the checker's arithmetic, in complex128.
"""
import os
import re

import numpy as np
import pytest

from oracle import nw_oracle as O

pytestmark = pytest.mark.gpu

import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAIL = 37


def fused_constants(f64=False):
    """Signals per block and XCD-tile groups as the kernel source defines them for the
    n = 16384 output kernels (kGroup / kTileG; fp64: NW_GROUP64_16K / NW_TILE64_G_16K)."""
    src = open(os.path.join(ROOT, 'ninwavelets_amd', 'csrc', 'nw_fused.hip')).read()
    if f64:
        return (int(re.search(r'#define NW_GROUP64_16K (\d+)', src).group(1)),
                int(re.search(r'#define NW_TILE64_G_16K (\d+)', src).group(1)))
    g = int(re.search(r'constexpr int kGroup = (\d+);', src).group(1))
    tg = int(re.search(r'constexpr int kTileF = \d+, kTileG = (\d+);', src).group(1))
    return g, tg


def synth(S, n, seed, dtype):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 1000.
    fc = rng.uniform(1, 100, (S, 1))
    ph = rng.uniform(0, 2 * np.pi, (S, 1))
    return (np.sin(2 * np.pi * fc * t + ph) + 0.1 * rng.standard_normal((S, n))).astype(dtype)


def sampled(S, chunk):
    """Signals in every G-round / XCD slot of the full chunk, and the ragged tail."""
    want = [0, 7, 255, 256, 263, 511, 767, 1023, chunk - 1, chunk, S - 1]
    return sorted({s for s in want if 0 <= s < S})


CASES = [
    # (n, compute dtype, chunk (bench.py DEFAULT_CHUNK), bench output, kernel)
    pytest.param(16384, 'float32', 512, 'cwt', 'nw_fused_kernel', id='c4-fp32-512'),
    pytest.param(16384, 'float64', 512, 'cwt', 'nw_fused_kernel', id='c4-fp64-512'),
    pytest.param(4096, 'float32', 1024, 'power', 'nw_fused_pair_kernel', id='c3-power-1024'),
]


@pytest.mark.parametrize('n,dtype,chunk,out_kind,kernel', CASES)
def test_bench_chunk_every_row(n, dtype, chunk, out_kind, kernel):
    import torch
    dev = torch.device('cuda', 0)
    f64 = dtype == 'float64'
    S, freqs = chunk + TAIL, np.arange(1, 257, dtype=np.float64)
    F = len(freqs)
    assert n == 16384 or not f64
    group, tile_g = fused_constants(f64)
    nsg = -(-chunk // group)
    nsg_pad = -(-nsg // (8 * tile_g)) * (8 * tile_g)
    assert nsg_pad // (8 * tile_g) >= 2, 'the chunk must span >= 2 XCD-tile G-rounds'

    x = synth(S, n, seed=n + chunk, dtype=np.float64 if f64 else np.float32)
    plan = nw.Plan(n, F, dtype, max_batch=chunk)          # bench.py run_leg's plan
    plan.set_wavelet('morse', [17.5, 3.0], freqs, L.trans_grid(n / 1000., 1000., False))
    xd = torch.from_numpy(x).to(dev)
    cdt = torch.complex128 if f64 else torch.complex64
    rdt = torch.float64 if f64 else torch.float32

    # fp64 numpy: the oracle's cached rows (pad_to'd) and the input spectra
    W = np.array([O.pad_to(r, n) for r in O.fft_wavelets('morse', freqs, 1000., n / 1000., False)])
    X = np.fft.fft(x.astype(np.float64), axis=-1)
    energy = (np.abs(X) ** 2) @ (np.abs(W) ** 2).T / n          # (S, F): sum_n |y|^2, Parseval
    Wd = torch.from_numpy(W).to(dev)
    Xd = torch.from_numpy(X).to(dev)
    tol = 1e-12 if f64 else 1e-5

    def check_rows(out, power=False):
        """Every row against y = ifft(W * X) in fp64 on the device: the parity contract per
        signal (max |dy| <= tol * max|y| over its scales; x2 for |.|^2) and every row on its
        own scale (max |dy_row| <= 5e-4 * max|y_row| fp32, 1e-10 fp64: a wrong tile, G-round or
        offset puts an O(1) error into some row), plus each row's Parseval energy."""
        worst_sig, worst_row = 0.0, 0.0
        row_tol = 1e-10 if f64 else 5e-4
        for s0 in range(0, S, 16):
            s1 = min(S, s0 + 16)
            ref = torch.fft.ifft(Wd[None, :, :] * Xd[s0:s1, None, :], dim=-1)
            got = out[s0:s1].to(torch.float64 if power else torch.complex128)
            if power:
                ref = ref.abs() ** 2
            d = (got - ref).abs().amax(dim=-1)                  # (signals, F)
            m = ref.abs().amax(dim=-1)
            worst_sig = max(worst_sig, float((d.amax(dim=-1) / m.amax(dim=-1)).max()))
            worst_row = max(worst_row, float((d / m.clamp_min(1e-300)).max()))
            e = (got if power else got.abs() ** 2).sum(dim=-1).cpu().numpy()
            np.testing.assert_allclose(e, energy[s0:s1], rtol=(8 if power else 4) * tol)
            del ref, got, d, m
        assert worst_sig <= (2 if power else 1) * tol, worst_sig
        assert worst_row <= row_tol, worst_row
        return worst_sig, worst_row

    picks = sampled(S, chunk)
    ref_cwt = {s: O.cwt('morse', x[s].astype(np.float64), freqs) for s in picks}
    if out_kind == 'cwt':
        out = torch.empty((S, F, n), dtype=cdt, device=dev)
        assert out.numel() * out.element_size() // S * chunk > (4 << 30), 'one launch writes > 4 GiB'
        plan.execute(xd, out, out_kind='cwt')
        torch.cuda.synchronize()
        st = plan.stats()
        assert st['engine'] == 'fused' and L.KERNEL_NAMES[st['kernel']] == kernel, st
        assert st['launches_fused'] == 2, st               # the full chunk, then the tail
        check_rows(out)
        for s in picks:
            got = out[s].cpu().numpy()
            ref = ref_cwt[s]
            assert np.max(np.abs(got - ref)) <= tol * np.max(np.abs(ref)), s
        del out
    else:
        # the bench's power output: every row's sum against Parseval, sampled rows vs the oracle
        pw = torch.empty((S, F, n), dtype=rdt, device=dev)
        assert pw.numel() * pw.element_size() > (4 << 30)
        plan.execute(xd, pw, out_kind='power')
        torch.cuda.synchronize()
        st = plan.stats()
        assert st['engine'] == 'fused' and L.KERNEL_NAMES[st['kernel']] == kernel, st
        check_rows(pw, power=True)
        for s in picks:
            got = pw[s].cpu().numpy()
            ref = np.abs(ref_cwt[s]) ** 2
            assert np.max(np.abs(got - ref)) <= 2 * tol * np.max(ref), s
        # the same plan's complex output over the same chunks (same kernel family and block
        # map): every row checked, and power == |cwt|^2 of it to 1e-6 of the signal's max (two
        # instantiations whose fp32 FFT rounding may differ by a few ulps: 4.4e-7 measured on
        # the bounds-checking debug build, whose code generation differs)
        out = torch.empty((S, F, n), dtype=cdt, device=dev)
        plan.execute(xd, out, out_kind='cwt')
        torch.cuda.synchronize()
        check_rows(out)
        for s0 in range(0, S, 64):
            s1 = min(S, s0 + 64)
            c2 = out[s0:s1].to(torch.complex128).abs() ** 2
            rel = float(((pw[s0:s1].to(torch.float64) - c2).abs().amax(dim=-1) /
                         c2.amax(dim=-1).clamp_min(1e-300)).max())
            assert rel <= 1e-6, (s0, rel)
        del out, pw
    plan.close()
    torch.cuda.empty_cache()

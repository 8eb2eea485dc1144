"""Diagnostic: per-phase cycle shares of the fused kernel (needs the NW_STAMPS build:
make -C ninwavelets_amd/csrc VARIANT=stamps DEFS=-DNW_STAMPS)."""
import ctypes, os, sys
import numpy as np
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
os.environ.setdefault('NINWAVE_LIB', os.path.join(root, 'ninwavelets_amd', 'libninwave_stamps.so'))
import torch  # noqa: E402  (one HIP runtime: torch first)
import ninwavelets_amd as nw  # noqa: E402
from ninwavelets_amd import _lib as L  # noqa: E402

n, F, S = int(os.environ.get('N', 16384)), int(os.environ.get('F', 256)), 256
out_kind = os.environ.get('OUT', 'cwt')
dtype = os.environ.get('DTYPE', 'float32')
plan = nw.Plan(n, F, dtype, max_batch=S)
plan.set_wavelet('morse', [17.5, 3.], np.arange(1, F + 1, dtype=np.float64), L.trans_grid(n / 1000., 1000., False))
x = torch.randn(S, n, device='cuda', dtype=torch.float32 if dtype == 'float32' else torch.float64)
odt = {('cwt', 'float32'): torch.complex64, ('cwt', 'float64'): torch.complex128}.get((out_kind, dtype),
                                                                                      x.dtype)
o = torch.empty(S, F, n, device='cuda', dtype=odt)
fn = L.lib().nw_debug_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 9)()
for it in range(3):
    plan.execute(x, o, out_kind)
    plan.sync()
    fn(buf, 1)
names = ['pass0 load+dft', 'exch 0->1', 'pass1 dft', 'exch 1->2', 'pass2 dft', 'exch 2->3', 'pass3 dft', 'stores']
tot = sum(buf[k] for k in range(8))
E = 32 if n >= 8192 else 16          # NW_FUSED_TABLE: E = 32 at n = 8192 / 16384 (fp32 and fp64)
sw = buf[8] * (n // E // 64)   # signal-waves
print(f'n={n} F={F} {dtype} {out_kind}: signal-waves={sw}, cycles/signal/wave={tot / max(1, sw):.0f}')
for k in range(8):
    if buf[k]:
        print(f'  {names[k]:16s} {buf[k] / tot * 100:5.1f}%  {buf[k] / max(1, sw):8.0f} cyc')

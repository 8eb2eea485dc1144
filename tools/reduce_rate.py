"""Epoch reductions vs the per-signal output on device tensors (the library given by
NINWAVE_LIB): power_mean / itc against power, 512 signals x 256 scales, per n and dtype.
    DTYPES="float64 float32" NS="1024 2048 4096 1201" python tools/reduce_rate.py [tag]"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ninwavelets_amd as nw
from ninwavelets_amd import _lib as L

tag = sys.argv[1] if len(sys.argv) > 1 else ''
for dt in os.environ.get('DTYPES', 'float64 float32').split():
    tdt = torch.float32 if dt == 'float32' else torch.float64
    for n in [int(v) for v in os.environ.get('NS', '1024 2048 4096').split()]:
        S, F, C = 512, 256, 128
        g = L.trans_grid(n / 1000., 1000., False)
        plan = nw.Plan(n, F, dt, max_batch=C)
        plan.set_wavelet('morse', [17.5, 3.], np.arange(1., F + 1), g)
        x = torch.randn((S, n), device='cuda', dtype=tdt)
        om = torch.empty((F, n), device='cuda', dtype=tdt)
        op = torch.empty((C, F, n), device='cuda', dtype=tdt)
        res = {}
        for kind in ('power_mean', 'itc', 'power'):
            def once():
                if kind != 'power':
                    plan.execute(x, om, out_kind=kind)
                else:
                    for s0 in range(0, S, C):
                        plan.execute(x[s0:s0 + C], op, out_kind=kind)
            once(); plan.sync(); torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter(); once(); plan.sync(); torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            res[kind] = min(ts) * 1e3
        pts = S * F * n
        print('%s %s n=%5d power_mean %.3f ms (%.3e pts/s, %.2fx power)  itc %.3f ms (%.2fx)  power %.3f ms' % (
            tag, dt, n, res['power_mean'], pts / res['power_mean'] * 1e3, res['power_mean'] / res['power'],
            res['itc'], res['itc'] / res['power'], res['power']), flush=True)
        plan.close()

"""A/B of the fused epoch power partials: power_mean vs per-signal power on device tensors,
the library given by NINWAVE_LIB (base: fused partials, _nopsum: power + accumulate)."""
import os, sys, time
import numpy as np
import torch
import ninwavelets_amd as nw
from ninwavelets_amd import _lib as L

tag = sys.argv[1]
for n in [int(v) for v in os.environ.get('NS', '1024 2048 4096').split()]:
    S, F = 512, 256
    g = L.trans_grid(n / 1000., 1000., False)
    plan = nw.Plan(n, F, 'float32', max_batch=128)
    plan.set_wavelet('morse', [17.5, 3.], np.arange(1., F + 1), g)
    x = torch.randn((S, n), device='cuda', dtype=torch.float32)
    om = torch.empty((F, n), device='cuda', dtype=torch.float32)
    op = torch.empty((128, F, n), device='cuda', dtype=torch.float32)
    res = {}
    for kind in ('power_mean', 'itc', 'power'):
        def once():
            if kind != 'power':
                plan.execute(x, om, out_kind=kind)
            else:
                for s0 in range(0, S, 128):
                    plan.execute(x[s0:s0 + 128], op, out_kind=kind)
        once(); plan.sync(); torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter(); once(); plan.sync(); torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res[kind] = min(ts) * 1e3
    pts = S * F * n
    print('%-8s n=%5d power_mean %.3f ms (%.3e pts/s)  itc %.3f ms  power %.3f ms (%.3e pts/s)' % (
        tag, n, res['power_mean'], pts / res['power_mean'] * 1e3, res['itc'], res['power'], pts / res['power'] * 1e3),
        flush=True)

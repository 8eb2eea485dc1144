"""Step time of the C2 workload with and without per-stage HIP events (diagnostic)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import ninwavelets_amd as nw
from ninwavelets_amd import _lib as L

n, F, S = 16384, 128, 64
x = torch.randn(S, n, device='cuda', dtype=torch.float32)
out = [torch.empty((S, F, n), dtype=torch.complex64, device='cuda') for _ in range(2)]
for timing in (True, False, True, False):
    plan = nw.Plan(n, F, 'float32', device=0, max_batch=S, timing=timing)
    plan.set_wavelet('morlet', [7.0, 0.0], np.arange(1, F + 1, dtype=np.float64), L.trans_grid(n / 1000., 1000., False))
    for i in range(5):
        plan.execute_ptr(x.data_ptr(), S, out[i % 2].data_ptr(), 'cwt')
    plan.sync(); torch.cuda.synchronize()
    K = 200
    t0 = time.perf_counter()
    for i in range(K):
        plan.execute_ptr(x.data_ptr(), S, out[i % 2].data_ptr(), 'cwt')
    plan.sync(); torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / K
    st = plan.stats()
    print(f'timing={timing} ms/step={el*1e3:.4f} fused_ms={st["ms_fused"]/max(1,st["launches_fused"]):.4f}', flush=True)

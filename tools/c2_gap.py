"""Where a C2 step's time goes beyond its fused kernel.

C2 (Morlet cwt 64 x 16384 x 128 fp32) is one forward R2C launch + one fused launch per step.
This runs the bench's C2 step loop in three forms on one plan and prints one JSON line:
  timing:    a plan with NW_TIMING (events around every launch), K steps;
  chain:     the bench's plan (NW_TIMING | NW_TIMING_CHAIN: stop events ride on the dispatches,
             every stage starts at the previous stage's stop, no marker packets);
  notiming:  the same loop on a plan without events;
(--reps R repeats the chain / notiming pair R times, alternating, on one box.)
  enqueue:   host time to enqueue K steps without waiting (is the host the bound?).
Run it under `rocprofv3 --kernel-trace` to get the kernels' own timeline (tools/trace_gaps.py).
    python tools/c2_gap.py [--steps 40] [--warmup 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--reps', type=int, default=1)
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import ninwavelets_amd as nw
    from ninwavelets_amd import _lib as L
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    n, F, S = 16384, 128, 64
    freqs = np.arange(1, 129, dtype=np.float64)
    x = bench.synth_device(torch, S, n, seed=1000, device=dev)
    out = torch.empty((S, F, n), dtype=torch.complex64, device=dev)
    grid = L.trans_grid(n / 1000., 1000., False)
    res = {}
    forms = [('timing', True, False)] + [(f'{nm}{i if args.reps > 1 else ""}', t, c)
                                         for i in range(args.reps)
                                         for nm, t, c in (('chain', True, True), ('notiming', False, False))]
    for name, timing, chain in forms:
        plan = nw.Plan(n, F, 'float32', device=0, max_batch=S, timing=timing, timing_chain=chain)
        plan.set_wavelet('morlet', [7.0, 0.0], freqs, grid)

        def step():
            plan.execute_ptr(x.data_ptr(), S, out.data_ptr(), 'cwt')

        for _ in range(args.warmup):
            step()
        plan.sync()
        torch.cuda.synchronize()
        plan.reset_stats()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        t_enq = time.perf_counter() - t0
        plan.sync()
        el = time.perf_counter() - t0
        st = plan.stats()
        r = {'ms_per_step': el / args.steps * 1e3, 'enqueue_ms_per_step': t_enq / args.steps * 1e3}
        if timing:
            r['event_ms_fused'] = st['ms_fused'] / max(1, st['launches_fused'])
            r['event_ms_forward_per_step'] = st['ms_forward'] / args.steps
        res[name] = r
        plan.close()
    print(json.dumps({'config': 'c2 Morlet cwt 64 x 16384 x 128 fp32', 'steps': args.steps,
                      'warmup': args.warmup, **res}), flush=True)


if __name__ == '__main__':
    main()

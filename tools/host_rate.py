"""Host-buffer (numpy in / numpy out) throughput of the drop-in API (diagnostic):
the PCIe-inclusive rate DESIGN.md quotes beside the HBM-resident bench value."""
import json
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime: torch first)

sys.path.insert(0, '.')
import ninwavelets_amd as nw  # noqa: E402


def main():
    S, n, F = 64, 16384, 128              # C2 shape: 1.07 GB complex64 out
    rng = np.random.default_rng(0)
    x = rng.standard_normal((S, n)).astype(np.float32)
    freqs = np.arange(1, F + 1, dtype=np.float64)
    w = nw.Morlet(1000, dtype='float32')
    out = w.cwt_batch(x, freqs)           # warm-up: plan, W table, first-touch of the host output
    res = {}
    for kind in ('cwt', 'power'):
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            out = w.cwt_batch(x, freqs, out=kind)
        el = (time.perf_counter() - t0) / reps
        res[kind] = {'s_per_call': el, 'points_per_s': S * n * F / el,
                     'GB_out_per_s': out.nbytes / el / 1e9}
    # the same, writing into one reused (already faulted-in) output array
    plan = w._plan(n, S, 0)
    o = np.empty((S, F, n), dtype=np.complex64)
    plan.execute(x, out=o, out_kind='cwt')
    t0 = time.perf_counter()
    for _ in range(3):
        plan.execute(x, out=o, out_kind='cwt')
    el = (time.perf_counter() - t0) / 3
    res['cwt_reused_out'] = {'s_per_call': el, 'points_per_s': S * n * F / el, 'GB_out_per_s': o.nbytes / el / 1e9}
    print(json.dumps(res))


if __name__ == '__main__':
    main()

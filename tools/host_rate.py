"""Host-buffer (numpy in / numpy out) throughput of the drop-in API (diagnostic):
the PCIe-inclusive rate DESIGN.md quotes beside the HBM-resident bench value."""
import json
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime: torch first)

sys.path.insert(0, '.')
import ninwavelets_amd as nw  # noqa: E402


def rate(dtype, reps=3):
    S, n, F = 64, 16384, 128              # C2 shape: 1.07 GB complex64 out (2.15 GB complex128)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((S, n)).astype(dtype)
    freqs = np.arange(1, F + 1, dtype=np.float64)
    w = nw.Morlet(1000, dtype=dtype)
    out = w.cwt_batch(x, freqs)           # warm-up: plan, W table
    del out
    res = {}
    for kind in ('cwt', 'power'):
        t0 = time.perf_counter()
        for _ in range(reps):             # a new result per call, dropped before the next one: the
            out = w.cwt_batch(x, freqs, out=kind)      # pool hands the same page-locked buffer back
            del out
        el = (time.perf_counter() - t0) / reps
        res[kind + '_recycled_result'] = {
            's_per_call': el, 'points_per_s': S * n * F / el,
            'GB_out_per_s': S * n * F * (2 if kind == 'cwt' else 1) * x.itemsize / el / 1e9}
    # results the caller KEEPS (the reference's new array per call, all alive): the pool fills
    # to its cap (engine.HOST_POOL.cap page-locked bytes), then results are fresh pageable
    # arrays advised onto huge pages (nw_host_advise)
    from ninwavelets_amd import engine
    nbytes = S * F * n * 2 * x.itemsize
    keep = int(min(24, max(4, 3 * engine.HOST_POOL.cap // nbytes)))
    kept = []
    t0 = time.perf_counter()
    for _ in range(keep):
        kept.append(w.cwt_batch(x, freqs))
    el = (time.perf_counter() - t0) / keep
    res['cwt_kept_results'] = {'s_per_call': el, 'points_per_s': S * n * F / el, 'GB_out_per_s': nbytes / el / 1e9,
                               'results_kept': keep, 'pool_cap_bytes': engine.HOST_POOL.cap,
                               'pooled_results': sum(1 for k in kept if engine.host_pinned_array(k))}
    del kept
    # the same, writing into one reused (already faulted-in) output array
    plan = w._plan(n, S, 0)
    o = np.empty((S, F, n), dtype=np.complex64 if dtype == 'float32' else np.complex128)
    plan.execute(x, out=o, out_kind='cwt')
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.execute(x, out=o, out_kind='cwt')
    el = (time.perf_counter() - t0) / reps
    res['cwt_reused_out'] = {'s_per_call': el, 'points_per_s': S * n * F / el, 'GB_out_per_s': o.nbytes / el / 1e9}
    return res


def main():
    print(json.dumps({'shape': 'C2: 64 x 16384 x 128 Morlet, numpy in / numpy out',
                      'float32': rate('float32'), 'float64': rate('float64')}))


if __name__ == '__main__':
    main()

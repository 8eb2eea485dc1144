"""bench.py's real multi-rank path with kernels (the driver's N-GPU runs take it with nccl):
two ranks started by bench.py's own launcher, gloo process group, both ranks on the lease's
one GPU (--same-device), real fused-engine launches, barrier-bracketed timing and the max
over ranks.  The batching sharded here is the reference's per-epoch loop
(/root/reference/ninwavelets/mneutils.py:39).  Also the default C4 line's fp64 leg (the
reference's complex128 precision, base.py:399-406) on a small epoch count."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def run_bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args], capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), r.stderr


def test_two_ranks_share_the_gpu_with_kernels():
    d, err = run_bench('--gpus', '2', '--backend', 'gloo', '--same-device', '--config', 'c3', '--epochs', '8',
                       '--steps', '2', '--warmup', '1', '--no-cpu-baseline')
    assert d['n_gpus'] == 2 and d['steps'] == 2
    assert d['value'] > 0 and d['ms_per_step'] > 0
    assert d['config']['parallelism'].startswith('dp2') and d['config']['same_device']
    assert d['config']['epochs'] == 16                      # weak scaling: 8 epochs per rank
    assert d['roofline']['kernel'] == 'nw_fused_pair_kernel' and d['roofline']['avg_launch_ms'] > 0
    assert d['valu_roofline']['frac'] > 0
    # both ranks ran real launches
    assert err.count('engine=fused') == 2, err[-2000:]
    # value = all ranks' points / the slowest rank's time
    pts = 2 * 8 * 64 * 4096 * 256 * 2
    assert abs(d['value'] - pts / (d['ms_per_step'] * 2e-3)) <= 1e-6 * d['value']


def test_c4_line_carries_an_fp64_leg():
    d, _ = run_bench('--config', 'c4', '--epochs', '2', '--steps', '1', '--warmup', '1', '--no-cpu-baseline')
    assert d['dtype'] == 'f32' and d['roofline']['kernel'] == 'nw_fused_kernel'
    f = d['fp64']
    assert f['dtype'] == 'f64' and f['value'] > 0 and 'complex128' in f['workload']
    assert f['roofline']['kernel'] == 'nw_fused_kernel' and f['roofline']['frac'] > 0
    # the fp64 leg moves twice the bytes per point
    assert f['roofline']['algorithmic_bytes_per_launch'] == pytest.approx(
        2 * d['roofline']['algorithmic_bytes_per_launch'])
    assert f['valu_roofline']['peak'] == 78.6

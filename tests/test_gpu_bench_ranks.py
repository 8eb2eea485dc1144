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
    d, _ = run_bench('--config', 'c4', '--epochs', '2', '--steps', '1', '--warmup', '1', '--no-cpu-baseline',
                     '--legs', 'fp64')
    assert d['dtype'] == 'f32' and d['roofline']['kernel'] == 'nw_fused_kernel'
    assert 'c3' not in d and 'c5' not in d
    f = d['fp64']
    assert f['dtype'] == 'f64' and f['value'] > 0 and 'complex128' in f['workload']
    assert f['roofline']['kernel'] == 'nw_fused_kernel' and f['roofline']['frac'] > 0
    # the fp64 leg moves twice the bytes per point
    assert f['roofline']['algorithmic_bytes_per_launch'] == pytest.approx(
        2 * d['roofline']['algorithmic_bytes_per_launch'])
    assert f['valu_roofline']['peak'] == 78.6


def test_default_line_carries_c3_and_c5_legs():
    """BASELINE.json's C3 (fused |.|^2, base.py:409-425) and C5 (2^24 samples x 512 scales,
    fp32 and fp64, base.py:404-406) ride on the default line with their own rooflines."""
    d, _ = run_bench('--config', 'c4', '--epochs', '2', '--steps', '1', '--warmup', '1', '--no-cpu-baseline',
                     '--legs', 'c2,c3,c5,c5_fp64', timeout=600)
    assert d['fp64'] is None
    c2 = d['c2']                                 # Morlet cwt 64 x 16384 x 128 (wavelets.py:132-136)
    assert c2['dtype'] == 'f32' and c2['output'] == 'cwt' and c2['roofline']['kernel'] == 'nw_fused_kernel'
    assert c2['value'] == pytest.approx(64 * 16384 * 128 / (c2['ms_per_step'] * 1e-3), rel=1e-9)
    assert (c2['steps'], c2['warmup']) == (400, 40)     # bench.LEG_MIN_STEPS: ~90 ms of steady state
    assert c2['scaling'] == 'weak' and c2['parallelism'].startswith('dp1')
    c3 = d['c3']
    assert c3['dtype'] == 'f32' and c3['output'] == 'power' and c3['value'] > 0
    assert c3['roofline']['kernel'] == 'nw_fused_pair_kernel' and c3['roofline']['frac'] > 0
    # --epochs scales C3's epochs down: 2 epochs x 64 ch x 4096 x 256 per step
    assert c3['value'] == pytest.approx(2 * 64 * 4096 * 256 / (c3['ms_per_step'] * 1e-3), rel=1e-9)
    assert c3['valu_roofline']['kernel'] == 'nw_fused_pair_kernel'
    for key, dt, peak in (('fp32', 'f32', 157.3), ('fp64', 'f64', 78.6)):
        c5 = d['c5'][key]
        assert c5['dtype'] == dt and c5['output'] == 'cwt'
        assert c5['roofline']['kernel'] == 'cols_kernel' and c5['roofline_rows']['kernel'] == 'rows_kernel'
        assert c5['value'] == pytest.approx((1 << 24) * 512 / (c5['ms_per_step'] * 1e-3), rel=1e-9)
        esz = 4 if dt == 'f32' else 8
        # end to end against X once + every output once
        assert c5['end_to_end_min_traffic']['bytes_per_step'] == pytest.approx(
            ((1 << 23) + 1) * 2 * esz + 512 * (1 << 24) * 2 * esz)
        assert c5['valu_roofline']['peak'] == peak
        assert c5['scaling'] == 'weak' and c5['parallelism'].startswith('dp1')     # one rank


def test_two_ranks_split_c5_scales_with_kernels():
    """The driver's N > 1 line on C5 (one 2^24-sample signal, base.py:404-406): each rank
    computes a contiguous slice of the 512 scales of the SAME signal (strong scaling, SURVEY
    §8e), with real two-pass launches on both ranks; value = the whole job's points / the
    slowest rank's time.  C2 rides the same line signal-sharded (weak)."""
    d, err = run_bench('--gpus', '2', '--backend', 'gloo', '--same-device', '--config', 'c4', '--epochs', '1',
                       '--steps', '1', '--warmup', '1', '--no-cpu-baseline', '--legs', 'c2,c5', timeout=600)
    assert d['n_gpus'] == 2 and d['scaling'] == 'weak'
    c5 = d['c5']['fp32']
    assert c5['scaling'] == 'strong' and c5['parallelism'].startswith('scales2')
    assert c5['scale_slices'] == [[0, 256], [256, 512]]
    assert c5['value'] == pytest.approx((1 << 24) * 512 / (c5['ms_per_step'] * 1e-3), rel=1e-9)
    assert c5['roofline']['kernel'] == 'cols_kernel'
    assert d['c2']['scaling'] == 'weak' and d['c2']['parallelism'].startswith('dp2')
    assert d['c2']['value'] == pytest.approx(2 * 64 * 16384 * 128 / (d['c2']['ms_per_step'] * 1e-3), rel=1e-9)
    assert err.count('c5: S=1 n=16777216 F=256') == 2, err[-3000:]


def test_rccl_single_rank_bench_path():
    """The driver's N-GPU launch (torchrun, one rank per GPU, backend nccl = RCCL) at N = 1 on
    the lease: process group over RCCL, barriers, the device all_reduce(MAX) of the elapsed
    time, real kernels (the sharded loop is mneutils.py:39's per-epoch batching)."""
    from test_dist_cpu import free_port
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
                        '--master-addr', '127.0.0.1', '--master-port', str(free_port()),
                        os.path.join(ROOT, 'bench.py'), '--config', 'c3', '--epochs', '4', '--steps', '2',
                        '--warmup', '1', '--backend', 'nccl', '--no-cpu-baseline'],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    d = json.loads(lines[0])
    assert d['config']['process_group'] == 'nccl' and d['n_gpus'] == 1
    assert d['value'] > 0 and d['roofline']['kernel'] == 'nw_fused_pair_kernel'


def _nccl_worker(rank, world, port, out_dir):
    import numpy as np
    import torch
    import torch.distributed as dist
    import ninwavelets_amd as nw
    from ninwavelets_amd import dist as D
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', 0))
    try:
        rng = np.random.default_rng(11)
        x = rng.standard_normal((7, 2048))
        freqs = [3., 9., 27., 81.]
        p = D.epochs_reduce(nw.Morse(1000), x, freqs, 'power_mean')
        local = nw.Morse(1000).cwt(x[0], freqs)              # one rank: its slice is every scale
        g = D.gather_scales(local, 4, device=torch.device('cuda', 0))
        np.savez(os.path.join(out_dir, 'nccl.npz'), power=p, gathered=g, local=local, x=x)
    finally:
        dist.destroy_process_group()


def test_rccl_device_collectives_of_dist(tmp_path):
    """dist.epochs_reduce's device all_reduce and gather_scales' all_gather through RCCL (one
    rank on the lease's GPU: RCCL takes one GPU per rank), against the oracle."""
    import numpy as np
    import torch.multiprocessing as mp
    from oracle import nw_oracle as O
    from test_dist_cpu import free_port
    mp.spawn(_nccl_worker, args=(1, free_port(), str(tmp_path)), nprocs=1, join=True)
    got = np.load(tmp_path / 'nccl.npz')
    c = O.epochs_cwt('morse', got['x'], [3., 9., 27., 81.])
    ref = np.mean(np.abs(c) ** 2, axis=0)
    assert np.max(np.abs(got['power'] - ref)) <= 1e-12 * np.max(ref)
    np.testing.assert_array_equal(got['gathered'], got['local'])

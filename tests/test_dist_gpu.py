"""dist.epochs_reduce end to end on the GPU box: two ranks (gloo process group, both on
the box's one GPU -- RCCL needs one GPU per rank) each reduce their block of epochs on
the device; one all_reduce gives every rank EpochsWavelet.power / itc (mneutils.py:42-71)."""
import os

import numpy as np
import pytest

from oracle import nw_oracle as O

pytestmark = pytest.mark.gpu

FREQS = [2., 5., 11., 23., 47., 95.]


def data(E=9, n=2048, seed=5):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 1000.
    return np.sin(2 * np.pi * rng.uniform(1, 60, (E, 1)) * t) + 0.1 * rng.standard_normal((E, n))


def _worker(rank, world, port, out_dir):
    import torch  # noqa: F401  (one HIP runtime: torch first)
    import torch.distributed as dist
    import ninwavelets_amd as nw
    from ninwavelets_amd import dist as D
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        x = data()
        p = D.epochs_reduce(nw.Morse(1000), x, FREQS, 'power_mean')
        i = D.epochs_reduce(nw.Morse(1000), x, FREQS, 'itc')
        np.savez(os.path.join(out_dir, f'rank{rank}.npz'), power=p, itc=i)
    finally:
        dist.destroy_process_group()


def test_two_rank_epochs_reduce_on_device(tmp_path):
    import torch.multiprocessing as mp
    from test_dist_cpu import free_port
    mp.spawn(_worker, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    c = O.epochs_cwt('morse', data(), FREQS)
    ref_p = np.mean(np.abs(c) ** 2, axis=0)
    ref_i = np.abs(np.mean(c / np.abs(c), axis=0))
    for r in range(2):
        got = np.load(tmp_path / f'rank{r}.npz')
        assert np.max(np.abs(got['power'] - ref_p)) <= 1e-12 * np.max(ref_p)
        assert np.max(np.abs(got['itc'] - ref_i)) <= 1e-10

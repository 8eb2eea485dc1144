"""The N > 1 path on CPU: world_size-2 gloo process groups (no GPU needed).

Covers the sharding of signals over ranks (contiguous blocks, no collective) and
the one real exchange, the all_reduce of fp64 epoch-reduction partial sums
(ninwavelets_amd/dist.py).  The per-rank partial sums here come from the CPU
oracle (the checker), standing in for each rank's device result."""
import os
import socket

import numpy as np
import pytest

from oracle import nw_oracle as O

from ninwavelets_amd import dist as D

FREQS = [2., 5., 11., 23., 47.]


def free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def epochs(E=7, n=512, seed=3):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 1000.
    x = np.sin(2 * np.pi * rng.uniform(1, 60, (E, 1)) * t) + 0.1 * rng.standard_normal((E, n))
    if E > 4:
        x[4] = 0.0                                # an all-zero epoch: ITC is NaN (mneutils.py:68)
    return x


def oracle_partials(x, s0, s1):
    c = O.epochs_cwt('morse', x[s0:s1], FREQS) if s1 > s0 else np.zeros((0, len(FREQS), x.shape[1]))
    with np.errstate(invalid='ignore', divide='ignore'):
        return np.sum(np.abs(c) ** 2, axis=0), np.sum(c / np.abs(c), axis=0)


def _worker(rank, world, port, E, out_dir):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        x = epochs(E)
        s0, s1 = D.shard(E, rank, world)
        pw, ph = oracle_partials(x, s0, s1)
        if s1 == s0:
            pw = np.zeros((len(FREQS), x.shape[1]))
            ph = np.zeros((len(FREQS), x.shape[1]), dtype=np.complex128)
        power = D.reduce_partials(pw, 'power_mean', E, np.float64)
        itc = D.reduce_partials(ph, 'itc', E, np.float64)
        np.savez(os.path.join(out_dir, f'rank{rank}.npz'), power=power, itc=itc)
    finally:
        dist.destroy_process_group()


def _scale_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        x = epochs(1, n=1024)[0]
        f0, f1 = D.shard(len(FREQS), rank, world)
        # this rank's slice of the scales (the oracle stands in for the rank's device)
        local = np.stack([O.cwt('morse', x, [f, f])[0] for f in FREQS[f0:f1]]) if f1 > f0 \
            else np.zeros((0, x.size), dtype=np.complex128)
        full = D.gather_scales(local, len(FREQS))
        np.save(os.path.join(out_dir, f'scales{rank}.npy'), full)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_scale_sharded_ranks_gather_the_full_cwt(tmp_path, world):
    """One signal, scales split over ranks: every rank computes its
    contiguous slice and gather_scales rebuilds the (F, n) result on every rank."""
    import torch.multiprocessing as mp
    mp.spawn(_scale_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    x = epochs(1, n=1024)[0]
    ref = O.cwt('morse', x, FREQS)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f'scales{r}.npy'), ref)


def test_shard_blocks_cover_every_signal_once():
    for nsig in [0, 1, 2, 7, 64, 1000, 262144]:
        for world in [1, 2, 3, 8]:
            blocks = [D.shard(nsig, r, world) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == nsig
            for (a0, a1), (b0, b1) in zip(blocks, blocks[1:]):
                assert a1 == b0 and a0 <= a1
    with pytest.raises(ValueError):
        D.shard(4, 2, 2)


def test_shard_is_balanced_and_never_empty():
    """Every block holds nsig // world or one more item, so no rank (device, scale slice)
    is empty while nsig >= world: e.g. 10 scales over 8 devices, 5 over 4."""
    for nsig in range(0, 70):
        for world in range(1, 10):
            sizes = [b - a for a, b in (D.shard(nsig, r, world) for r in range(world))]
            assert sum(sizes) == nsig
            assert max(sizes) - min(sizes) <= 1
            if nsig >= world:
                assert min(sizes) >= 1, (nsig, world)
    assert [D.shard(10, r, 8) for r in range(8)][-1] == (9, 10)
    assert D.shard(5, 3, 4) == (4, 5)


def test_finalize_matches_numpy_mean():
    rng = np.random.default_rng(0)
    c = rng.standard_normal((9, 3, 17)) + 1j * rng.standard_normal((9, 3, 17))
    p = D.finalize('power_mean', np.sum(np.abs(c) ** 2, axis=0), 9, np.float64)
    np.testing.assert_allclose(p, np.mean(np.abs(c) ** 2, axis=0), rtol=1e-14)
    i = D.finalize('itc', np.sum(c / np.abs(c), axis=0), 9, np.float32)
    assert i.dtype == np.float32
    np.testing.assert_allclose(i, np.abs(np.mean(c / np.abs(c), axis=0)), rtol=1e-6)


@pytest.mark.parametrize('E', [7, 1])
def test_two_rank_gloo_epoch_reduction(tmp_path, E):
    """world_size 2: each rank sums its block, one all_reduce, every rank gets the
    reference's power / ITC (E = 1 leaves rank 1 with no epochs)."""
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, free_port(), E, str(tmp_path)), nprocs=2, join=True)
    x = epochs(E)
    c = O.epochs_cwt('morse', x, FREQS)
    with np.errstate(invalid='ignore', divide='ignore'):
        ref_p = np.mean(np.abs(c) ** 2, axis=0)
        ref_i = np.abs(np.mean(c / np.abs(c), axis=0))
    for r in range(2):
        got = np.load(tmp_path / f'rank{r}.npz')
        np.testing.assert_allclose(got['power'], ref_p, rtol=1e-12)
        np.testing.assert_array_equal(np.isnan(got['itc']), np.isnan(ref_i))
        ok = ~np.isnan(ref_i)
        np.testing.assert_allclose(got['itc'][ok], ref_i[ok], rtol=1e-12, atol=1e-14)

"""One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on MI355X).

The CWT shards with no exchange at all: signals (epoch x channel) are independent,
so rank r transforms the contiguous block ``shard(nsig, r, world)`` of them (the
same split nw_execute_multi uses across devices).  The only real
exchange is the epoch reduction of EpochsWavelet.power / itc (mneutils.py:42-71):
each rank sums its block in fp64 on its device (``power_sum`` / ``phase_sum``),
one all_reduce adds the partial sums, and every rank finalises the mean -- F x n
values per collective, independent of the number of epochs.

One long signal (C5: 1 x 2^24) cannot shard by signal: there the ranks split the SCALE
list instead (``shard(nfreq, rank, world)``, each rank computing every signal for its
contiguous slice, its own forward FFT, no exchange), and ``gather_scales`` is the
optional all_gather of the slices when one process needs the whole (..., F, n) result.
"""
from __future__ import annotations

import numpy as np

from .engine import REDUCTIONS

_SUM_OF = {'power_mean': 'power_sum', 'itc': 'phase_sum',
           'power_sum': 'power_sum', 'phase_sum': 'phase_sum'}


def shard(nsig: int, rank: int, world: int) -> tuple[int, int]:
    """[s0, s1) of rank's contiguous block, balanced: nsig // world items per rank and one
    more for the first nsig % world ranks, so no rank is empty while nsig >= world (the
    same split nw_execute_multi / nw_execute_multi_scales use across devices)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f'bad rank {rank} of {world}')
    base, extra = divmod(nsig, world)
    s0 = rank * base + min(rank, extra)
    return s0, s0 + base + (1 if rank < extra else 0)


def finalize(kind: str, total: np.ndarray, nsig: int, dtype) -> np.ndarray:
    """Mean (np.mean's sum / count) or |mean of phasors| from fp64 sums, as the device's
    k_finalize and nw_execute_multi do."""
    if kind in ('power_sum', 'phase_sum'):
        return total
    with np.errstate(invalid='ignore', divide='ignore'):
        if kind == 'power_mean':
            return (total / nsig).astype(dtype)
        return np.hypot(total.real / nsig, total.imag / nsig).astype(dtype)


def reduce_partials(partial: np.ndarray, kind: str, nsig: int, dtype, group=None,
                    device=None) -> np.ndarray:
    """all_reduce(SUM) the fp64 partial sums of every rank, then finalise ``kind``.
    ``device``: where the collective runs (a CUDA device for RCCL; None = CPU for gloo)."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(partial))
    if t.is_complex():
        t = torch.view_as_real(t)
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    t = t.cpu()
    total = torch.view_as_complex(t).numpy() if partial.dtype == np.complex128 else t.numpy()
    return finalize(kind, total, nsig, dtype)


def epochs_reduce(wavelet, waves: np.ndarray, freqs, kind: str, group=None) -> np.ndarray:
    """EpochsWavelet.power / itc of ``waves`` (epochs, n) over all ranks of ``group``:
    this rank transforms only its block of epochs on its GPU, then one all_reduce."""
    import torch
    import torch.distributed as dist
    if kind not in REDUCTIONS:
        raise ValueError(f'kind must be one of {REDUCTIONS}')
    waves = np.asarray(waves)
    nsig, n = waves.shape[0], waves.shape[-1]
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if wavelet._cache is None:
        wavelet._build_cache(freqs, n / wavelet.sfreq)     # reuse=True semantics (mneutils.py:39)
    s0, s1 = shard(nsig, rank, world)
    sum_kind = _SUM_OF[kind]
    nf = len(wavelet._cache.freqs)
    if s1 > s0:
        part = wavelet.cwt_batch(waves[s0:s1], freqs, reuse=True, out=sum_kind)
    else:
        part = np.zeros((nf, n), dtype=np.complex128 if sum_kind == 'phase_sum' else np.float64)
    dev = None
    if dist.get_backend(group) == 'nccl':
        dev = torch.device('cuda', torch.cuda.current_device())
    return reduce_partials(part, kind, nsig, wavelet.dtype, group, dev)


def gather_scales(local: np.ndarray, nfreq: int, group=None, device=None) -> np.ndarray:
    """All ranks' scale slices -> the full (..., nfreq, n) array on every rank.  ``local``
    is this rank's (..., f1 - f0, n) result for ``shard(nfreq, rank, world)``; slices are
    padded to ceil(nfreq / world) rows for the fixed-size all_gather and trimmed after.
    ``device``: where the collective runs (a CUDA device for RCCL; None = CPU for gloo)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    per = -(-nfreq // world)
    loc = np.ascontiguousarray(local)
    pad = np.zeros(loc.shape[:-2] + (per, loc.shape[-1]), dtype=loc.dtype)
    pad[..., :loc.shape[-2], :] = loc
    t = torch.from_numpy(pad)
    if t.is_complex():
        t = torch.view_as_real(t)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    rows = []
    for r, part in enumerate(parts):
        part = part.cpu()
        a = torch.view_as_complex(part).numpy() if np.iscomplexobj(loc) else part.numpy()
        f0, f1 = shard(nfreq, r, world)
        rows.append(a[..., :f1 - f0, :])
    return np.concatenate(rows, axis=-2)

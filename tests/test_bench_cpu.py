"""bench.py's multi-rank plumbing on CPU (no GPU, no kernels): the launcher that starts
N fresh ranks itself, the gloo process group, the barrier-bracketed timing and the
MAX over ranks (the driver's N = 1, 2, 4, 8 runs take the same path with nccl)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run(*args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args], capture_output=True,
                       text=True, timeout=240, env=e)
    return r


@pytest.mark.parametrize('gpus', [1, 2, 3])
def test_launcher_runs_n_ranks_dry(gpus):
    r = run('--gpus', str(gpus), '--dry-run', '--steps', '3', '--warmup', '1')
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1                       # rank 0's line only
    d = json.loads(lines[0])
    assert d['n_gpus'] == gpus and d['steps'] == 3 and d['warmup'] == 1
    assert d['config']['parallelism'] == f'dp{gpus}'
    # rank r sleeps 10 ms * (r + 1) per step: the reported step is the slowest rank's
    assert d['ms_per_step'] >= 10.0 * gpus * 0.95


def test_world_size_mismatch_fails_loudly():
    r = run('--gpus', '4', '--dry-run', env={'WORLD_SIZE': '2', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert r.returncode != 0
    assert 'WORLD_SIZE' in r.stderr


def test_pmc_traffic_needs_current_sources(tmp_path, monkeypatch):
    """A committed PMC summary is attached only when its engine-source hash matches."""
    h = bench.source_hash()
    assert len(h) == 16 and h == bench.source_hash()
    prof = tmp_path / 'profiles'
    prof.mkdir()
    cfg = {'chunk': 8, 'n': 4096, 'dtype': 'float32', 'out': 'power'}
    (prof / 'pmc_cx_a.json').write_text(json.dumps({'kernel': 'k', 'hbm_bytes_per_launch': 5.0,
                                                    'config': dict(cfg, src_hash='0' * 16)}))
    monkeypatch.setattr(bench, 'ROOT', str(tmp_path))
    monkeypatch.setattr(bench, 'source_hash', lambda: h)
    assert bench.pmc_traffic('k', 'cx', 8, 'fused', 'float32', 'power', 4096) == (None, None)
    (prof / 'pmc_cx_b.json').write_text(json.dumps({'kernel': 'k', 'hbm_bytes_per_launch': 7.0,
                                                    'config': dict(cfg, src_hash=h)}))
    got, src = bench.pmc_traffic('k', 'cx', 8, 'fused', 'float32', 'power', 4096)
    assert got == 7.0 and src.endswith('pmc_cx_b.json')
    assert bench.pmc_traffic('k', 'cx', 16, 'fused', 'float32', 'power', 4096) == (None, None)


def test_cpu_model_is_reported():
    assert isinstance(bench.cpu_model(), str) and bench.cpu_model()


def test_launcher_fails_fast_when_a_rank_dies():
    """Rank 1 exits 3 before the rendezvous: the launcher must notice, terminate rank 0
    (which would otherwise wait for its peer until the process-group timeout) and return 3."""
    import time
    t0 = time.monotonic()
    r = run('--gpus', '2', '--dry-run', '--steps', '2', '--warmup', '1', '--fail-rank', '1')
    el = time.monotonic() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert el < bench.PG_TIMEOUT_S / 2, el
    assert 'rank 1 exited with 3' in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith('{')]


def test_launcher_fails_fast_when_rank0_dies():
    r = run('--gpus', '3', '--dry-run', '--steps', '2', '--warmup', '1', '--fail-rank', '0')
    assert r.returncode == 3, r.stderr[-2000:]


def test_fft_flops_model():
    # 5 n log2 n + 2 n per row; the chirp-z form: two M-point transforms, M = 2^ceil(log2(2n - 1))
    assert bench.fft_flops_per_row(4096, 'nw_fused_pair_kernel') == 5 * 4096 * 12 + 2 * 4096
    assert bench.fft_flops_per_row(1201, 'nw_chirp_kernel') == 2 * 5 * 4096 * 12 + 2 * 1201


@pytest.mark.parametrize('gpus', [2, 3])
def test_c5_ranks_split_the_scales_dry(gpus):
    """C5 is one 2^24-sample signal per config: at N > 1 ranks the default partition (--shard
    auto) gives every rank a contiguous slice of the 512 scales of the same signal (strong
    scaling); the slices, gathered from the ranks themselves, tile [0, 512)."""
    r = run('--gpus', str(gpus), '--dry-run', '--config', 'c5', '--steps', '1', '--warmup', '0')
    assert r.returncode == 0, r.stderr
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][0])
    assert d['scaling'] == 'strong' and d['config']['parallelism'] == f'scales{gpus}'
    sl = d['config']['scale_slices']
    assert len(sl) == gpus and sl[0][0] == 0 and sl[-1][1] == 512
    assert all(a[1] == b[0] for a, b in zip(sl, sl[1:])) and all(b - a >= 512 // gpus for a, b in sl)


def test_partition_rule():
    assert bench.shards_scales('auto', 1, 8) and not bench.shards_scales('auto', 1, 1)
    assert not bench.shards_scales('auto', 32768, 8) and bench.shards_scales('scales', 32768, 2)
    assert not bench.shards_scales('signals', 1, 8)
    assert set(bench.LEGS) == {'fp64', 'c2', 'c3', 'c5', 'c5_fp64'}

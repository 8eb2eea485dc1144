"""Throughput bench of the MI355X CWT engine (driver contract: one JSON line).

Default workload (the north_star target, BASELINE.json configs[3]): Morse CWT of
512 epochs x 64 channels x 16384 samples x 256 freqs PER GPU, fp32 -- weak
scaling, so 8 GPUs process the full 4096-epoch config.  A "step" is one pass of
the hot path over that batch: forward rocFFT of every signal, then the
spectrum-multiply / inverse-FFT engine writing every (signal, freq, sample)
output point to HBM.  Inputs are resident in HBM before timing starts; the
complex output (1.1 TB per GPU per step) is streamed through two rotating HBM
chunk buffers.  Signals are sharded over ranks with no collective on the data
path (the barrier and a max-reduce of the elapsed time are timing only).

    python bench.py [--gpus N --steps K --warmup W] [--config c4|c3|c2|c5] [--engine auto|rocfft|fused]

Multi-GPU: under torchrun (WORLD_SIZE set) every process is one rank.  Without it,
``--gpus N`` (N > 1) makes this process a launcher that never touches the GPU: it starts
N fresh child processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT), waits for them and prints rank 0's line.  ``--dry-run --backend gloo``
runs the same multi-rank flow on CPU without any kernel (tests/test_bench_cpu.py).
"""
from __future__ import annotations

import argparse
import copy
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

DEFAULT_CHUNK = {'c4': 512, 'c3': 1024, 'c2': 64, 'c5': 1}   # signals per fused launch (tools/chunk_sweep.sh)
PEAK_HBM_GBPS = 8000.0     # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)

CONFIGS = {
    # name: (kind, epochs per GPU, chans, n, freqs, out, dtype, workload text)
    'c4': ('morse', 512, 64, 16384, np.arange(1, 257, dtype=np.float64), 'cwt', 'float32',
           'C4 Morse CWT, 512 epochs x 64 ch x 16384 samples x 256 freqs per GPU '
           '(4096 epochs at 8 GPUs), complex64 out'),
    'c3': ('morse', 512, 64, 4096, np.arange(1, 257, dtype=np.float64), 'power', 'float32',
           'C3 Morse power, 512 epochs x 64 ch x 4096 samples x 256 freqs per GPU, float32 out'),
    'c2': ('morlet', 1, 64, 16384, np.arange(1, 129, dtype=np.float64), 'cwt', 'float32',
           'C2 Morlet CWT, 64 ch x 16384 samples x 128 freqs per GPU, complex64 out'),
    'c5': ('morse', 1, 1, 1 << 24, np.linspace(0.5, 250, 512), 'cwt', 'float32',
           'C5 Morse CWT, 1 signal x 2^24 samples x 512 freqs (linspace 0.5..250) per GPU, '
           'complex64 out (written into one HBM buffer)'),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synth_device(torch, S, n, seed, device, sfreq=1000., dtype=None):
    """Synthetic multi-channel sinusoids + noise, generated on the device."""
    dtype = dtype or torch.float32
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.empty((S, n), dtype=dtype, device=device)
    t = torch.arange(n, device=device, dtype=torch.float64) / sfreq
    step = 1024
    for s0 in range(0, S, step):
        s1 = min(S, s0 + step)
        fc = torch.rand((s1 - s0, 1), generator=g, device=device, dtype=torch.float64) * 99 + 1
        ph = torch.rand((s1 - s0, 1), generator=g, device=device, dtype=torch.float64) * 2 * np.pi
        noise = torch.randn((s1 - s0, n), generator=g, device=device, dtype=torch.float32)
        x[s0:s1] = ((torch.sin(2 * np.pi * fc * t + ph)) + 0.1 * noise).to(dtype)
    return x


def source_hash() -> str:
    """sha256 (16 hex) over the engine's sources (csrc/*.hip, *.h, *.cpp, include/ninwave.h):
    a PMC summary is attached to a bench line only when it was collected on these sources."""
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, 'ninwavelets_amd', 'csrc')
    files = sorted(f for f in os.listdir(csrc) if f.endswith(('.hip', '.h', '.cpp')))
    for f in files + ['../../include/ninwave.h']:
        with open(os.path.join(csrc, f), 'rb') as fh:
            h.update(os.path.basename(f).encode() + b'\0' + fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel, config, chunk, engine, dtype='float32', out=None, n=None):
    """(HBM bytes per launch, source) of `kernel` from the committed rocprofv3 PMC summary
    of this same bench command (tools/prof_counters.sh -> profiles/pmc_<config>_*.json):
    None unless the summary was taken on this kernel, chunk, dtype, output kind, n AND on
    the current engine sources (source_hash), so a stale profile is never reported."""
    import glob
    want = source_hash()
    for path in sorted(glob.glob(os.path.join(ROOT, 'profiles', f'pmc_{config}_*.json'))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        c = d.get('config', {})
        if d.get('kernel') != kernel or c.get('chunk') != chunk or c.get('dtype', 'float32') != dtype:
            continue
        if (out is not None and c.get('out', out) != out) or (n is not None and c.get('n', n) != n):
            continue
        if c.get('src_hash') != want:
            continue
        return d.get('hbm_bytes_per_launch'), os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(kind, n, freqs, out_kind, budget_s=12.0, piece_rows_log2=22):
    """The CPU oracle (numpy + scipy.fftpack, the reference's arithmetic) on one core.
    The wavelet rows are built untimed (reuse=True caches them in the reference); the
    timed work is fft(x) per signal, then pad_to + multiply + ifft (+ |.|^2) per piece
    of <= 32 MiB of rows, so C5's 2^24-sample rows are timed a few at a time."""
    from oracle import nw_oracle as O
    rng = np.random.default_rng(0)
    t = np.arange(n) / 1000.
    fc = int(max(2, min(len(freqs), (1 << piece_rows_log2) // n)))     # >= 2: freq_dist needs two (base.py:272)
    pieces, rows_done, sigs, el = {}, 0, 0, 0.0
    while el < budget_s:
        x = np.sin(2 * np.pi * rng.uniform(1, 100) * t) + 0.1 * rng.standard_normal(n)
        t0 = time.perf_counter()
        spec = O.fft(x)
        el += time.perf_counter() - t0
        sigs += 1
        for j in range(0, len(freqs), fc):
            if j not in pieces:
                pieces[j] = O.fft_wavelets(kind, freqs[j:j + fc], 1000., n / 1000., False)
            t0 = time.perf_counter()
            y = O.ifft(np.array([O.pad_to(r, n) for r in pieces[j]]) * spec)
            if out_kind == 'power':
                y = np.abs(y) ** 2
            el += time.perf_counter() - t0
            rows_done += len(pieces[j])
            if el >= budget_s:
                break
    return {'value': rows_done * n / el, 'unit': 'points/s', 'cores': 1, 'kind': 'port',
            'cpu_model': cpu_model(), 'sample_seconds': el, 'rows_done': rows_done,
            'sample': f'{rows_done} (signal, freq) rows of {n} samples over {sigs} signal(s) '
                      f'({kind} {out_kind}, oracle/nw_oracle.py single process, wavelet rows '
                      f'cached), {el:.1f} s'}


def _pool_worker(args):
    kind, n, freqs, out_kind, budget_s, seed = args
    import numpy as _np
    # 4x smaller pieces than the single-process leg: os.cpu_count() workers share host RAM
    r = cpu_baseline(kind, n, _np.asarray(freqs), out_kind, budget_s, piece_rows_log2=20)
    return r['value'] * r['sample_seconds'], r['sample_seconds'], r['rows_done']


def cpu_model() -> str:
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cpu_baseline_pool(kind, n, freqs, out_kind, budget_s=8.0, workers=None):
    """The same oracle work in multiprocessing.Pool(os.cpu_count()) over signals
    (BASELINE.md §3 mode b, uncapped): each worker times its own bounded sample; the rate
    is the sum of the workers' rates.  cores = the pool size; the CPUs this process may
    run on (sched_getaffinity) and the CPU model are recorded beside it."""
    import multiprocessing as mp
    workers = workers or os.cpu_count() or 1
    with mp.get_context('spawn').Pool(workers) as pool:
        res = pool.map(_pool_worker, [(kind, n, list(freqs), out_kind, budget_s, i) for i in range(workers)])
    rate = sum(pts / el for pts, el, _ in res)
    rows = sum(r for _, _, r in res)
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = None
    return {'value': rate, 'unit': 'points/s', 'cores': workers, 'kind': 'port',
            'cpu_model': cpu_model(), 'os_cpu_count': os.cpu_count(), 'cpus_allowed': allowed,
            'sample': f'{rows} (signal, freq) rows of {n} samples over {workers} processes '
                      f'(multiprocessing.Pool(os.cpu_count()), each ~{budget_s:.0f} s; sum of '
                      f'per-process rates)'}


def free_port() -> int:
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


PG_TIMEOUT_S = 120      # process-group rendezvous / collective timeout (a lost rank fails the run)


def launch_ranks(nranks: int, argv, poll_s: float = 0.2) -> int:
    """Parent of an N-rank run started without torchrun: it never touches the GPU (no
    torch import), starts one fresh child per rank (children are never exec'd from a GPU
    process) and forwards rank 0's stdout.  Every child is polled: the first one that exits
    non-zero has its siblings terminated (a rank waiting in a rendezvous for a dead peer
    would otherwise hang until the driver's time limit) and its exit status is returned."""
    import threading
    port = free_port()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out0 = []
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read().decode()), daemon=True)
    reader.start()
    failed = None
    while True:
        rcs = [p.poll() for p in procs]
        bad = [(r, rc) for r, rc in enumerate(rcs) if rc not in (None, 0)]
        if bad:
            failed = bad[0]
            break
        if all(rc == 0 for rc in rcs):
            break
        time.sleep(poll_s)
    if failed is not None:
        log(f'[bench] rank {failed[0]} exited with {failed[1]}: terminating the other ranks')
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    reader.join(timeout=10)
    for ln in ''.join(out0).splitlines():      # the JSON line to stdout, library chatter to stderr
        (sys.stdout if ln.startswith('{') else sys.stderr).write(ln + '\n')
    sys.stdout.flush()
    rcs = [p.returncode for p in procs]
    if failed is not None:
        log(f'[bench] rank exit codes: {rcs}')
        return failed[1] if failed[1] > 0 else 1
    return 0


# VALU peaks (MI355X_MICROARCH.md chip table: FP32 vector 157.3 TFLOPS spec; FP64 vector is
# half the FP32 rate on gfx950, 78.6 TFLOPS spec)
PEAK_VALU_TFLOPS = {'float32': 157.3, 'float64': 78.6}


def fft_flops_per_row(n: int, kname: str) -> float:
    """Nominal flops of one (signal, scale) row on the dominant kernel: 5 n log2 n for the
    inverse FFT (the radix-2 operation count), + 2 n for the real-W x complex-X product.
    The chirp-z form runs two M-point transforms per row (M = 2^ceil(log2(2n - 1)))."""
    import math
    if kname == 'nw_chirp_kernel':
        m = 1 << (2 * n - 1).bit_length()
        return 2 * 5.0 * m * math.log2(m) + 2.0 * n
    return 5.0 * n * math.log2(n) + 2.0 * n


def run_leg(args, torch, dist, nw, L, world, rank, dev, backend, cfg_name, dtype_override=None, fp64_leg=False,
            overrides=True):
    """One measured workload: warmup, barrier-bracketed timed steps, max over ranks.
    Returns (line fields, plan stats, extra) for rank 0's JSON line.  overrides=False: the
    config as CONFIGS names it (the extra legs of the default line ignore the diagnostic
    flags; --epochs still scales the multi-epoch legs down, for tests)."""
    kind, epochs, chans, n, freqs, out_kind, dtype, text = CONFIGS[cfg_name]
    if args.epochs and (overrides or epochs > 1):
        epochs = args.epochs
    if overrides and args.output:
        out_kind = args.output
    if overrides and args.samples:
        n = args.samples
    if overrides and args.wavelet and args.wavelet != kind:
        text = text.replace(kind.capitalize(), args.wavelet.capitalize(), 1)
        kind = args.wavelet
        if kind == 'shannon':
            text += (' [Shannon ignores the freq (wavelets.py:256-262): its one distinct row is '
                     'computed once per signal and copied to every scale]')
    want = dtype_override or (args.dtype if overrides else None)
    if want and want != dtype:
        dtype = want
        text = (text.replace('complex64 out', 'complex128 out') if fp64_leg else
                text + f' [compute dtype overridden: {dtype}, outputs in {dtype} / its complex type]')
    S = epochs * chans                       # signals on this rank
    F = len(freqs)
    F_all, by_scales = F, shards_scales(args.shard, S, world)
    f0, f1 = 0, F
    if by_scales:                            # this rank: a contiguous slice of the scales
        from ninwavelets_amd.dist import shard
        f0, f1 = shard(F, rank, world)
        freqs = freqs[f0:f1]
        F = f1 - f0
    slices = gather_slices(dist, (f0, f1)) if by_scales else None
    C = min((args.chunk if overrides else None) or DEFAULT_CHUNK.get(cfg_name, 256), S)
    f64 = dtype == 'float64'
    x = synth_device(torch, S, n, seed=1000 + (0 if by_scales else rank), device=dev,
                     dtype=torch.float64 if f64 else torch.float32)
    odt = {('cwt', False): torch.complex64, ('cwt', True): torch.complex128}.get(
        (out_kind, f64), torch.float64 if f64 else torch.float32)
    bufs = [torch.empty((C, F, n), dtype=odt, device=dev) for _ in range(1 if C >= S else 2)]
    # HIP events on the plan's own (dedicated) stream: each stage's stop event rides on its
    # kernel dispatch and its start is the previous stage's stop (NW_TIMING_CHAIN), so the
    # timed steps carry no event marker packets
    plan = nw.Plan(n, F, dtype, device=dev.index, max_batch=C,
                   engine=None if args.engine == 'auto' else args.engine, timing=True, timing_chain=True)
    grid = L.trans_grid(n / 1000., 1000., False)
    params = {'morse': [17.5, 3.0], 'morlet': [7.0, 0.0], 'shannon': []}[kind]
    plan.set_wavelet(kind, params, freqs, grid)
    esz = 8 if f64 else 4
    x_ptr, x_row = x.data_ptr(), n * esz

    def step():
        for i, s0 in enumerate(range(0, S, C)):
            c = min(C, S - s0)
            plan.execute_ptr(x_ptr + s0 * x_row, c, bufs[i % len(bufs)].data_ptr(), out_kind)

    def barrier():
        torch.cuda.synchronize()
        plan.sync()
        if dist.is_initialized():
            dist.barrier()

    log(f'[bench] rank {rank}/{world} {cfg_name}{" fp64 leg" if fp64_leg else ""}: S={S} n={n} F={F} '
        f'chunk={C} dtype={dtype} engine={plan.stats()["engine"]} device={dev}')
    for w in range(args.warmup):
        step()
        barrier()
        log(f'[bench] warmup {w + 1}/{args.warmup} done')
    plan.reset_stats()
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
    barrier()
    el = time.perf_counter() - t0
    el = max_over_ranks(torch, dist, el, dev if backend == 'nccl' else None)
    st = plan.stats()
    points = float(S) * F_all * n * args.steps * (1 if by_scales else world)
    res = {'value': points / el, 'ms_per_step': el / args.steps * 1e3, 'steps': args.steps, 'warmup': args.warmup,
           'dtype': 'f64' if f64 else 'f32',
           'workload': text, 'kind': kind, 'epochs': epochs * (1 if by_scales else world), 'chans': chans,
           'n': n, 'freqs': freqs, 'F': F, 'F_all': F_all, 'out_kind': out_kind, 'chunk': C,
           'by_scales': by_scales, 'dtype_name': dtype, 'scale_slices': slices,
           'scaling': 'strong' if by_scales else 'weak', 'parallelism': parallelism_of(by_scales, world)}
    extra = roofline_of(args, cfg_name, st, S, F, n, C, out_kind, dtype, esz, el, L) if rank == 0 else {}
    plan.close()
    del bufs, x
    torch.cuda.empty_cache()
    return res, st, extra


def shards_scales(shard: str, nsig: int, world: int) -> bool:
    """Whether the ranks split the scale list (strong scaling) rather than the signals.
    'auto': the scales exactly when a rank's share of the config is ONE signal (C5: 1 x 2^24,
    which cannot shard by signal -- SURVEY §8e splits its 512 scales over the GPUs)."""
    if world <= 1:
        return False
    return shard == 'scales' or (shard == 'auto' and nsig == 1)


def parallelism_of(by_scales: bool, world: int) -> str:
    return (f'scales{world} (each rank a contiguous slice of the scales of the same signal, '
            f'no collective)' if by_scales else f'dp{world} (signals sharded, no collective)')


def gather_slices(dist, sl):
    """Every rank's [f0, f1) scale slice, in rank order (rank 0 reports them)."""
    if not dist.is_initialized():
        return [list(sl)]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, list(sl))
    return out


def roofline_of(args, cfg_name, st, S, F, n, C, out_kind, dtype, esz, el, L):
    """The dominant kernel's HBM roofline (event-timed average launch, algorithmic bytes),
    its VALU roofline (nominal FFT flops) and the end-to-end figures."""
    f64 = dtype == 'float64'
    # dominant kernel: the fused kernel, or K1 (the spectrum multiply) on the rocFFT engine
    fused = st['engine'] == 'fused'
    two_pass = fused and st['launches_rows'] > 0     # n > 16384: nw_large.hip
    launches = st['launches_fused'] if fused else st['launches_multiply']
    ms = (st['ms_fused'] if fused else st['ms_multiply']) / max(1, launches)
    out_e = (2 if out_kind == 'cwt' else 1) * esz
    if not fused:
        out_e = 2 * esz                    # K1 always writes the complex product
    extra = {}
    uniq = st['unique_rows']
    rows_launch = float(S) * F * args.steps / max(1, launches)     # (signal, scale) rows per launch
    if uniq < F and st['launches_expand'] > 0:
        # repeated rows (Shannon): the engine computed `uniq` rows per signal and
        # k_expand_rows wrote every output row, reading each computed row once -- the
        # expand kernel moves the dominant bytes
        comp_ms = (st['ms_fused'] + st['ms_rows'] + st['ms_multiply'] + st['ms_inverse'] +
                   st['ms_epilogue']) / args.steps
        extra['computed_rows'] = {'unique_rows': uniq, 'engine_ms_per_step': round(comp_ms, 3),
                                  'engine_launches': launches}
        ex_l = st['launches_expand']
        ms = st['ms_expand'] / ex_l
        out_e = (2 if out_kind == 'cwt' else 1) * esz
        per_launch = float(S) * F * n * args.steps / ex_l * out_e * (1 + uniq / F)
        kname = 'k_expand_rows'
        rows_launch = 0.0
    elif two_pass:
        # column pass (the kernel that writes the output): reads B once (2e B/pt, complex
        # in the compute dtype) and writes each output point once; the row pass writes B
        # once and reads the transposed spectrum Xt once per launch (from L2 across the
        # scales of a tile)
        b_e = 2 * esz
        pts_launch = float(S) * F * n * args.steps / max(1, launches)
        per_launch = pts_launch * (b_e + out_e)
        rows_l = max(1, st['launches_rows'])
        rows_pts = float(S) * F * n * args.steps / rows_l
        rows_bytes = rows_pts * b_e + n * b_e
        rows_ms = st['ms_rows'] / rows_l
        kname = 'cols_kernel'
        extra['roofline_rows'] = {
            'kernel': 'rows_kernel', 'bound': 'hbm',
            'achieved': round(rows_bytes / (rows_ms * 1e-3) / 1e9, 1), 'peak': PEAK_HBM_GBPS,
            'unit': 'GB/s', 'frac': round(rows_bytes / (rows_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
            'avg_launch_ms': round(rows_ms, 4), 'algorithmic_bytes_per_launch': rows_bytes}
        rt, rsrc = pmc_traffic('rows_kernel', cfg_name, C, st['engine'], dtype, out_kind, n)
        extra['roofline_rows'].update(traffic=rt, traffic_source=(
            f'{rsrc}: rocprofv3 PMC passes, 2*FETCH_SIZE + WRITE_SIZE per launch, on engine sources '
            f'{source_hash()}' if rsrc else 'no PMC summary on the current engine sources'))
    else:
        per_launch = C * ((n // 2 + 1) * 2 * esz + F * n * out_e)   # X read once + out written once
        kname = L.KERNEL_NAMES[st['kernel']]          # the kernel rocprofv3 shows for this launch
    if two_pass or kname == 'k_expand_rows':
        # end to end against the path's minimum traffic (X read once, every output once)
        oe = (2 if out_kind == 'cwt' else 1) * esz
        min_bytes = float(S) * ((n // 2 + 1) * 2 * esz + F * n * oe)
        extra['end_to_end_min_traffic'] = {
            'bytes_per_step': min_bytes,
            'achieved': round(min_bytes / (el / args.steps) / 1e9, 1), 'unit': 'GB/s',
            'frac': round(min_bytes / (el / args.steps) / 1e9 / PEAK_HBM_GBPS, 4)}
    achieved = per_launch / (ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(kname, cfg_name, C, st['engine'], dtype, out_kind, n)
    roof = {'kernel': kname, 'bound': 'hbm',
            'achieved': round(achieved, 1), 'peak': PEAK_HBM_GBPS, 'unit': 'GB/s',
            'frac': round(achieved / PEAK_HBM_GBPS, 4),
            'traffic': traffic,
            'traffic_source': (f'{traffic_src}: rocprofv3 PMC passes of this command, 2*FETCH_SIZE + '
                               f'WRITE_SIZE per launch, on engine sources {source_hash()}'
                               if traffic_src else 'no PMC summary on the current engine sources'),
            'avg_launch_ms': round(ms, 4), 'algorithmic_bytes_per_launch': per_launch}
    if rows_launch > 0 and kname in ('nw_fused_kernel', 'nw_fused_pair_kernel', 'nw_chirp_kernel', 'cols_kernel'):
        # the other roof: nominal FFT flops of the rows this kernel finishes per launch (the
        # two-pass form's flops are split between its row and column passes: both counted
        # against the column pass's time would overstate it, so it is priced per step)
        fl = fft_flops_per_row(n, kname)
        if two_pass:
            t_s, flops, what = el / args.steps, float(S) * F * fl, 'per step (row + column passes)'
        else:
            t_s, flops, what = ms * 1e-3, rows_launch * fl, 'per launch'
        tf = flops / t_s / 1e12
        extra['valu_roofline'] = {
            'kernel': kname, 'bound': 'valu', 'achieved': round(tf, 2), 'peak': PEAK_VALU_TFLOPS[dtype],
            'unit': 'TFLOP/s', 'frac': round(tf / PEAK_VALU_TFLOPS[dtype], 4),
            'flops': flops, 'flops_basis': f'5 n log2 n + 2 n per (signal, scale) row {what} '
                                           f'(nominal radix-2 count; pruned rows do less)'}
    extra['stage_ms_per_step'] = {k: round(st[k] / args.steps, 3) for k in
                                  ('ms_forward', 'ms_multiply', 'ms_inverse', 'ms_epilogue', 'ms_fused', 'ms_rows',
                                   'ms_expand', 'ms_copy')}
    extra['roofline'] = roof
    return extra


# extra legs of the default line: key -> (config, compute dtype)
LEGS = {'fp64': ('c4', 'float64'), 'c2': ('c2', 'float32'), 'c3': ('c3', 'float32'), 'c5': ('c5', 'float32'),
        'c5_fp64': ('c5', 'float64')}
# at least this many timed steps / warmups for a leg whose step is short (C2: one 0.2-0.25 ms
# launch). The clock ramps for tens of ms after an idle gap: 3 steps (< 1 ms) varied +-10 %, and
# 40 steps after 5 warmups (10 ms) still ran 0.274 ms per step where 400 after 40 ran 0.224 on
# the same box (profiles/r06_c2_steps_ab.txt), so the leg times ~90 ms of steady state after
# ~10 ms of warmup; the headline line keeps exactly --steps / --warmup
LEG_MIN_STEPS = {'c2': (400, 40)}


def leg_fields(r, st, ex):
    """One extra leg's fields on the default line: its value, its workload, the dominant
    kernel's HBM roofline (+ the row pass's for the two-pass form), the VALU roofline and
    the end-to-end figure against the path's minimum traffic."""
    d = {'value': r['value'], 'unit': 'points/s', 'ms_per_step': r['ms_per_step'], 'steps': r['steps'],
         'warmup': r['warmup'], 'dtype': r['dtype'],
         'workload': r['workload'], 'output': r['out_kind'], 'chunk_signals': r['chunk'], 'engine': st['engine'],
         'scaling': r['scaling'], 'parallelism': r['parallelism'], 'roofline': ex['roofline']}
    if r['scale_slices'] is not None:
        d['scale_slices'] = r['scale_slices']
    for k in ('roofline_rows', 'valu_roofline', 'end_to_end_min_traffic', 'computed_rows', 'stage_ms_per_step'):
        if k in ex:
            d[k] = ex[k]
    return d


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='c4', choices=sorted(CONFIGS))
    ap.add_argument('--engine', default='auto', choices=['auto', 'rocfft', 'fused'])
    ap.add_argument('--chunk', type=int, default=None,
                    help='signals per device chunk (default per config: c4 512, c3 1024; measured '
                         'vs 256: +1 %% / +7 %% from fewer launch gaps and forward-FFT launches)')
    ap.add_argument('--epochs', type=int, default=None, help='override epochs per GPU')
    ap.add_argument('--output', default=None, choices=['cwt', 'abs', 'power'],
                    help='override the config\'s output kind (diagnostics)')
    ap.add_argument('--samples', type=int, default=None, help='override the signal length (diagnostics)')
    ap.add_argument('--dtype', default=None, choices=['float32', 'float64'],
                    help='override the compute dtype (diagnostics)')
    ap.add_argument('--wavelet', default=None, choices=['morse', 'morlet', 'shannon'],
                    help="override the config's wavelet (C5 is 'Shannon + Morse': --config c5 "
                         "--wavelet shannon is its Shannon line)")
    ap.add_argument('--shard', default='auto', choices=['auto', 'signals', 'scales'],
                    help='what the ranks split: signals (weak scaling, every rank its own epochs) '
                         'or the scale list of the same signals (strong scaling; the C5 split for '
                         'one long signal, SURVEY §8e); auto = scales for the one-signal config (C5), '
                         'signals otherwise')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-fp64', action='store_true',
                    help='skip the fp64 leg (the same workload at the reference\'s complex128 precision, '
                         'reported under the "fp64" key of the default C4 line)')
    ap.add_argument('--legs', default=','.join(LEGS),
                    help='extra legs of the default C4 line, comma-separated (default: all of '
                         f'{",".join(LEGS)}; "none" for none)')
    ap.add_argument('--backend', default=None, choices=['nccl', 'gloo'],
                    help='process-group backend for N > 1 ranks (default: nccl = RCCL over xGMI; '
                         'gloo with --dry-run)')
    ap.add_argument('--same-device', action='store_true',
                    help='rank r uses device LOCAL_RANK %% device_count (several ranks share a GPU: the '
                         'multi-rank path with real kernels on a 1-GPU box; use --backend gloo)')
    ap.add_argument('--dry-run', action='store_true',
                    help='no GPU and no kernels: exercise the launcher, the process group, the '
                         'barriers and the max-over-ranks timing on CPU (tests)')
    ap.add_argument('--fail-rank', type=int, default=None, help=argparse.SUPPRESS)   # tests: that rank exits 3
    args = ap.parse_args(argv)
    bad = [l for l in args.legs.split(',') if l and l != 'none' and l not in LEGS]
    if bad:
        raise SystemExit(f'bench.py: unknown --legs {bad} (choose from {sorted(LEGS)})')

    if 'WORLD_SIZE' in os.environ:           # torchrun or our own launcher: this process is a rank
        world = int(os.environ['WORLD_SIZE'])
        if args.gpus != 1 and args.gpus != world:
            raise SystemExit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}')
    elif args.gpus > 1:                      # launcher: N fresh ranks, no GPU call here
        return launch_ranks(args.gpus, sys.argv[1:] if argv is None else argv)
    else:
        world = 1
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    backend = args.backend or ('gloo' if args.dry_run else 'nccl')
    if args.fail_rank is not None and args.fail_rank == rank:
        log(f'[bench] rank {rank}: --fail-rank, exiting with 3 before the rendezvous')
        return 3

    import datetime
    import torch
    import torch.distributed as dist
    timeout = datetime.timedelta(seconds=PG_TIMEOUT_S)
    if args.dry_run:
        return dry_run(args, torch, dist, world, rank, backend, timeout)
    import ninwavelets_amd as nw
    from ninwavelets_amd import _lib as L

    if args.same_device:
        local = local % max(1, torch.cuda.device_count())
    # a process group whenever there are several ranks, or one rank launched by torchrun with
    # an explicit --backend (the driver's N-GPU path, RCCL included, at N = 1)
    if world > 1 or (args.backend is not None and 'MASTER_ADDR' in os.environ):
        torch.cuda.set_device(local)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local), timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)

    res, st, extra = run_leg(args, torch, dist, nw, L, world, rank, dev, backend, args.config)
    # The default (C4) line also carries BASELINE.json's other headline workloads, each measured
    # in this same run after the previous leg's buffers are freed, with its own roofline:
    #   fp64: C4 at the reference's precision (complex128 out, base.py:399-406);
    #   c2:   Morlet cwt 64 x 16384 x 128 (wavelets.py:132-136);
    #   c3:   Morse power 512 x 64 x 4096 x 256 (the fused |.|^2 path, base.py:409-425);
    #   c5:   Morse cwt 1 x 2^24 x 512, fp32 and fp64 (the long-signal regime, base.py:404-406);
    #         at N > 1 ranks its 512 scales are split over the ranks (strong scaling).
    default_line = (args.config == 'c4' and res['dtype'] == 'f32' and not args.dtype and not args.output and
                    not args.samples and not args.wavelet and not args.chunk)
    want = [l for l in args.legs.split(',') if l and l != 'none']
    legs = [] if not default_line else [l for l in LEGS if l in want and not (args.no_fp64 and l == 'fp64')]
    leg_out = {}
    for leg in legs:
        cfg_name, dt = LEGS[leg]
        largs = copy.copy(args)
        ms, mw = LEG_MIN_STEPS.get(leg, (0, 0))
        largs.steps, largs.warmup = max(args.steps, ms), max(args.warmup, mw)
        r_, st_, ex_ = run_leg(largs, torch, dist, nw, L, world, rank, dev, backend, cfg_name,
                               dtype_override=dt, fp64_leg=(dt == 'float64'), overrides=(leg == 'fp64'))
        if rank == 0:
            leg_out[leg] = leg_fields(r_, st_, ex_)
    fp64 = leg_out.pop('fp64', None)
    if 'c5' in leg_out or 'c5_fp64' in leg_out:
        leg_out['c5'] = {'fp32': leg_out.pop('c5', None), 'fp64': leg_out.pop('c5_fp64', None)}

    if rank == 0:
        cpu = cpu_pool = None
        if world == 1 and not args.no_cpu_baseline:
            log('[bench] cpu baseline ...')
            cpu = cpu_baseline(res['kind'], res['n'], res['freqs'], res['out_kind'])
            for k in ('sample_seconds', 'rows_done'):
                cpu.pop(k)
            if res['n'] <= (1 << 16):
                log('[bench] cpu baseline (process pool) ...')
                cpu_pool = cpu_baseline_pool(res['kind'], res['n'], res['freqs'], res['out_kind'])
        roof = extra.pop('roofline')
        stage_ms = extra.pop('stage_ms_per_step')
        line = {
            'metric': 'CWT throughput (epochs*chans*samples*freqs)/s',
            'value': res['value'], 'unit': 'points/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': res['ms_per_step'], 'higher_is_better': True,
            'scaling': res['scaling'], 'vs_baseline': None, 'dtype': res['dtype'],
            'data': 'synthetic',
            'config': {'workload': res['workload'], 'wavelet': res['kind'], 'epochs': res['epochs'],
                       'chans': res['chans'], 'samples': res['n'], 'freqs': res['F_all'], 'output': res['out_kind'],
                       'engine': st['engine'], 'chunk_signals': res['chunk'],
                       'parallelism': res['parallelism'],
                       **({'scale_slices': res['scale_slices']} if res['scale_slices'] else {}),
                       **({'backend': backend, 'same_device': True} if args.same_device else {}),
                       **({'process_group': dist.get_backend()} if dist.is_initialized() else {})},
            'roofline': roof, **extra, 'fp64': fp64, **leg_out, 'cpu_baseline': cpu, 'cpu_baseline_pool': cpu_pool,
            'stage_ms_per_step': stage_ms,
        }
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def max_over_ranks(torch, dist, el, device):
    """The step time the job took: the MAX of every rank's elapsed time."""
    if not dist.is_initialized():
        return el
    t = torch.tensor([el], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def dry_run(args, torch, dist, world, rank, backend, timeout=None):
    """The multi-rank flow without a GPU: process group, warmup, barrier-bracketed timed
    steps (a fixed CPU stand-in per step), MAX over ranks, rank 0's line, and the same
    signal / scale partition run_leg takes (C5's scale slices gathered from every rank).
    Its value is not a measurement; it proves the launcher and the rank plumbing (tests)."""
    if world > 1:
        dist.init_process_group(backend, **({'timeout': timeout} if timeout else {}))
    kind, epochs, chans, n, freqs, out_kind, dtype, text = CONFIGS[args.config]
    by_scales = shards_scales(args.shard, epochs * chans, world)
    slices = None
    if by_scales:
        from ninwavelets_amd.dist import shard
        slices = gather_slices(dist, shard(len(freqs), rank, world))

    def step():
        time.sleep(0.01 * (1 + rank))        # ranks of unequal speed: the max must win

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
        barrier()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    el = max_over_ranks(torch, dist, time.perf_counter() - t0, None)
    if rank == 0:
        print(json.dumps({
            'metric': 'CWT throughput (epochs*chans*samples*freqs)/s', 'value': None, 'unit': 'points/s',
            'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': el / max(1, args.steps) * 1e3, 'higher_is_better': True,
            'scaling': 'strong' if by_scales else 'weak',
            'vs_baseline': None, 'dtype': 'f64' if dtype == 'float64' else 'f32',
            'data': 'dry run: no GPU, no kernels', 'backend': backend,
            'config': {'workload': text, 'parallelism': f'scales{world}' if by_scales else f'dp{world}',
                       **({'scale_slices': slices} if slices else {})}}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())

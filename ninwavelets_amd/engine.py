"""Thin Python owner of one ``nw_plan`` (one device, one signal length n).

This is the batched entry point that replaces the serial per-epoch loop of
the reference (mneutils.py:39): one call transforms S = epochs x channels
signals.  Inputs/outputs may be numpy arrays (host, synchronous) or device
buffers (torch tensors on the plan's device or raw pointers; asynchronous on
the plan stream).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import numpy as np

from . import _lib as L

OUT_KINDS = {'cwt': L.NW_OUT_CWT, 'abs': L.NW_OUT_ABS, 'power': L.NW_OUT_POWER,
             # reductions over the signals -> (F, n) (EpochsWavelet, mneutils.py:42-71)
             'power_mean': L.NW_OUT_POWER_MEAN, 'itc': L.NW_OUT_ITC,
             'power_sum': L.NW_OUT_POWER_SUM, 'phase_sum': L.NW_OUT_PHASE_SUM}
REDUCTIONS = ('power_mean', 'itc', 'power_sum', 'phase_sum')
KINDS = {'morse': L.NW_MORSE, 'morlet': L.NW_MORLET, 'shannon': L.NW_SHANNON, 'table': L.NW_TABLE,
         # WaveletMode.Normal tables built on the device (base.py:249-256)
         'mexican_hat': L.NW_MEXICAN_HAT, 'haar': L.NW_HAAR}
TABLE_KINDS = ('table', 'mexican_hat', 'haar')


def np_dtype(dtype) -> np.dtype:
    dt = np.dtype(dtype)
    if dt not in (np.float32, np.float64):
        raise ValueError(f'compute dtype must be float32 or float64, got {dt}')
    return dt


def out_dtype(dtype, out_kind: str) -> np.dtype:
    dt = np_dtype(dtype)
    if out_kind == 'power_sum':                 # fp64 partial sums whatever the compute dtype
        return np.dtype(np.float64)
    if out_kind == 'phase_sum':
        return np.dtype(np.complex128)
    if out_kind == 'cwt':
        return np.dtype(np.complex64 if dt == np.float32 else np.complex128)
    return dt


class HostPool:
    """Page-locked result arrays, recycled (nw_host_alloc).

    The reference returns a new array per call (base.py:378-407).  A fresh pageable numpy
    array of a large result is faulted in page by page while the copy-out writes it, which
    bounded the host path at a third of the PCIe rate; a page-locked destination is written
    by DMA directly.  A pooled result is an ordinary numpy array owning its buffer: when the
    caller drops it (and every view of it), the buffer returns to the pool for the next
    result of the same size.  At most ``cap`` bytes are page-locked at a time (results the
    caller keeps count too); past that, results are fresh pageable arrays advised onto huge
    pages (nw_host_advise).  ``min_bytes``: smaller results are not worth a page-locked buffer.

    Released buffers are handed back by a weakref finalizer, which may run inside a garbage
    collection triggered anywhere -- including inside this pool's own locked region.  The
    finalizer therefore never takes the lock or calls into the library: it only appends
    (ptr, nbytes) to a deque (thread-safe append), and the pool drains that queue at the top
    of its next take, outside any finalizer."""

    def __init__(self, cap: int, min_bytes: int = 32 << 20, keep_free: int = 2, alloc=None, free=None,
                 advise=None):
        import collections
        import threading
        self.cap, self.min_bytes, self.keep_free = int(cap), int(min_bytes), int(keep_free)
        self._alloc, self._free_fn = alloc or self._nw_alloc, free or self._nw_free
        self._advise = advise if advise is not None else self._nw_advise
        self._lock = threading.Lock()
        self._free: dict = {}            # nbytes -> [ptr]
        self._returned = collections.deque()   # (ptr, nbytes) released by finalizers, not yet filed
        self.held = 0                    # page-locked bytes, in use or free

    @staticmethod
    def _nw_alloc(nbytes):
        p = ctypes.c_void_p()
        L.check(L.lib().nw_host_alloc(int(nbytes), ctypes.byref(p)))
        return p.value

    @staticmethod
    def _nw_free(ptr):
        L.check(L.lib().nw_host_free(ctypes.c_void_p(ptr)))

    @staticmethod
    def _nw_advise(arr):
        lib = L.lib()
        # an older diagnostic library (NINWAVE_LIB, A/B runs) may lack the symbol: no advice then
        if hasattr(lib, 'nw_host_advise'):
            L.check(lib.nw_host_advise(ctypes.c_void_p(arr.ctypes.data), int(arr.nbytes), None))

    def free_bytes(self) -> int:
        self._drain()
        with self._lock:
            return sum(n * len(v) for n, v in self._free.items())

    def trim(self) -> int:
        """Free every idle pooled buffer now and return the bytes released.  Buffers come back
        lazily: a dropped result is filed by the next empty() / free_bytes() / trim(), so up to
        the cap stays page-locked (and counted in ``held``) after the last result is gone until
        one of them runs."""
        self._drain()
        drop = []
        with self._lock:
            for n, lst in self._free.items():
                while lst:
                    drop.append((lst.pop(), n))
                    self.held -= n
        for ptr, _ in drop:
            self._free_fn(ptr)
        return sum(n for _, n in drop)

    def _drain(self):
        """File the buffers finalizers returned: keep up to keep_free per size, free the rest
        (the library calls happen outside the lock)."""
        drop = []
        with self._lock:
            while self._returned:
                ptr, nbytes = self._returned.popleft()
                lst = self._free.get(nbytes)
                if lst is None:
                    lst = self._free[nbytes] = []
                if len(lst) < self.keep_free:
                    lst.append(ptr)
                else:
                    self.held -= nbytes
                    drop.append(ptr)
        for ptr in drop:
            self._free_fn(ptr)

    def _take(self, nbytes):
        self._drain()
        drop = []
        with self._lock:
            lst = self._free.get(nbytes)
            if lst:
                return lst.pop()
            # make room: drop free buffers of other sizes first
            for n in list(self._free):
                while self._free[n] and self.held + nbytes > self.cap:
                    drop.append(self._free[n].pop())
                    self.held -= n
            ok = self.held + nbytes <= self.cap
            if ok:
                self.held += nbytes
        for ptr in drop:
            self._free_fn(ptr)
        if not ok:
            return None
        try:
            return self._alloc(nbytes)
        except Exception:
            with self._lock:
                self.held -= nbytes
            return None

    def _release(self, ptr, nbytes):
        # finalizer context: no lock, no library call (see the class docstring)
        self._returned.append((ptr, nbytes))

    def empty(self, shape, dtype) -> np.ndarray:
        """np.empty(shape, dtype), page-locked when large enough and within the cap."""
        import weakref
        dt = np.dtype(dtype)
        nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
        if nbytes < self.min_bytes:
            return np.empty(shape, dtype=dt)
        ptr = self._take(nbytes)
        if ptr is None:
            arr = np.empty(shape, dtype=dt)
            self._advise(arr)                # our own fresh array: huge pages for the copy-out
            return arr
        owner = _PooledBuffer(ptr, tuple(int(s) for s in shape), dt)
        f = weakref.finalize(owner, self._release, ptr, nbytes)
        f.atexit = False                 # the process is ending: the OS reclaims it
        return np.asarray(owner)


class _PooledBuffer:
    """Owner of one pooled buffer: exposes it to numpy (__array_interface__); every array or
    view made from it keeps it alive."""

    def __init__(self, ptr, shape, dtype):
        self.__array_interface__ = {'data': (ptr, False), 'shape': shape, 'typestr': dtype.str, 'version': 3}


def host_pinned_array(a) -> bool:
    """Whether numpy array ``a`` (or the array it views) is a pooled page-locked result."""
    b = a
    while b is not None:
        if isinstance(b, _PooledBuffer):
            return True
        b = getattr(b, 'base', None)
    return False


def default_pool_cap(total_ram: int | None = None, local_ranks: int | None = None) -> int:
    """Page-locked bytes one process may pool by default: 8 GiB, at most 1/8 of the host's RAM,
    shared by the ranks of one node (LOCAL_WORLD_SIZE processes each hold their own pool, so
    eight ranks of a node pin no more than one process would).  NINWAVE_HOST_POOL_BYTES
    overrides it."""
    if total_ram is None:
        try:
            total_ram = os.sysconf('SC_PAGE_SIZE') * os.sysconf('SC_PHYS_PAGES')
        except (ValueError, OSError, AttributeError):
            total_ram = 64 << 30
    if local_ranks is None:
        local_ranks = local_rank_count()
    return int(min(8 << 30, total_ram // 8) // max(1, local_ranks))


def local_rank_count(env=None) -> int:
    """Processes of this job on this node: torchrun's LOCAL_WORLD_SIZE, else the launcher's
    node-local count (Slurm, Open MPI, MPICH/Hydra), else 1.  Never the global WORLD_SIZE: on a
    multi-node launch that would shrink every rank's pool by the total rank count."""
    env = os.environ if env is None else env
    for k in ('LOCAL_WORLD_SIZE', 'SLURM_NTASKS_PER_NODE', 'OMPI_COMM_WORLD_LOCAL_SIZE', 'MPI_LOCALNRANKS'):
        v = env.get(k)
        if v:
            try:
                return max(1, int(str(v).split('(')[0].split(',')[0]))
            except ValueError:
                continue
    return 1


HOST_POOL = HostPool(int(os.environ.get('NINWAVE_HOST_POOL_BYTES') or default_pool_cap()))


def _is_device_tensor(a) -> bool:
    return hasattr(a, 'data_ptr') and getattr(a, 'is_cuda', False)


class Plan:
    """One nw_plan: signals of length ``n``, ``nfreq`` scales, compute ``dtype``."""

    def __init__(self, n: int, nfreq: int, dtype='float32', device: int = 0, max_batch: int = 1,
                 interpolate: bool = False, engine: str | None = None, timing: bool = False,
                 dedup: bool = True, timing_chain: bool = False):
        self.n, self.nfreq, self.device, self.max_batch = int(n), int(nfreq), int(device), int(max_batch)
        self.dtype = np_dtype(dtype)
        self.interpolate = bool(interpolate)
        flags = L.NW_INTERPOLATE if interpolate else 0
        if engine == 'rocfft':
            flags |= L.NW_ENGINE_ROCFFT
        elif engine == 'fused':
            flags |= L.NW_ENGINE_FUSED
        elif engine not in (None, 'auto'):
            raise ValueError(f'engine must be rocfft, fused or auto, got {engine!r}')
        if timing:
            flags |= L.NW_TIMING
            if timing_chain:     # a dedicated stream: stage events chained across executes
                flags |= L.NW_TIMING_CHAIN
        if not dedup:            # compute every scale row even when wavelet rows repeat
            flags |= L.NW_NO_DEDUP
        self._h = ctypes.c_void_p()
        L.check(L.lib().nw_plan_create(ctypes.byref(self._h), self.device, self.n, self.max_batch,
                                       self.nfreq, L.NW_F32 if self.dtype == np.float32 else L.NW_F64,
                                       flags))
        self.wavelet_token = None

    # -- wavelet -----------------------------------------------------------------
    def set_wavelet(self, kind: str, params, freqs, grid: L.nw_grid, table=None, token=None,
                    row_len=None):
        freqs = np.ascontiguousarray(freqs, dtype=np.float64)
        if freqs.shape != (self.nfreq,):
            raise ValueError(f'expected {self.nfreq} freqs, got {freqs.shape}')
        p = np.ascontiguousarray(params if params is not None else [], dtype=np.float64)
        tab_ptr = rl_ptr = None
        if KINDS[kind] == L.NW_TABLE:
            table = np.ascontiguousarray(table, dtype=np.complex128)
            if table.shape != (self.nfreq, grid.len_full):
                raise ValueError(f'table must be ({self.nfreq}, {grid.len_full}), got {table.shape}')
            tab_ptr = table.ctypes.data_as(ctypes.c_void_p)
            if row_len is not None:
                row_len = np.ascontiguousarray(row_len, dtype=np.int64)
                rl_ptr = row_len.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
        L.check(L.lib().nw_plan_set_wavelet(
            self._h, KINDS[kind], p.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), int(p.size),
            freqs.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(grid), tab_ptr, rl_ptr))
        self.kind, self.grid = kind, grid
        if kind in TABLE_KINDS:                      # the width the device settled on
            lf = ctypes.c_int64()
            lens = np.empty(self.nfreq, dtype=np.int64)
            L.check(L.lib().nw_plan_wavelet_shape(self._h, ctypes.byref(lf),
                                                  lens.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
            self.grid = L.nw_grid(1.0, lf.value, lf.value)
            self.row_len = lens
        self.wavelet_token = token

    def rows(self) -> np.ndarray:
        """Device-evaluated cached wavelet rows (nfreq, len_full)."""
        dt = self.dtype if self.kind not in TABLE_KINDS else out_dtype(self.dtype, 'cwt')
        out = np.empty((self.nfreq, self.grid.len_full), dtype=dt)
        L.check(L.lib().nw_plan_wavelet_rows(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def row_support(self, scan: bool = False) -> np.ndarray:
        """Two-pass engine diagnostic: each row's last bin above the tail threshold (the row
        pass's pruning bound, nw_plan_row_support); scan=True by scanning every bin."""
        out = np.empty(self.nfreq, dtype=np.int32)
        L.check(L.lib().nw_plan_row_support(self._h, 1 if scan else 0, out.ctypes.data_as(ctypes.c_void_p)))
        return out

    # -- execute -----------------------------------------------------------------
    def execute(self, x, out=None, out_kind: str = 'cwt'):
        """x: (S, n) numpy array (host) -> returns (S, nfreq, n); or device tensors."""
        kind = OUT_KINDS[out_kind]
        reduce = out_kind in REDUCTIONS
        if _is_device_tensor(x):
            if out is None:
                raise ValueError('device execute needs an output tensor')
            nsig = self._check_device_input(x)
            self._check_device_buffers(x, out, nsig, out_kind)
            with self._ordered_with_torch(x.device):
                L.check(L.lib().nw_execute(self._h, ctypes.c_void_p(x.data_ptr()), nsig,
                                           ctypes.c_void_p(out.data_ptr()), kind, L.NW_MEM_DEVICE))
            return out
        x = np.ascontiguousarray(x, dtype=self.dtype)
        if x.shape[-1] != self.n:
            raise ValueError(f'signal length {x.shape[-1]} != plan n {self.n}')
        lead = x.shape[:-1]
        nsig = int(np.prod(lead)) if lead else 1
        odt = out_dtype(self.dtype, out_kind)
        shape = (self.nfreq, self.n) if reduce else lead + (self.nfreq, self.n)
        if out is None:
            out = HOST_POOL.empty(shape, odt)
        elif out.dtype != odt or not out.flags.c_contiguous or out.size != int(np.prod(shape)):
            raise ValueError('out must be a C-contiguous array of the right dtype and size')
        L.check(L.lib().nw_execute(self._h, x.ctypes.data_as(ctypes.c_void_p), nsig,
                                   out.ctypes.data_as(ctypes.c_void_p), kind, L.NW_MEM_HOST))
        return out

    def stream_ptr(self) -> int:
        """The hipStream_t the plan launches on."""
        h = ctypes.c_void_p()
        L.check(L.lib().nw_plan_get_stream(self._h, ctypes.byref(h)))
        return h.value or 0

    @contextlib.contextmanager
    def _ordered_with_torch(self, device):
        """Order a device-tensor execute with torch's current stream on both sides: the
        plan stream waits for the work that produced the input, and torch's stream waits
        for the plan's kernels before anything later reads the output or the caching
        allocator reuses either buffer."""
        import torch
        cur = torch.cuda.current_stream(device)
        plan_stream = torch.cuda.ExternalStream(self.stream_ptr(), device=device)
        plan_stream.wait_stream(cur)
        try:
            yield
        finally:
            cur.wait_stream(plan_stream)

    def execute_ptr(self, x_ptr: int, nsig: int, out_ptr: int, out_kind: str = 'cwt'):
        """Raw device pointers on the plan's device (asynchronous on the plan stream; the
        caller orders it against its own streams, e.g. with plan.sync())."""
        L.check(L.lib().nw_execute(self._h, ctypes.c_void_p(x_ptr), int(nsig), ctypes.c_void_p(out_ptr),
                                   OUT_KINDS[out_kind], L.NW_MEM_DEVICE))

    def _check_device_input(self, x) -> int:
        """The input half of _check_device_buffers: a contiguous (nsig, n) tensor of the
        compute dtype on the plan's device, whole rows only.  Returns nsig."""
        import torch
        want_x = torch.float32 if self.dtype == np.float32 else torch.float64
        if not _is_device_tensor(x):
            raise ValueError(f'device input must be a torch tensor on device {self.device}')
        if x.dtype != want_x:
            raise ValueError(f'device input must be {want_x}, got {x.dtype}')
        if not x.is_contiguous():
            raise ValueError('device input must be contiguous')
        if x.numel() % self.n:
            raise ValueError(f'device input of {x.numel()} values is not a whole number of '
                             f'{self.n}-sample signals')
        if x.device.index != self.device:
            raise ValueError(f'device input must live on device {self.device}, got {x.device}')
        return x.numel() // self.n

    def _check_device_buffers(self, x, out, nsig, out_kind):
        import torch
        if self._check_device_input(x) != nsig:
            raise ValueError('device buffer sizes do not match (S, n) -> (S, nfreq, n) / (nfreq, n)')
        want_o = {('cwt', np.float32): torch.complex64, ('cwt', np.float64): torch.complex128}.get(
            (out_kind, self.dtype.type), x.dtype)
        if out_kind == 'power_sum':
            want_o = torch.float64
        elif out_kind == 'phase_sum':
            want_o = torch.complex128
        if out.dtype != want_o:
            raise ValueError(f'device buffers must be {x.dtype} in / {want_o} out')
        if not out.is_contiguous():
            raise ValueError('device buffers must be contiguous')
        rows = 1 if out_kind in REDUCTIONS else nsig
        if out.numel() != rows * self.nfreq * self.n:
            raise ValueError('device buffer sizes do not match (S, n) -> (S, nfreq, n) / (nfreq, n)')
        if out.device.index != self.device:
            raise ValueError(f'device buffers must live on device {self.device}')

    # -- misc --------------------------------------------------------------------
    def set_stream(self, stream_ptr: int | None):
        L.check(L.lib().nw_plan_set_stream(self._h, ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def sync(self):
        L.check(L.lib().nw_plan_sync(self._h))

    def stats(self) -> dict:
        s = L.nw_stats()
        L.check(L.lib().nw_plan_stats(self._h, ctypes.byref(s)))
        d = s.as_dict()
        d['engine'] = 'fused' if d['engine'] == L.NW_ENGINE_FUSED else 'rocfft'
        return d

    def reset_stats(self):
        L.check(L.lib().nw_plan_reset_stats(self._h))

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, '_h', None) and self._h.value:
            L.lib().nw_plan_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def execute_multi(plans, x: np.ndarray, out_kind: str = 'cwt', shard: str = 'signals') -> np.ndarray:
    """Several single-device plans, one host thread each.
    shard='signals': identical plans, contiguous blocks of the host signals per device
    (nw_execute_multi).  shard='scales': plan i holds the i-th contiguous slice of the
    scale list and transforms every signal for it (nw_execute_multi_scales) -- the split
    for one long signal (C5)."""
    if shard not in ('signals', 'scales'):
        raise ValueError(f"shard must be 'signals' or 'scales', got {shard!r}")
    p0 = plans[0]
    x = np.ascontiguousarray(x, dtype=p0.dtype)
    lead = x.shape[:-1]
    nsig = int(np.prod(lead)) if lead else 1
    nf = sum(p.nfreq for p in plans) if shard == 'scales' else p0.nfreq
    shape = (nf, p0.n) if out_kind in REDUCTIONS else lead + (nf, p0.n)
    out = HOST_POOL.empty(shape, out_dtype(p0.dtype, out_kind))
    arr = (ctypes.c_void_p * len(plans))(*[p.handle.value for p in plans])
    fn = L.lib().nw_execute_multi_scales if shard == 'scales' else L.lib().nw_execute_multi
    L.check(fn(arr, len(plans), x.ctypes.data_as(ctypes.c_void_p), nsig,
               out.ctypes.data_as(ctypes.c_void_p), OUT_KINDS[out_kind]))
    return out


def execute_multi_device(plans, xs, outs, out_kind: str = 'cwt'):
    """Device-resident sharding (nw_execute_multi_device): plan i transforms
    the torch tensor xs[i] (on plan i's device, (nsig_i, n)) into outs[i]; for the
    reductions outs[0] receives the (F, n) result over every signal of every device.
    One host thread per device; returns when every device is done."""
    if not (len(plans) == len(xs) == len(outs)):
        raise ValueError('one input and one output tensor per plan')
    red = out_kind in REDUCTIONS
    nsig = []
    for i, (p, x, o) in enumerate(zip(plans, xs, outs)):
        # every input is validated (dtype, contiguity, whole rows, device): its raw pointer
        # goes to nw_execute as device memory of plan i; for the reductions only outs[0] is
        # written, so the other outputs may be None
        ns = p._check_device_input(x)
        if not red or i == 0:
            p._check_device_buffers(x, o, ns, out_kind)
        nsig.append(ns)
    import torch
    for p, x in zip(plans, xs):                 # inputs produced on torch's streams are complete
        torch.cuda.current_stream(x.device).synchronize()
    P = ctypes.c_void_p
    arr = (P * len(plans))(*[p.handle.value for p in plans])
    xa = (P * len(plans))(*[x.data_ptr() for x in xs])
    oa = (P * len(plans))(*[(o.data_ptr() if o is not None else 0) for o in outs])
    na = (ctypes.c_int64 * len(plans))(*nsig)
    L.check(L.lib().nw_execute_multi_device(arr, len(plans), xa, na, oa, OUT_KINDS[out_kind]))
    return outs[0] if red else outs


def make_wavelets(kind: str, params, freqs, sfreq: float, real_wave_length: float, device: int = 0) -> list:
    """Time-domain wavelets of a stock kind on the device (nw_make_wavelets,
    base.py:346-376): a list of complex128 rows of their true (ragged) lengths."""
    fr = np.ascontiguousarray(list(freqs), dtype=np.float64)
    p = np.ascontiguousarray(params if params is not None else [], dtype=np.float64)
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int64)
    lens = np.zeros(fr.size, dtype=np.int64)
    mx = ctypes.c_int64()
    args = (device, KINDS[kind], p.ctypes.data_as(dp), int(p.size), fr.ctypes.data_as(dp), int(fr.size),
            float(sfreq), float(real_wave_length))
    L.check(L.lib().nw_make_wavelets(*args, None, ctypes.byref(mx), lens.ctypes.data_as(ip)))
    out = np.zeros((fr.size, mx.value), dtype=np.complex128)
    L.check(L.lib().nw_make_wavelets(*args, out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(mx),
                                     lens.ctypes.data_as(ip)))
    return [out[i, :lens[i]].copy() for i in range(fr.size)]

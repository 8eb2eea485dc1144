"""ctypes binding of libninwave.so (the C ABI declared in include/ninwave.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C ninwavelets_amd/csrc``).  There is no fallback: if the library is
missing or a GPU is absent, calls raise instead of computing on the CPU.

Mixing with PyTorch in one process: torch wheels bundle their own HIP runtime.
Import torch BEFORE this package, so libninwave.so binds to torch's already
loaded libamdhip64/librocfft (same sonames) and the process keeps one runtime.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('NINWAVE_LIB', os.path.join(_HERE, 'libninwave.so'))

# status codes / constants (ninwave.h)
NW_OK = 0
NW_E_INVALID = -1
NW_E_HIP = -2
NW_E_ROCFFT = -3
NW_E_NOMEM = -4
NW_E_STATE = -5
NW_E_NODEVICE = -6
NW_E_BOUNDS = -7

NW_F32, NW_F64 = 0, 1
NW_MORSE, NW_MORLET, NW_SHANNON, NW_TABLE = 1, 2, 3, 4
NW_MEXICAN_HAT, NW_HAAR = 5, 6
NW_INTERPOLATE = 0x1
NW_ENGINE_ROCFFT = 0x10
NW_ENGINE_FUSED = 0x20
NW_TIMING = 0x100
NW_TIMING_CHAIN = 0x800
NW_NO_DEDUP = 0x200
NW_NO_CHIRP = 0x400
NW_OUT_CWT, NW_OUT_ABS, NW_OUT_POWER = 0, 1, 2
NW_OUT_POWER_MEAN, NW_OUT_ITC, NW_OUT_POWER_SUM, NW_OUT_PHASE_SUM = 3, 4, 5, 6
NW_MEM_HOST, NW_MEM_DEVICE = 0, 1
# nw_stats.kernel -> the kernel name rocprofv3 shows
KERNEL_NAMES = {0: None, 1: 'nw_fused_kernel', 2: 'nw_fused_pair_kernel', 3: 'nw_chirp_kernel',
                4: 'cols_kernel', 5: 'k1_multiply'}
NW_BL = {'mean': 0, 'ratio': 1, 'percent': 2, 'log': 3, 'zscore': 4, 'zlog': 5}


class nw_grid(ctypes.Structure):
    _fields_ = [('delta', ctypes.c_double), ('len_full', ctypes.c_int64), ('len_valid', ctypes.c_int64)]


class nw_stats(ctypes.Structure):
    _fields_ = [('executes', ctypes.c_int64), ('chunks', ctypes.c_int64),
                ('ms_forward', ctypes.c_double), ('ms_multiply', ctypes.c_double),
                ('ms_inverse', ctypes.c_double), ('ms_epilogue', ctypes.c_double),
                ('ms_fused', ctypes.c_double), ('ms_copy', ctypes.c_double),
                ('launches_multiply', ctypes.c_int64), ('launches_fused', ctypes.c_int64),
                ('engine', ctypes.c_int64), ('ms_rows', ctypes.c_double),
                ('launches_rows', ctypes.c_int64), ('ms_expand', ctypes.c_double),
                ('launches_expand', ctypes.c_int64), ('unique_rows', ctypes.c_int64),
                ('kernel', ctypes.c_int64), ('device_bytes', ctypes.c_int64)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# every symbol of include/ninwave.h: (name, restype, argtypes)
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
SIGNATURES = [
    ('nw_last_error', ctypes.c_char_p, []),
    ('nw_version', ctypes.c_char_p, []),
    ('nw_set_log_level', ctypes.c_int, [ctypes.c_int]),
    ('nw_debug_bounds', ctypes.c_int, []),
    ('nw_debug_selftest', ctypes.c_int, [ctypes.c_int]),
    ('nw_device_count', ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ('nw_trans_grid', ctypes.c_int, [ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.POINTER(nw_grid)]),
    ('nw_fused_supported', ctypes.c_int, [_I64, ctypes.c_int]),
    ('nw_plan_create', ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, _I64, _I64, ctypes.c_int32,
                                      ctypes.c_int, ctypes.c_uint32]),
    ('nw_plan_set_wavelet', ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(nw_grid), _P,
                                           ctypes.POINTER(ctypes.c_int64)]),
    ('nw_plan_wavelet_shape', ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    ('nw_plan_wavelet_rows', ctypes.c_int, [_P, _P]),
    ('nw_plan_row_support', ctypes.c_int, [_P, ctypes.c_int, _P]),
    ('nw_execute', ctypes.c_int, [_P, _P, _I64, _P, ctypes.c_int, ctypes.c_int]),
    ('nw_execute_multi', ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, _P, _I64, _P, ctypes.c_int]),
    ('nw_execute_multi_scales', ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, _P, _I64, _P, ctypes.c_int]),
    ('nw_execute_multi_device', ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.POINTER(_P),
                                               ctypes.POINTER(_I64), ctypes.POINTER(_P), ctypes.c_int]),
    ('nw_baseline', ctypes.c_int, [ctypes.c_int, ctypes.c_int, _P, _I64, _I64, _I64, _I64, ctypes.c_int, _P,
                                   ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    ('nw_make_wavelets', ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_double,
                                        ctypes.c_double, _P, ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_int64)]),
    ('nw_host_alloc', ctypes.c_int, [_I64, ctypes.POINTER(_P)]),
    ('nw_host_free', ctypes.c_int, [_P]),
    ('nw_host_advise', ctypes.c_int, [_P, _I64, ctypes.POINTER(_I64)]),
    ('nw_plan_set_stream', ctypes.c_int, [_P, _P]),
    ('nw_plan_get_stream', ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    ('nw_plan_sync', ctypes.c_int, [_P]),
    ('nw_plan_stats', ctypes.c_int, [_P, ctypes.POINTER(nw_stats)]),
    ('nw_plan_reset_stats', ctypes.c_int, [_P]),
    ('nw_plan_destroy', ctypes.c_int, [_P]),
]


class NinwaveError(RuntimeError):
    """A non-zero status from libninwave.so (message from nw_last_error())."""

    def __init__(self, code, msg):
        super().__init__(f'libninwave status {code}: {msg}')
        self.code = code


_lib = None


def lib():
    """Load libninwave.so once; raise loudly if it is missing (no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f'{LIB_PATH} not found: build it with '
                              '`python -c "import __graft_entry__ as g; g.build()"` '
                              'or `make -C ninwavelets_amd/csrc`')
        handle = ctypes.CDLL(LIB_PATH)
        # the product library must export every entry point; a diagnostic build of an older
        # tree (NINWAVE_LIB, tools/ab.sh A/B against a past round) may lack the newer ones,
        # which then stay unbound (calling one raises AttributeError)
        product = os.path.abspath(LIB_PATH) in (os.path.join(_HERE, 'libninwave.so'),
                                                os.path.join(_HERE, 'libninwave_debug.so'))
        for name, res, args in SIGNATURES:
            fn = getattr(handle, name, None)
            if fn is None:
                if product:
                    raise ImportError(f'{LIB_PATH} does not export {name}: rebuild it')
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc):
    if rc != NW_OK:
        msg = lib().nw_last_error().decode(errors='replace')
        if rc == NW_E_INVALID:
            raise ValueError(msg)
        raise NinwaveError(rc, msg)


def set_log_level(level: int) -> int:
    """NW_LOG diagnostics on stderr (0 silent, 1 decisions and errors, 2 every launch); returns
    the previous level."""
    return int(lib().nw_set_log_level(int(level)))


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().nw_device_count(ctypes.byref(n))
    return n.value if rc == NW_OK else 0


def trans_grid(real_length: float, sfreq: float, interpolate: bool) -> nw_grid:
    g = nw_grid()
    check(lib().nw_trans_grid(float(real_length), float(sfreq), int(bool(interpolate)), ctypes.byref(g)))
    return g


def fused_supported(n: int, dtype: int) -> bool:
    return bool(lib().nw_fused_supported(int(n), int(dtype)))

import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# torch wheels bundle their own HIP runtime (libamdhip64.so, librocfft.so).  When
# torch is loaded first, libninwave.so binds to that same runtime (matching
# sonames); loaded the other way round the process would hold two HIP runtimes.
# So the suite imports torch first, exactly as bench.py does.
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the product
    torch = None
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs on the GPU box via gpurun)')


def golden_names(prefix=''):
    return sorted(f[:-4] for f in os.listdir(GOLDEN)
                  if f.endswith('.npz') and f.startswith(prefix))


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d['meta'] = json.loads(str(d['meta']))
    return d


def long_signal(n: int, seed: int, sfreq: float = 1000.) -> np.ndarray:
    """Input of the benchmark-length goldens (tests/golden/make_golden_long.py), rebuilt from
    its seed: two sinusoids + 0.1 N(0, 1) noise from np.random.default_rng(seed)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sfreq
    f1, f2 = rng.uniform(3, 120, 2)
    return (np.sin(2 * np.pi * f1 * t) + 0.5 * np.sin(2 * np.pi * f2 * t + 1.0)
            + 0.1 * rng.standard_normal(n))


def x_digest(x: np.ndarray) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(x, dtype=np.float64).tobytes()).hexdigest()


@pytest.fixture(scope='session')
def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False

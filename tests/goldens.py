"""Golden-fixture helpers shared by the tests and by tests/torchfree_parity.py (which must not
import torch, so these live outside conftest.py)."""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


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

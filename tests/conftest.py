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
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from goldens import GOLDEN, golden_names, load_golden, long_signal, x_digest  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs on the GPU box via gpurun)')


@pytest.fixture(scope='session')
def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False

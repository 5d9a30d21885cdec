import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
GOLDEN = os.path.join(ROOT, "tests", "golden")

CASES = ["testfloat", "rand16k", "u10_16k", "eq16k", "himeno", "unit64k", "q2", "ramp20k", "edge"]
BOUNDS = [1e-3, 1e-6]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from pyoracle import Oracle
    return Oracle()


_golden_cache = {}


def golden(bound):
    if bound not in _golden_cache:
        with np.load(os.path.join(GOLDEN, "golden_%g.npz" % bound), allow_pickle=False) as z:
            _golden_cache[bound] = {k: z[k] for k in z.files}
    return _golden_cache[bound]


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dc():
    """libdcamd on cuda:0 -- must load and initialise on the GPU box (no fallback).  torch's HIP
    runtime is brought up first (tests hand torch device buffers to the library), as bench.py does."""
    try:
        import torch
        torch.zeros(1, device="cuda")
    except ImportError:
        pass
    import dcamd
    L = dcamd.Lib()
    L.init(0)
    return L


CASES64 = ["testdouble", "u10_16k", "eq16k", "unit32k", "q2", "ramp20k", "mixed", "edge"]
_golden64_cache = {}


def golden64(bound):
    """Double-codec fixtures of tests/golden/make_golden64.py (compiled reference outputs)."""
    if bound not in _golden64_cache:
        with np.load(os.path.join(GOLDEN, "golden64_%g.npz" % bound), allow_pickle=False) as z:
            _golden64_cache[bound] = {k: z[k] for k in z.files}
    return _golden64_cache[bound]

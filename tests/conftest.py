"""Shared fixtures.  Markers: `gpu` = needs a real MI355X (run with -m gpu)."""
import importlib.util
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (HIP kernels in libsdr.so)")


def _load_oracle():
    spec = importlib.util.spec_from_file_location("fm_oracle", os.path.join(ROOT, "oracle", "fm_oracle.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def oracle():
    return _load_oracle()


@pytest.fixture(scope="session")
def sdr():
    import rtsdr
    return rtsdr


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
                cache[name] = {k: z[k] for k in z.files}
        return cache[name]
    return load


@pytest.fixture(scope="session")
def gpu_ctx(sdr):
    """The default libsdr context; fails loudly (no skip) when the GPU path is missing."""
    return sdr.get_context()


def rms(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2))) if a.size else 0.0


def maxabs(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b))) if a.size else 0.0


# the long-call PLL's pseudo-block geometry (csrc/pll.hip long_geom: <= 14 336 steps, so that a
# pseudo-block plus its pre-roll of <= 2 048 steps is one 16 384-step solve)
LONG_PB = 14336


def long_blocks(n):
    """pseudo-blocks of a PLL call of n samples (csrc/pll.hip long_geom): beyond 16 385 steps
    pseudo-blocks of <= 14 336; else 1"""
    return -(-n // LONG_PB) if n > 16385 else 1

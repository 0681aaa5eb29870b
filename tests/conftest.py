"""pytest configuration: the ``gpu`` marker and shared fixtures.

``-m "not gpu"`` runs everywhere (oracle vs golden fixtures, host logic, ABI load and
symbol checks).  ``-m gpu`` runs on the MI355X box and calls the HIP library through
its C-ABI; those tests FAIL (not skip) when the library or the GPU is missing, so a
silent CPU path can never pass them.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libolpe.so)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_golden(name)
        return cache[name]
    return get


@pytest.fixture(scope="session")
def lib_loaded():
    """libolpe.so loaded and a GPU visible to it (GPU tests fail, not skip, without)."""
    import ctypes as C
    from olpefit_amd import _lib
    lib = _lib.load()
    n = C.c_int(0)
    lib.olpe_device_count(C.byref(n))
    assert n.value >= 1, "no GPU visible to libolpe"
    return lib

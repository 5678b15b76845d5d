"""Test configuration: the `gpu` marker and import paths.

`-m "not gpu"` tests run on a CPU-only host (oracle vs golden vectors, host logic,
C-ABI symbol exports); `-m gpu` tests need an MI355X and call the HIP path through
the C-ABI, checking it against the oracle and the golden fixtures.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'auxiliary-pm-mcmc_amd')
for p in (PKG, os.path.join(REPO, 'oracle'), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP path through the C-ABI)')


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False)


def _gpu_selected(config):
    """The run asked for the GPU tests (`-m gpu`, not `-m "not gpu"`)."""
    expr = (config.getoption('markexpr', '') or '').replace(' ', '')
    return 'gpu' in expr and 'notgpu' not in expr


@pytest.fixture(scope='session')
def gpu_available(request):
    """A HIP device seen by libapm.so itself (not torch). A run selected with `-m gpu` on a host
    where the library or the device is missing FAILS (a broken ROCm runtime must not read as
    green-with-skips); other selections skip."""
    from gpdemo import _native
    try:
        _native.load_library()
        ok, why = True, ''
    except _native.NativeUnavailableError as e:
        ok, why = False, str(e)
    if not ok:
        if _gpu_selected(request.config):
            pytest.fail('-m gpu run without a usable HIP path: ' + why, pytrace=False)
        pytest.skip('no GPU: ' + why)
    return True

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


@pytest.fixture(scope='session')
def gpu_available():
    import torch  # only for device discovery on the GPU box
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return True

"""The C-ABI library loads on a CPU-only host and exports every symbol include/apm.h declares
(no compute calls without a GPU); the product refuses to run without a device (no fallback)."""
import os
import re

import pytest

from conftest import REPO


def _header_symbols():
    txt = open(os.path.join(REPO, 'include', 'apm.h')).read()
    return sorted(set(re.findall(r'\b(apm_[A-Za-z0-9_]+)\s*\(', txt)))


def test_header_and_binding_agree():
    from gpdemo import _native
    assert _header_symbols() == _native.exported_symbols()


def test_library_exports_every_symbol():
    from gpdemo import _native
    lib = _native.load_library(check_device=False)
    for name in _header_symbols():
        assert hasattr(lib, name), name
    assert lib.apm_version() >= 1


def test_no_cpu_fallback_without_device():
    import numpy as np
    from gpdemo import _native
    lib = _native.load_library(check_device=False)
    if lib.apm_device_count() > 0:
        pytest.skip('a GPU is visible')
    import gpdemo.estimators as est
    import gpdemo.kernels as krn
    import gpdemo.latent_posterior_approximations as lpa
    with pytest.raises(_native.NativeUnavailableError):
        est.LogMarginalLikelihoodApproxPosteriorISEstimator(
            np.zeros((4, 2)), np.ones(4), krn.make_kernel_func('ard'), lpa.laplace_approximation)
    with pytest.raises(_native.NativeUnavailableError):
        krn.diagonal_squared_exponential_kernel(np.empty((4, 4)), np.zeros((4, 2)), np.zeros(3))


def test_invalid_arguments_rejected():
    from gpdemo import _native
    lib = _native.load_library(check_device=False)
    assert lib.apm_create(0, 1, None, 0, 0, 0, None, 1e-8, 1, 1, 1, 1) is None
    assert b'invalid' in lib.apm_global_error()

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


@pytest.mark.gpu
def test_cache_slot_lifetimes_through_the_c_abi(gpu_available):
    """apm_cache_acquire / _copy / _release: the MH protocol of
    samplers.py:563-584 through the C-ABI alone - current and proposal caches owned at once, on
    accept the proposal's handle becomes current (one more owner) and the old slot is dropped; a
    released slot is reused; owner counts are checked; misuse is refused, not ignored."""
    import ctypes
    import numpy as np
    from gpdemo import _native
    lib = _native.load_library()
    rng = np.random.RandomState(0)
    X = rng.normal(size=(40, 3))
    y = np.where(rng.normal(size=40) > 0, 1., -1.)
    ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, 8, max_batch=1, n_slots=2, n_ubufs=1)
    h = ctx._h
    s = ctypes.c_int64(-1)
    assert lib.apm_cache_acquire(h, ctypes.byref(s)) == 0
    cur = s.value
    assert lib.apm_cache_acquire(h, ctypes.byref(s)) == 0
    prop = s.value
    assert cur != prop and lib.apm_cache_refcount(h, cur) == 1
    assert lib.apm_cache_acquire(h, ctypes.byref(s)) == _native.APM_E_NOMEM  # both owned
    ctx.u_upload(0, rng.normal(size=(40, 8)))
    th = np.zeros(4)
    v_cur, st, _ = ctx.theta_eval(_native.EST_IS, th[None], [0], [cur])
    v_prop, st2, _ = ctx.theta_eval(_native.EST_IS, (th + 0.3)[None], [0], [prop])
    assert st[0] == 0 and st2[0] == 0
    # accept: the sampler's new current handle is a copy of the proposal's
    assert lib.apm_cache_copy(h, prop) == 0 and lib.apm_cache_refcount(h, prop) == 2
    assert lib.apm_cache_release(h, cur) == 0 and lib.apm_cache_refcount(h, cur) == 0
    assert lib.apm_cache_release(h, prop) == 0  # the proposal variable goes out of scope
    assert lib.apm_cache_refcount(h, prop) == 1
    # the surviving cache still serves u-calls: same value as a fresh theta-call at that theta
    u1, _ = ctx.u_eval([prop], [0])
    np.testing.assert_allclose(u1[0], v_prop[0], rtol=0, atol=1e-9 * max(1., abs(v_prop[0])))
    assert lib.apm_cache_acquire(h, ctypes.byref(s)) == 0 and s.value == cur  # reused
    assert lib.apm_cache_release(h, cur) == 0
    assert lib.apm_cache_release(h, cur) == _native.APM_E_INVALID  # double release refused
    assert lib.apm_cache_copy(h, cur) == _native.APM_E_INVALID      # copy of a free slot refused
    assert lib.apm_cache_refcount(h, 99) < 0
    ctx.close()

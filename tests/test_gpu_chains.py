"""End-to-end drop-in parity: the API-compatible samplers (auxpm.samplers) driving the GPU
estimators (gpdemo.estimators -> libapm.so) reproduce chains of the reference.

* test_gp_chain_matches_reference: the reference's own APM E-SS + RD-SS chain
  (tests/golden/make_golden.py::gp_chain_fixture, reference estimator + reference sampler,
  E-SS+RD-SS.ipynb:157-176 wiring) re-run with the GPU estimator. Same host RNG stream, so every
  slice/accept decision agrees unless an estimate lands within the fp32 tolerance of a
  threshold: the traces must agree to 1e-6 and n_cubic_ops exactly.
* test_config1_ess_mh_chain_matches_oracle: BASELINE.json configs[1] shape (Pima-sized N=768,
  D=8, ARD-SE, APM with E-SS on u + MH on theta, N_imp=64): GPU estimator vs the oracle's CPU
  restatement of the reference estimator, driven by the same sampler and seed, and vs the
  reference's own chain (tests/golden/config1_ref.npz).
"""
import numpy as np
import pytest

import apm_oracle as orc
import auxpm.samplers as smp
import gpdemo.estimators as est
import gpdemo.kernels as krn
import gpdemo.latent_posterior_approximations as lpa
import gpdemo.utils as utils
from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def nat(gpu_available):
    from gpdemo import _native
    _native.load_library()
    return _native


def _x_sha256(X):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(X, dtype=np.float64).tobytes()).hexdigest()


def _closure(e, P, prior):
    """The notebooks' log_f_estimator closure (E-SS+RD-SS.ipynb:167-173): estimator + log-Gamma
    priors on every theta component (utils.py:39-59)."""
    def log_f_estimator(u, theta=None, cached_res=None):
        val, new_cache = e(u, theta, cached_res)
        lp = utils.log_gamma_log_pdf(theta[0], prior['a_sigma'], prior['b_sigma'])
        for k in range(1, P):
            lp += utils.log_gamma_log_pdf(theta[k], prior['a_tau'], prior['b_tau'])
        return val + lp, new_cache
    return log_f_estimator


@pytest.mark.parametrize('kind', ['iso', 'ard'])
def test_gp_chain_matches_reference(nat, kind):
    g = golden('gp_chain')
    X, y = g[kind + '_X'], g[kind + '_y']
    n, d = X.shape
    s = int(g[kind + '_s'])
    P = 2 if kind == 'iso' else d + 1
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    e = est.LogMarginalLikelihoodApproxPosteriorISEstimator(
        X, y, krn.make_kernel_func(kind, 1e-8), lpa.laplace_approximation)
    prng = np.random.RandomState(1234)

    def dir_w():
        dd = prng.normal(size=P)
        dd /= dd.dot(dd) ** 0.5
        return dd, 1.

    sampler = smp.APMEllSSPlusRandDirSliceSampler(
        _closure(e, P, prior), lambda: prng.normal(size=(n, s)), prng, dir_w, 0)
    prng.seed(77)
    theta_init = np.r_[np.log(prng.gamma(prior['a_sigma'], 1. / prior['b_sigma'])),
                       np.log(prng.gamma(prior['a_tau'], 1. / prior['b_tau'], size=P - 1))]
    np.testing.assert_array_equal(theta_init, g[kind + '_theta_init'])
    e.reset_cubic_op_count()
    th = sampler.get_samples(theta_init, g[kind + '_thetas'].shape[0])
    np.testing.assert_allclose(th, g[kind + '_thetas'], rtol=1e-6, atol=1e-6)
    assert e.n_cubic_ops == int(g[kind + '_n_cubic_ops'])


def test_config1_ess_mh_chain_matches_oracle(nat):
    n, d, s, n_sample = 768, 8, 64, 8
    X, y = utils.synthetic_gp_data(n, d, 1)
    P = d + 1
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    e_gpu = est.LogMarginalLikelihoodApproxPosteriorISEstimator(
        X, y, krn.make_kernel_func('ard', 1e-8), lpa.laplace_approximation)
    e_cpu = orc.ISEstimatorCPU(X, y, orc.make_kernel_func('ard', 1e-8))
    theta_init = np.r_[0.0, np.full(d, np.log(np.sqrt(d)))]
    runs = []
    for e in (e_gpu, e_cpu):
        prng = np.random.RandomState(4321)
        sampler = smp.APMEllSSPlusMHSampler(
            _closure(e, P, prior), lambda xp, xc, sc: -0.5 * np.sum(((xp - xc) / sc) ** 2),
            lambda x, sc: x + sc * prng.normal(size=x.shape), np.full(P, 0.05),
            lambda: prng.normal(size=(n, s)), prng)
        runs.append(sampler.get_samples(theta_init, n_sample))
    (th_g, nrej_g), (th_c, nrej_c) = runs
    assert nrej_g == nrej_c
    assert nrej_g < n_sample - 1  # the chain moved: the comparison covers accepted proposals
    np.testing.assert_allclose(th_g, th_c, rtol=1e-10, atol=1e-10)
    # ... and the REFERENCE's own chain with this wiring (tests/golden/make_golden_config1.py:
    # reference sampler + reference estimator, same data, seeds and draws)
    g = golden('config1_ref')
    assert str(g['x_sha256']) == _x_sha256(X)
    np.testing.assert_array_equal(y, g['y'])
    assert nrej_g == int(g['n_reject'])
    np.testing.assert_allclose(th_g, g['thetas'], rtol=1e-9, atol=1e-9)
    assert e_gpu.n_cubic_ops == int(g['n_cubic_ops'])

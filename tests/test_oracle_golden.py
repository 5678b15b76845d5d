"""Pin the CPU oracle (oracle/apm_oracle.py, oracle/gram.c) against golden vectors
produced by the reference itself (tests/golden/make_golden.py)."""
import numpy as np
import pytest

import apm_oracle as orc
from conftest import golden


def _gram_cases():
    g = golden('gram')
    keys = sorted({k.rsplit('_', 1)[0] for k in g.files if k.endswith('_thetas')})
    return g, keys


@pytest.mark.parametrize('impl', ['numpy', 'c'])
def test_gram_matches_reference(impl):
    g, keys = _gram_cases()
    for key in keys:
        kind = key.split('_')[0]
        X = g[key + '_X']
        for th, Kref in zip(g[key + '_thetas'], g[key + '_K']):
            K = np.empty_like(Kref)
            if impl == 'c':
                orc.c_gram(kind, K, X, th, 1e-8)
                # same op order, same libm exp -> bit-exact with the Cython build
                np.testing.assert_array_equal(K, Kref)
            else:
                (orc.iso_se_kernel if kind == 'iso' else orc.ard_se_kernel)(K, X, th, 1e-8)
                np.testing.assert_allclose(K, Kref, rtol=1e-14, atol=1e-300)


def test_gram_extra_theta_ignored():
    g = golden('gram')
    K = np.empty((9, 9))
    orc.c_gram('iso', K, g['extra_theta_X'], np.array([0.1, 0.2, 99.]), 1e-8)
    np.testing.assert_array_equal(K, g['extra_theta_K'])


def _cases():
    g = golden('estimators')
    for ci in range(int(g['n_cases'])):
        pre = 'c{0}_'.format(ci)
        yield ci, {k[len(pre):]: g[k] for k in g.files if k.startswith(pre)}


def test_laplace_matches_reference():
    for ci, c in _cases():
        f, C, lml, nops = orc.laplace_approximation(c['K'], c['y'], True, True)
        np.testing.assert_allclose(f, c['lap_f'], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(C, c['lap_C'], rtol=1e-9, atol=1e-12)
        assert abs(lml - float(c['lap_lml'])) < 1e-9 * max(1., abs(float(c['lap_lml'])))
        assert nops == int(c['lap_nops_cov_lml'])
        f2, nops2 = orc.laplace_approximation(c['K'], c['y'], False, False)
        assert nops2 == int(c['lap_nops_plain'])


def test_is_estimator_matches_reference():
    for ci, c in _cases():
        kf = orc.make_kernel_func(str(c['kind']), 1e-8)
        v1, cache, ops = orc.is_estimate(c['X'], c['y'], kf, c['ns1'], c['theta'])
        assert abs(v1 - float(c['is_logf1'])) < 1e-8 * max(1., abs(v1)), ci
        assert ops == int(c['is_ops'])
        v2, _, ops2 = orc.is_estimate(c['X'], c['y'], kf, c['ns2'], None, cache)
        assert abs(v2 - float(c['is_logf2'])) < 1e-8 * max(1., abs(v2)), ci
        assert ops2 == 0
        np.testing.assert_allclose(cache[2], c['f_post'], rtol=1e-10, atol=1e-12)


def test_priormc_and_laplace_estimators_match_reference():
    for ci, c in _cases():
        kf = orc.make_kernel_func(str(c['kind']), 1e-8)
        p1, Kc, ops = orc.priormc_estimate(c['X'], c['y'], kf, c['ns1'], c['theta'])
        assert abs(p1 - float(c['pmc_logf1'])) < 1e-9 * max(1., abs(p1))
        p2, _, _ = orc.priormc_estimate(c['X'], c['y'], kf, c['ns2'], None, Kc)
        assert abs(p2 - float(c['pmc_logf2'])) < 1e-9 * max(1., abs(p2))
        lml, ops = orc.laplace_estimate(c['X'], c['y'], kf, c['theta'])
        assert abs(lml - float(c['lapest_lml'])) < 1e-9 * max(1., abs(lml))
        assert ops == int(c['lapest_ops'])


def test_reformulated_is_equals_reference_form():
    """The GPU computes the algebraically identical form of estimators.py:221-241
    (DESIGN.md §3); pin that identity on the reference's own outputs."""
    for ci, c in _cases():
        st = orc.theta_state_reformulated(c['K'], c['y'])
        for ns, key in ((c['ns1'], 'is_logf1'), (c['ns2'], 'is_logf2')):
            v = orc.is_estimate_reformulated(c['y'], st, ns)
            ref = float(c[key])
            assert abs(v - ref) < 1e-7 * max(1., abs(ref)), (ci, v, ref)


def test_consistent_is_equals_reference_form():
    """The self-consistent form the device evaluates (ugemm.hip: nothing but f_s per sample,
    z = a + W f_post = C^-1 f_post) equals the reference's estimates on its own outputs, and -
    unlike the u-expanded form - it is insensitive to a perturbation of f_s's factor: with C_chol
    rounded to fp32 (the slot's precision) it moves by far less than the u-expanded form does."""
    for ci, c in _cases():
        st = orc.theta_state_reformulated(c['K'], c['y'])
        L32 = st['C_chol'].astype(np.float32).astype(np.float64)
        for ns, key in ((c['ns1'], 'is_logf1'), (c['ns2'], 'is_logf2')):
            ref = float(c[key])
            v = orc.is_estimate_consistent(c['y'], st, ns)
            assert abs(v - ref) < 1e-7 * max(1., abs(ref)), (ci, v, ref)
            d_cons = abs(orc.is_estimate_consistent(c['y'], st, ns, L32) - ref)
            st32 = dict(st, C_chol=L32)
            d_exp = abs(orc.is_estimate_reformulated(c['y'], st32, ns) - ref)
            assert d_cons <= max(d_exp, 1e-9), (ci, d_cons, d_exp)


def test_laplace_max_iters_error():
    e = golden('errors')
    with pytest.raises(orc.MaximumIterationsExceededError) as ei:
        orc.laplace_approximation(e['K'], e['y'], max_iters=1)
    assert str(ei.value) == str(e['laplace_maxiter_msg'])


def test_utils_match_reference():
    u = golden('utils')
    np.testing.assert_allclose(orc.log_gamma_log_pdf(u['x'], 1.1, 0.1), u['lgl'], rtol=1e-14)
    Xn, mn, sd = orc.normalise_inputs(u['Xraw'])
    np.testing.assert_allclose(Xn, u['Xn'], rtol=1e-14)


def test_pushthrough_factor_equals_reference_chol_c():
    """The device's route to C_chol (chol(K), M = I + L_K^T W L_K, UL Cholesky; DESIGN.md §3.1
    step 3), restated in fp64 by the oracle, reproduces the reference's chol(C), g, log|B| and
    estimates on the reference's own outputs."""
    for ci, c in _cases():
        pt = orc.theta_state_pushthrough(c['K'], c['y'])
        rf = orc.theta_state_reformulated(c['K'], c['y'])
        scale = np.abs(c['C_chol']).max()
        np.testing.assert_allclose(pt['C_chol'], c['C_chol'], rtol=0, atol=1e-8 * scale)
        assert abs(pt['logdet_B'] - rf['logdet_B']) < 1e-8 * max(1., abs(rf['logdet_B']))
        np.testing.assert_allclose(pt['g'], rf['g'], rtol=1e-6, atol=1e-8 * np.abs(rf['g']).max())
        for ns, key in ((c['ns1'], 'is_logf1'), (c['ns2'], 'is_logf2')):
            v = orc.is_estimate_reformulated(c['y'], pt, ns)
            assert abs(v - float(c[key])) < 1e-7 * max(1., abs(float(c[key]))), (ci, key)


def test_extreme_theta_errors_match_reference():
    """Reference behaviour at extreme theta (tests/golden/errors.npz): chol(K) failing raises
    LinAlgError (estimators.py:206), chol(C) failing raises InvalidCovarianceMatrixError
    (estimators.py:208-215); the oracle restatement raises the same, with the same message
    prefix. The push-through route the device takes does not form C and returns a finite
    state at the InvalidCovarianceMatrixError thetas (the documented deviation)."""
    e = golden('errors')
    X, y, ns = e['extreme_X'], e['extreme_y'], e['extreme_ns']
    kf = orc.make_kernel_func('iso', 1e-8)
    with pytest.raises(np.linalg.LinAlgError):
        orc.is_estimate(X, y, kf, ns, e['cholk_theta'])
    assert str(e['cholk_raised']) == 'LinAlgError'
    for name in ('icm_a', 'icm_b'):
        assert str(e[name + '_raised']) == 'InvalidCovarianceMatrixError'
        with pytest.raises(orc.InvalidCovarianceMatrixError) as ei:
            orc.is_estimate(X, y, kf, ns, e[name + '_theta'])
        assert str(ei.value).startswith('Posterior covariance matrix not PSD: sum of negative '
                                        'eigenvalues -')
        K = np.empty((X.shape[0],) * 2)
        kf(K, X, e[name + '_theta'])
        st = orc.theta_state_pushthrough(K, y)
        assert np.isfinite(orc.is_estimate_reformulated(y, st, ns))


def test_pmmh_chain_fixture_consistent():
    """configs[0] golden chain (make_golden.py::pmmh_chain_fixture): its recorded estimator
    calls re-evaluate with the oracle (Laplace phase exactly; IS phase with the same u draws
    replayed from the seeded prng is checked on the GPU in test_gpu_configs)."""
    g = golden('pmmh_chain')
    X, y = g['X'], g['y']
    kf = orc.make_kernel_func('iso', 1e-8)
    lml, _ = orc.laplace_estimate(X, y, kf, g['theta_init'])
    assert abs(lml - float(g['calls'][0])) < 1e-8 * max(1., abs(lml))
    assert g['thetas'].shape == (30, 2) and int(g['n_adapt_calls']) == 30


def test_philox_known_answers():
    """The oracle's Philox4x32-10 reproduces the published known-answer vectors."""
    for inp, out in orc.PHILOX_KAT:
        np.testing.assert_array_equal(orc.philox4x32_10(inp[:4], inp[4:])[0],
                                      np.array(out, dtype=np.uint32))


def test_config1_chain_oracle_equals_reference():
    """BASELINE configs[1] (E-SS + MH, ARD-SE, N=768 D=8, N_imp=64): the API sampler over the
    oracle's CPU estimator reproduces the reference's own chain (tests/golden/config1_ref.npz,
    make_golden_config1.py: reference sampler + reference estimator, same data, seeds, draws)."""
    import hashlib
    import auxpm.samplers as smp
    import gpdemo.utils as utils
    g = golden('config1_ref')
    n, d, s = 768, 8, 64
    X, y = utils.synthetic_gp_data(n, d, 1)
    assert hashlib.sha256(np.ascontiguousarray(X, np.float64).tobytes()).hexdigest() == \
        str(g['x_sha256'])
    np.testing.assert_array_equal(y, g['y'])
    P = d + 1
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    e = orc.ISEstimatorCPU(X, y, orc.make_kernel_func('ard', 1e-8))

    def log_f(u, theta=None, cached_res=None):
        val, new_cache = e(u, theta, cached_res)
        lp = utils.log_gamma_log_pdf(theta[0], prior['a_sigma'], prior['b_sigma'])
        for k in range(1, P):
            lp += utils.log_gamma_log_pdf(theta[k], prior['a_tau'], prior['b_tau'])
        return val + lp, new_cache
    prng = np.random.RandomState(4321)
    sampler = smp.APMEllSSPlusMHSampler(
        log_f, lambda xp, xc, sc: -0.5 * np.sum(((xp - xc) / sc) ** 2),
        lambda x, sc: x + sc * prng.normal(size=x.shape), np.full(P, 0.05),
        lambda: prng.normal(size=(n, s)), prng)
    th, nrej = sampler.get_samples(g['theta_init'], g['thetas'].shape[0])
    assert nrej == int(g['n_reject'])
    np.testing.assert_allclose(th, g['thetas'], rtol=1e-10, atol=1e-10)
    assert e.n_cubic_ops == int(g['n_cubic_ops'])

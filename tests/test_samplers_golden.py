"""Host sampler logic (auxpm) against traces recorded from the reference samplers with a cheap
analytic estimator (tests/golden/make_golden.py::sampler_fixture). Bit-exact: same RNG draw
order, same float expressions, same cache protocol."""
import warnings

import numpy as np
import pytest

import auxpm.mcmc_updates as mcmc
import auxpm.samplers as smp
import gpdemo.utils as utils
from conftest import golden

P = 3
N_S = 40
U_SHAPE = (5, 2)


def analytic_log_f_u(u, theta, cached=None):
    if cached is None:
        cached = (np.atleast_1d(theta).copy(),)
    th = cached[0]
    m = 0.3 * np.tanh(u.mean())
    return float(-0.5 * np.sum((th - m) ** 2 / np.arange(1, th.shape[0] + 1))), cached


@pytest.fixture(scope='module')
def g():
    return golden('samplers')


@pytest.mark.parametrize('variant', ['met', 'mh'])
def test_pmmh(g, variant):
    def lf_theta(theta):
        return float(-0.5 * np.sum(theta ** 2 / np.arange(1, P + 1)))
    prng = np.random.RandomState(1)
    prop = lambda x, s: x + s * prng.normal(size=x.shape)  # noqa: E731
    lpd = None if variant == 'met' else (lambda xp, xc, s: -0.5 * np.sum(((xp - xc) / s) ** 2))
    s = smp.PMMHSampler(lf_theta, lpd, prop, np.ones(P) * 0.8, prng)
    th, nrej = s.get_samples(np.ones(P) * 0.5, N_S)
    np.testing.assert_array_equal(th, g['pmmh_{0}_thetas'.format(variant)])
    assert nrej == int(g['pmmh_{0}_nrej'.format(variant)])
    prng.seed(5)
    s.prop_scales = np.ones(P) * 3.
    ath, aps, aar = s.adaptive_run(np.zeros(P), 10, 4, 0.15, 0.30, utils.adapt_factor_func)
    np.testing.assert_array_equal(ath, g['pmmh_{0}_adapt'.format(variant)])
    np.testing.assert_array_equal(aps, g['pmmh_{0}_adapt_scales'.format(variant)])
    np.testing.assert_array_equal(aar, g['pmmh_{0}_adapt_rates'.format(variant)])


def test_apm_mi_mh(g):
    prng = np.random.RandomState(2)
    s = smp.APMMetIndPlusMHSampler(
        analytic_log_f_u, None, lambda x, sc: x + sc * prng.normal(size=x.shape), np.ones(P) * 0.7,
        lambda: prng.normal(size=U_SHAPE), prng)
    th, nrej = s.get_samples(np.zeros(P), N_S)
    np.testing.assert_array_equal(th, g['mimh_thetas'])
    assert tuple(nrej) == tuple(g['mimh_nrej'])


def test_apm_ess_mh_and_adaptive(g):
    prng = np.random.RandomState(3)
    s = smp.APMEllSSPlusMHSampler(
        analytic_log_f_u, lambda xp, xc, sc: -0.5 * np.sum(((xp - xc) / sc) ** 2),
        lambda x, sc: x + sc * prng.normal(size=x.shape), np.ones(P) * 0.7,
        lambda: prng.normal(size=U_SHAPE), prng)
    th, nrej = s.get_samples(np.zeros(P), N_S)
    np.testing.assert_array_equal(th, g['essmh_thetas'])
    assert nrej == int(g['essmh_nrej'])
    ath, aps, aar = s.adaptive_run(np.zeros(P), 8, 3, 0.15, 0.30, utils.adapt_factor_func)
    np.testing.assert_array_equal(ath, g['essmh_adapt'])
    np.testing.assert_array_equal(aps, g['essmh_adapt_scales'])
    np.testing.assert_array_equal(aar, g['essmh_adapt_rates'])


@pytest.mark.parametrize('name', ['miseq', 'mirdss', 'essrdss', 'essrdss_so', 'essess'])
def test_slice_samplers(g, name):
    prng = np.random.RandomState(int(g[name + '_seed']))

    def dir_w():
        d = prng.normal(size=P)
        d /= d.dot(d) ** 0.5
        return d, 1.

    mk = {
        'miseq': lambda: smp.APMMetIndPlusSeqSliceSampler(
            analytic_log_f_u, lambda: prng.normal(size=U_SHAPE), prng, np.ones(P) * 0.9, 2),
        'mirdss': lambda: smp.APMMetIndPlusRandDirSliceSampler(
            analytic_log_f_u, lambda: prng.normal(size=U_SHAPE), prng, dir_w, 0),
        'essrdss': lambda: smp.APMEllSSPlusRandDirSliceSampler(
            analytic_log_f_u, lambda: prng.normal(size=U_SHAPE), prng, dir_w, 0),
        'essrdss_so': lambda: smp.APMEllSSPlusRandDirSliceSampler(
            analytic_log_f_u, lambda: prng.normal(size=U_SHAPE), prng, dir_w, 3),
        'essess': lambda: smp.APMEllSSPlusEllSSSampler(
            analytic_log_f_u, lambda: prng.normal(size=U_SHAPE), lambda: prng.normal(size=P),
            prng),
    }[name]
    res = mk().get_samples(np.full(P, 0.2), N_S)
    if isinstance(res, tuple):
        th, nrej = res
        assert np.all(np.atleast_1d(nrej) == g[name + '_nrej'])
    else:
        th = res
        assert name + '_nrej' not in g.files
    np.testing.assert_array_equal(th, g[name + '_thetas'])


def test_raw_updates(g):
    prng = np.random.RandomState(9)
    lf = lambda x: float(-0.5 * np.sum(np.atleast_1d(x) ** 2))  # noqa: E731
    xs = []
    x, l = np.array([0.3, -0.2]), lf(np.array([0.3, -0.2]))
    for _ in range(10):
        x, l = mcmc.elliptical_slice_step(x, l, lf, prng, prng.normal(size=2))
        xs.append(x.copy())
    np.testing.assert_array_equal(np.array(xs), g['ess_steps'])
    xs = []
    x, l = 0.1, lf(0.1)
    for mso in (0, 1, 4, 0, 7):
        x, l = mcmc.linear_slice_step(x, l, lf, 0.5, prng, mso)
        xs.append(x)
    np.testing.assert_array_equal(np.array(xs), g['lss_steps'])
    xs = []
    x, l = np.zeros(2), lf(np.zeros(2))
    for mode in range(4):
        if mode == 0:
            x, l, r = mcmc.metropolis_indepedence_step(x, l, lf, prng, lambda: prng.normal(size=2))
        elif mode == 1:
            x, l, r = mcmc.metropolis_indepedence_step(
                x, l, lf, prng, lambda: prng.normal(size=2), None, lambda z: -0.5 * np.sum(z ** 2))
        elif mode == 2:
            x, l, r = mcmc.metropolis_indepedence_step(
                x, l, lf, prng, lambda p: p * prng.normal(size=2), 2.0,
                lambda z, p: -0.5 * np.sum((z / p) ** 2))
        else:
            x, l, r = mcmc.metropolis_indepedence_step(
                x, l, lf, prng, lambda p: p * prng.normal(size=2), 2.0)
        xs.append(np.r_[x, l, r])
    np.testing.assert_array_equal(np.array(xs), g['mi_steps'])


def test_slice_max_iters_error(g):
    prng = np.random.RandomState(4)
    with pytest.raises(mcmc.MaximumIterationsExceededError) as ei:
        mcmc.linear_slice_step(0., 0., lambda x: -np.inf, 1., prng, 0, 5)
    assert str(ei.value) == str(g['lss_maxiter_msg'])


def test_slice_collapse_warns():
    class Zero(object):
        def uniform(self):
            return 0.5
    # x_prop == x_curr: bracket [x-0.5w, x+0.5w], uniform 0.5 -> x_prop == x_curr
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        x, l = mcmc.linear_slice_step(1.0, 0.0, lambda x: -1.0, 2.0, Zero(), 0, 10)
    assert x == 1.0 and l == 0.0 and any('collapsed' in str(i.message) for i in w)


def test_utils_golden():
    u = golden('utils')
    np.testing.assert_array_equal(utils.log_gamma_log_pdf(u['x'], 1.1, 0.1), u['lgl'])
    np.testing.assert_array_equal(utils.gamma_log_pdf(np.exp(u['x']), 1.1, 0.1), u['gl'])
    np.testing.assert_array_equal(np.array([utils.adapt_factor_func(b, 20) for b in range(25)]),
                                  u['adapt'])
    Xn, mn, sd = utils.normalise_inputs(u['Xraw'])
    np.testing.assert_array_equal(Xn, u['Xn'])


def test_save_run_schema(tmp_path):
    res, par = utils.save_run(str(tmp_path), 'x', np.zeros((3, 2)), (1, 2), 7, 1.5, {'a': 1})
    z = np.load(res)
    np.testing.assert_array_equal(z['n_reject_n_cubic_ops_comp_time'], [1, 2, 7, 1.5])
    res, par = utils.save_adaptive_run(str(tmp_path), 'y', np.zeros((2, 2)), np.ones((1, 2)),
                                       np.ones(1), np.zeros((3, 2)), 4, 7, 1.5, {'a': 1})
    z = np.load(res)
    assert set(z.files) == {'adapt_thetas', 'adapt_prop_scales', 'adapt_accept_rates', 'thetas',
                            'n_reject_n_cubic_ops_comp_time'}


def test_load_uci_data(tmp_path, monkeypatch):
    """Notebook data path (E-SS+RD-SS.ipynb :39, :85-87): $DATA_DIR/uci/<set>_{X,y}.txt read with
    genfromtxt, X normalised with normalise_inputs."""
    u = golden('utils')
    uci = tmp_path / 'uci'
    uci.mkdir()
    y = np.where(np.arange(u['Xraw'].shape[0]) % 3 == 0, 1., -1.)
    np.savetxt(str(uci / 'toy_X.txt'), u['Xraw'])
    np.savetxt(str(uci / 'toy_y.txt'), y)
    monkeypatch.setenv('DATA_DIR', str(tmp_path))
    X, yy, mn, sd = utils.load_uci_data('toy')
    np.testing.assert_allclose(X, u['Xn'], rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(mn, u['mn'], rtol=1e-14)
    np.testing.assert_array_equal(yy, y)
    Xr, _ = utils.load_uci_data('toy', str(uci), normalise=False)
    np.testing.assert_allclose(Xr, u['Xraw'], rtol=1e-15)
    np.savetxt(str(uci / 'bad_X.txt'), u['Xraw'])
    np.savetxt(str(uci / 'bad_y.txt'), np.abs(y) * 0.)
    with pytest.raises(ValueError):
        utils.load_uci_data('bad', str(uci))


def test_log_prior_ard_batch_matches_scalar():
    """The batched sampler's vectorised prior equals the notebook closure's per-theta sum."""
    prior = dict(a_tau=1., b_tau=1. / 32 ** 0.5, a_sigma=1.1, b_sigma=0.1)
    th = np.random.RandomState(0).normal(scale=2., size=(64, 33))
    ref = np.array([utils.log_prior_ard(t, prior) for t in th])
    np.testing.assert_allclose(utils.log_prior_ard_batch(th, prior), ref, rtol=1e-14, atol=1e-12)
    np.testing.assert_allclose(utils.log_prior_ard_batch(th[:, :2], prior),
                               [utils.log_prior_ard(t, prior) for t in th[:, :2]], rtol=1e-14)

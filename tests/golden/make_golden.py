"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference, read-only, and the reference's
kernels.pyx compiled by `make -C oracle ref` into oracle/_ref/):

    python tests/golden/make_golden.py

Nothing from the reference is copied: the fixtures are inputs + the reference's outputs.
Import-time adaptations (no source edits, documented in DESIGN.md §6):
  * scipy.misc.logsumexp was moved to scipy.special.logsumexp (scipy >= 1.3);
    gpdemo/estimators.py:14 imports the old name, so the alias is set before import.
  * auxpm/samplers.py:11 is a Python-2 implicit relative import (`import mcmc_updates`);
    sys.modules['mcmc_updates'] is pointed at auxpm.mcmc_updates before import.
Bytecode writing is disabled so nothing is written under /root/reference.
"""
import glob
import importlib.util
import os
import sys

sys.dont_write_bytecode = True

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

import numpy as np  # noqa: E402
import scipy.misc  # noqa: E402
import scipy.special  # noqa: E402

scipy.misc.logsumexp = scipy.special.logsumexp
sys.path.insert(0, REF)
import auxpm.mcmc_updates as ref_mcmc  # noqa: E402

sys.modules['mcmc_updates'] = ref_mcmc
import auxpm.samplers as ref_smp  # noqa: E402
import gpdemo.estimators as ref_est  # noqa: E402
import gpdemo.latent_posterior_approximations as ref_lpa  # noqa: E402
import gpdemo.utils as ref_utils  # noqa: E402

_so = glob.glob(os.path.join(REPO, 'oracle', '_ref', 'kernels*.so'))
if not _so:
    raise SystemExit('build the reference Gram first: make -C oracle ref')
_spec = importlib.util.spec_from_file_location('gpdemo.kernels', _so[0])
ref_krn = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(ref_krn)


def synth_data(n, d, seed, kind='ard'):
    """Synthetic probit GP-classification data: X ~ N(0,1) normalised,
    y = sign(f*) with f* a GP prior draw at log sigma = 0, log tau_k = log sqrt(D)."""
    rng = np.random.RandomState(seed)
    X, _, _ = ref_utils.normalise_inputs(rng.normal(size=(n, d)))
    theta_star = np.r_[0., np.full(d if kind == 'ard' else 1, 0.5 * np.log(d))]
    K = np.empty((n, n))
    if kind == 'ard':
        ref_krn.diagonal_squared_exponential_kernel(K, X, theta_star, 1e-6)
    else:
        ref_krn.isotropic_squared_exponential_kernel(K, X, theta_star, 1e-6)
    f = np.linalg.cholesky(K).dot(rng.normal(size=n))
    y = np.where(f >= 0, 1., -1.)
    return X, y


def kfunc(kind, eps):
    if kind == 'ard':
        return lambda K, X, th: ref_krn.diagonal_squared_exponential_kernel(K, X, th, eps)
    return lambda K, X, th: ref_krn.isotropic_squared_exponential_kernel(K, X, th, eps)


def gram_fixture():
    rng = np.random.RandomState(11)
    out = {}
    for kind, n, d in (('iso', 37, 3), ('ard', 37, 5), ('ard', 130, 8), ('iso', 1, 2)):
        X = rng.normal(size=(n, d))
        P = 2 if kind == 'iso' else d + 1
        thetas = np.stack([np.zeros(P), rng.normal(scale=1.5, size=P),
                           np.r_[0.7, np.full(P - 1, 3.0)], np.r_[-1.0, np.full(P - 1, -2.0)]])
        Ks = []
        for th in thetas:
            K = np.empty((n, n))
            kfunc(kind, 1e-8)(K, X, th)
            Ks.append(K)
        key = '{0}_n{1}_d{2}'.format(kind, n, d)
        out[key + '_X'] = X
        out[key + '_thetas'] = thetas
        out[key + '_K'] = np.stack(Ks)
    # extra theta entries are ignored (kernels.pyx reads theta[0], theta[1] / theta[:D+1])
    X = rng.normal(size=(9, 2))
    K = np.empty((9, 9))
    ref_krn.isotropic_squared_exponential_kernel(K, X, np.array([0.1, 0.2, 99.]), 1e-8)
    out['extra_theta_X'] = X
    out['extra_theta_K'] = K
    np.savez_compressed(os.path.join(HERE, 'gram.npz'), **out)


def estimator_fixture():
    out = {}
    cases = [('iso', 60, 3, 4, np.array([0.3, 0.4])),
             ('ard', 97, 4, 16, np.array([0.5, 0.1, 0.6, -0.2, 0.9])),
             ('ard', 200, 8, 64, np.r_[1.2, np.full(8, np.log(np.sqrt(8.)) + 1.0)]),
             ('ard', 128, 6, 1, np.r_[-0.5, np.full(6, 0.3)])]
    for ci, (kind, n, d, s, theta) in enumerate(cases):
        X, y = synth_data(n, d, 100 + ci, kind)
        rng = np.random.RandomState(200 + ci)
        ns1 = rng.normal(size=(n, s))
        ns2 = rng.normal(size=(n, s))
        kf = kfunc(kind, 1e-8)
        est = ref_est.LogMarginalLikelihoodApproxPosteriorISEstimator(
            X, y, kf, ref_lpa.laplace_approximation)
        v1, cache = est(ns1, theta)
        ops1 = est.n_cubic_ops
        v2, cache2 = est(ns2, theta, cache)
        K_chol, C_chol, f_post = cache
        # Laplace internals (stand-alone laplace_approximation on the same K)
        K = np.empty((n, n))
        kf(K, X, theta)
        f_l, C_l, lml_l, nops_cl = ref_lpa.laplace_approximation(K, y, True, True)
        f_o, nops_o = ref_lpa.laplace_approximation(K, y, False, False)
        lap = ref_est.LogMarginalLikelihoodLaplaceEstimator(X, y, kf)
        lml_e = lap(theta)
        pmc = ref_est.LogMarginalLikelihoodPriorMCEstimator(X, y, kf)
        p1, Kc = pmc(ns1, theta)
        p2, _ = pmc(ns2, None, Kc)
        pre = 'c{0}_'.format(ci)
        out.update({pre + 'kind': np.array(kind), pre + 'X': X, pre + 'y': y,
                    pre + 'theta': theta, pre + 'ns1': ns1, pre + 'ns2': ns2,
                    pre + 'is_logf1': v1, pre + 'is_logf2': v2, pre + 'is_ops': ops1,
                    pre + 'K': K, pre + 'K_chol': K_chol, pre + 'C_chol': C_chol,
                    pre + 'f_post': f_post, pre + 'lap_f': f_l, pre + 'lap_C': C_l,
                    pre + 'lap_lml': lml_l, pre + 'lap_nops_cov_lml': nops_cl,
                    pre + 'lap_nops_plain': nops_o, pre + 'lapest_lml': lml_e,
                    pre + 'lapest_ops': lap.n_cubic_ops,
                    pre + 'pmc_logf1': p1, pre + 'pmc_logf2': p2,
                    pre + 'pmc_ops': pmc.n_cubic_ops})
    out['n_cases'] = len(cases)
    np.savez_compressed(os.path.join(HERE, 'estimators.npz'), **out)


def error_fixture():
    X, y = synth_data(40, 3, 7, 'ard')
    K = np.empty((40, 40))
    kfunc('ard', 1e-8)(K, X, np.r_[1., 0., 0., 0.])
    raised = ''
    try:
        ref_lpa.laplace_approximation(K, y, max_iters=1)
    except ref_lpa.MaximumIterationsExceededError as e:
        raised = str(e)
    est = ref_est.LogMarginalLikelihoodApproxPosteriorISEstimator(
        X, y, kfunc('ard', 1e-8), ref_lpa.laplace_approximation)
    try:
        est(np.zeros((40, 2)))
        verr = ''
    except ValueError as e:
        verr = str(e)
    # extreme theta (iso, N=60 D=3): chol(K) fails -> numpy LinAlgError (estimators.py:206,
    # uncaught), and the two thetas where chol(K) succeeds but chol(C) of C = K - V^T V fails ->
    # InvalidCovarianceMatrixError (estimators.py:208-215), found by a grid search over
    # log sigma in 6..16, log tau in 1..5
    Xe, ye = synth_data(60, 3, 100, 'iso')
    kf = kfunc('iso', 1e-8)
    ns = np.random.RandomState(0).normal(size=(60, 4))
    cases = {'cholk': np.array([20., 6.]), 'icm_a': np.array([15., 5.]),
             'icm_b': np.array([16., 3.])}
    out = {}
    for name, th in cases.items():
        est = ref_est.LogMarginalLikelihoodApproxPosteriorISEstimator(
            Xe, ye, kf, ref_lpa.laplace_approximation)
        try:
            est(ns, th)
            kind = 'none'
            msg = ''
        except ref_est.InvalidCovarianceMatrixError as e:
            kind, msg = 'InvalidCovarianceMatrixError', str(e)
        except np.linalg.LinAlgError as e:
            kind, msg = 'LinAlgError', str(e)
        out[name + '_theta'] = th
        out[name + '_raised'] = np.array(kind)
        out[name + '_msg'] = np.array(msg)
    np.savez_compressed(os.path.join(HERE, 'errors.npz'), X=X, y=y, K=K,
                        laplace_maxiter_msg=np.array(raised), valueerror_msg=np.array(verr),
                        extreme_X=Xe, extreme_y=ye, extreme_ns=ns, **out)


# ----------------------------------------------------------------------------- sampler traces


def analytic_log_f_u(u, theta, cached=None):
    """Cheap analytic stand-in for log_f_estimator(u, theta[, cached]) used to pin the
    sampler control flow: a Gaussian in theta whose mean depends on u."""
    if cached is None:
        cached = (np.atleast_1d(theta).copy(),)
    th = cached[0]
    m = 0.3 * np.tanh(u.mean())
    return float(-0.5 * np.sum((th - m) ** 2 / np.arange(1, th.shape[0] + 1))), cached


def sampler_fixture():
    out = {}
    P = 3
    n_s = 40
    u_shape = (5, 2)

    # PM-MH (Metropolis + MH variants)
    def lf_theta(theta):
        return float(-0.5 * np.sum(theta ** 2 / np.arange(1, P + 1)))
    for variant in ('met', 'mh'):
        prng = np.random.RandomState(1)
        prop = lambda x, s: x + s * prng.normal(size=x.shape)  # noqa: E731
        lpd = None if variant == 'met' else (lambda xp, xc, s: -0.5 * np.sum(((xp - xc) / s) ** 2))
        smp = ref_smp.PMMHSampler(lf_theta, lpd, prop, np.ones(P) * 0.8, prng)
        th, nrej = smp.get_samples(np.ones(P) * 0.5, n_s)
        out['pmmh_{0}_thetas'.format(variant)] = th
        out['pmmh_{0}_nrej'.format(variant)] = nrej
        # adaptive run
        prng.seed(5)
        smp.prop_scales = np.ones(P) * 3.
        ath, aps, aar = smp.adaptive_run(np.zeros(P), 10, 4, 0.15, 0.30, ref_utils.adapt_factor_func)
        out['pmmh_{0}_adapt'.format(variant)] = ath
        out['pmmh_{0}_adapt_scales'.format(variant)] = aps
        out['pmmh_{0}_adapt_rates'.format(variant)] = aar

    # APM MI + MH
    prng = np.random.RandomState(2)
    smp = ref_smp.APMMetIndPlusMHSampler(
        analytic_log_f_u, None, lambda x, s: x + s * prng.normal(size=x.shape), np.ones(P) * 0.7,
        lambda: prng.normal(size=u_shape), prng)
    th, nrej = smp.get_samples(np.zeros(P), n_s)
    out['mimh_thetas'] = th
    out['mimh_nrej'] = np.array(nrej)

    # APM ESS + MH (with log prop density, and adaptive)
    prng = np.random.RandomState(3)
    smp = ref_smp.APMEllSSPlusMHSampler(
        analytic_log_f_u, lambda xp, xc, s: -0.5 * np.sum(((xp - xc) / s) ** 2),
        lambda x, s: x + s * prng.normal(size=x.shape), np.ones(P) * 0.7,
        lambda: prng.normal(size=u_shape), prng)
    th, nrej = smp.get_samples(np.zeros(P), n_s)
    out['essmh_thetas'] = th
    out['essmh_nrej'] = np.array(nrej)
    ath, aps, aar = smp.adaptive_run(np.zeros(P), 8, 3, 0.15, 0.30, ref_utils.adapt_factor_func)
    out['essmh_adapt'] = ath
    out['essmh_adapt_scales'] = aps
    out['essmh_adapt_rates'] = aar

    def dir_w():
        d = prng.normal(size=P)
        d /= d.dot(d) ** 0.5
        return d, 1.

    # APM MI + seq SS, MI + RD-SS, ESS + RD-SS (with and without step-out), ESS + ESS
    for name, mk in (
            ('miseq', lambda: ref_smp.APMMetIndPlusSeqSliceSampler(
                analytic_log_f_u, lambda: prng.normal(size=u_shape), prng, np.ones(P) * 0.9, 2)),
            ('mirdss', lambda: ref_smp.APMMetIndPlusRandDirSliceSampler(
                analytic_log_f_u, lambda: prng.normal(size=u_shape), prng, dir_w, 0)),
            ('essrdss', lambda: ref_smp.APMEllSSPlusRandDirSliceSampler(
                analytic_log_f_u, lambda: prng.normal(size=u_shape), prng, dir_w, 0)),
            ('essrdss_so', lambda: ref_smp.APMEllSSPlusRandDirSliceSampler(
                analytic_log_f_u, lambda: prng.normal(size=u_shape), prng, dir_w, 3)),
            ('essess', lambda: ref_smp.APMEllSSPlusEllSSSampler(
                analytic_log_f_u, lambda: prng.normal(size=u_shape),
                lambda: prng.normal(size=P), prng))):
        prng = np.random.RandomState(len(name) * 7 + 1)
        smp = mk()
        res = smp.get_samples(np.full(P, 0.2), n_s)
        if isinstance(res, tuple):
            th, nrej = res
            out[name + '_nrej'] = np.array(nrej)
        else:
            th = res
        out[name + '_thetas'] = th
        out[name + '_seed'] = len(name) * 7 + 1

    # raw mcmc_updates: ESS / linear slice / MI steps on a 1-D target, incl. step-out
    prng = np.random.RandomState(9)
    lf = lambda x: float(-0.5 * np.sum(np.atleast_1d(x) ** 2))  # noqa: E731
    xs = []
    x, l = np.array([0.3, -0.2]), lf(np.array([0.3, -0.2]))
    for _ in range(10):
        x, l = ref_mcmc.elliptical_slice_step(x, l, lf, prng, prng.normal(size=2))
        xs.append(x.copy())
    out['ess_steps'] = np.array(xs)
    xs = []
    x, l = 0.1, lf(0.1)
    for mso in (0, 1, 4, 0, 7):
        x, l = ref_mcmc.linear_slice_step(x, l, lf, 0.5, prng, mso)
        xs.append(x)
    out['lss_steps'] = np.array(xs)
    # MI step with and without log proposal density / prop params
    xs = []
    x, l = np.zeros(2), lf(np.zeros(2))
    for mode in range(4):
        if mode == 0:
            x, l, r = ref_mcmc.metropolis_indepedence_step(
                x, l, lf, prng, lambda: prng.normal(size=2))
        elif mode == 1:
            x, l, r = ref_mcmc.metropolis_indepedence_step(
                x, l, lf, prng, lambda: prng.normal(size=2), None,
                lambda z: -0.5 * np.sum(z ** 2))
        elif mode == 2:
            x, l, r = ref_mcmc.metropolis_indepedence_step(
                x, l, lf, prng, lambda p: p * prng.normal(size=2), 2.0,
                lambda z, p: -0.5 * np.sum((z / p) ** 2))
        else:
            x, l, r = ref_mcmc.metropolis_indepedence_step(
                x, l, lf, prng, lambda p: p * prng.normal(size=2), 2.0)
        xs.append(np.r_[x, l, r])
    out['mi_steps'] = np.array(xs)

    # slice non-termination -> MaximumIterationsExceededError message prefix
    prng = np.random.RandomState(4)
    try:
        ref_mcmc.linear_slice_step(0., 0., lambda x: -np.inf, 1., prng, 0, 5)
        msg = ''
    except ref_mcmc.MaximumIterationsExceededError as e:
        msg = str(e)
    out['lss_maxiter_msg'] = np.array(msg)
    np.savez_compressed(os.path.join(HERE, 'samplers.npz'), **out)


def gp_chain_fixture():
    """A short APM E-SS + RD-SS chain on a small real GP problem with the reference
    estimator: pins the wiring of E-SS+RD-SS.ipynb:157-176 (closure adds log-Gamma priors)."""
    out = {}
    for kind, n, d, s in (('iso', 48, 3, 2), ('ard', 64, 4, 8)):
        X, y = synth_data(n, d, 31 if kind == 'iso' else 32, kind)
        P = 2 if kind == 'iso' else d + 1
        prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
        est = ref_est.LogMarginalLikelihoodApproxPosteriorISEstimator(
            X, y, kfunc(kind, 1e-8), ref_lpa.laplace_approximation)

        def log_f_estimator(u, theta=None, cached_res=None):
            val, new_cache = est(u, theta, cached_res)
            lp = ref_utils.log_gamma_log_pdf(theta[0], prior['a_sigma'], prior['b_sigma'])
            for k in range(1, P):
                lp += ref_utils.log_gamma_log_pdf(theta[k], prior['a_tau'], prior['b_tau'])
            return val + lp, new_cache

        prng = np.random.RandomState(1234)

        def dir_w():
            dd = prng.normal(size=P)
            dd /= dd.dot(dd) ** 0.5
            return dd, 1.

        smp = ref_smp.APMEllSSPlusRandDirSliceSampler(
            log_f_estimator, lambda: prng.normal(size=(n, s)), prng, dir_w, 0)
        prng.seed(77)
        theta_init = np.r_[np.log(prng.gamma(prior['a_sigma'], 1. / prior['b_sigma'])),
                           np.log(prng.gamma(prior['a_tau'], 1. / prior['b_tau'], size=P - 1))]
        est.reset_cubic_op_count()
        th = smp.get_samples(theta_init, 12)
        out[kind + '_X'] = X
        out[kind + '_y'] = y
        out[kind + '_thetas'] = th
        out[kind + '_theta_init'] = theta_init
        out[kind + '_n_cubic_ops'] = est.n_cubic_ops
        out[kind + '_s'] = s
    np.savez_compressed(os.path.join(HERE, 'gp_chain.npz'), **out)


def pmmh_chain_fixture():
    """BASELINE.json configs[0]: the PM-MH protocol of Pseudo-Marginal MH.ipynb (cells 12-14):
    isotropic SE kernel, N_imp = 1, Laplace-estimator adaptive phase, then the ApproxPosteriorIS
    main phase with fresh u from the shared prng at every proposal. Pima-shaped synthetic data
    (N=768, D=8; the UCI file is not available), a shortened schedule (3 adaptive batches of 10,
    30 main iterations). Records every estimator value in call order so the GPU replay can be
    checked call by call."""
    n, d, n_imp = 768, 8, 1
    X, y = synth_data(n, d, 20151009, 'iso')
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    kf = kfunc('iso', 1e-8)
    prng = np.random.RandomState()
    det = ref_est.LogMarginalLikelihoodLaplaceEstimator(X, y, kf)
    imp = ref_est.LogMarginalLikelihoodApproxPosteriorISEstimator(
        X, y, kf, ref_lpa.laplace_approximation)
    calls = []

    def lp(theta):
        return (ref_utils.log_gamma_log_pdf(theta[0], prior['a_sigma'], prior['b_sigma']) +
                ref_utils.log_gamma_log_pdf(theta[1], prior['a_tau'], prior['b_tau']))

    def log_f_adapt(theta):
        v = det(theta)
        calls.append(v)
        return v + lp(theta)

    def log_f_main(theta):
        v = imp(prng.normal(size=(y.shape[0], n_imp)), theta)[0]
        calls.append(v)
        return v + lp(theta)

    def prop_sampler(theta, s):
        return np.r_[theta[0] + s[0] * prng.normal(), theta[1] + s[1] * prng.normal()]

    def log_prop_density(tp, tc, s):
        return -0.5 * (((tp[0] - tc[0]) / s[0]) ** 2 + ((tp[1] - tc[1]) / s[1]) ** 2)

    init_scales = np.array([0.5, 0.5])
    sampler = ref_smp.PMMHSampler(log_f_adapt, log_prop_density, prop_sampler, init_scales, prng)
    prng.seed(4321)
    theta_init = np.array([np.log(prng.gamma(prior['a_sigma'], 1. / prior['b_sigma'])),
                           np.log(prng.gamma(prior['a_tau'], 1. / prior['b_tau']))])
    ath, aps, aar = sampler.adaptive_run(theta_init, 10, 3, 0.15, 0.30,
                                         ref_utils.adapt_factor_func, False)
    n_adapt_calls = len(calls)
    sampler.log_f_estimator = log_f_main
    imp.reset_cubic_op_count()
    thetas, n_reject = sampler.get_samples(ath[-1], 30)
    np.savez_compressed(os.path.join(HERE, 'pmmh_chain.npz'), X=X, y=y, theta_init=theta_init,
                        adapt_thetas=ath, adapt_scales=aps, adapt_rates=aar, thetas=thetas,
                        n_reject=n_reject, n_cubic_ops=imp.n_cubic_ops, calls=np.array(calls),
                        n_adapt_calls=n_adapt_calls, seed=4321, det_ops=det.n_cubic_ops)


def utils_fixture():
    x = np.linspace(-3, 3, 13)
    out = dict(x=x, lgl=ref_utils.log_gamma_log_pdf(x, 1.1, 0.1),
               gl=ref_utils.gamma_log_pdf(np.exp(x), 1.1, 0.1),
               adapt=np.array([ref_utils.adapt_factor_func(b, 20) for b in range(25)]))
    Xr = np.random.RandomState(3).normal(loc=2., scale=3., size=(17, 4))
    Xn, mn, sd = ref_utils.normalise_inputs(Xr)
    out.update(Xraw=Xr, Xn=Xn, mn=mn, sd=sd)
    np.savez_compressed(os.path.join(HERE, 'utils.npz'), **out)


if __name__ == '__main__':
    np.seterr(all='ignore')
    gram_fixture()
    estimator_fixture()
    error_fixture()
    sampler_fixture()
    gp_chain_fixture()
    utils_fixture()
    pmmh_chain_fixture()
    for f in sorted(glob.glob(os.path.join(HERE, '*.npz'))):
        print(os.path.basename(f), os.path.getsize(f))

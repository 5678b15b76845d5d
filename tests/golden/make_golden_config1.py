"""BASELINE.json configs[1] chain fixture made by running the REFERENCE (build container only):
APMEllSSPlusMHSampler (auxpm/samplers.py:421-585) over the reference IS estimator
(gpdemo/estimators.py:152-241, gpdemo/kernels.pyx Gram, latent_posterior_approximations.py
Laplace), with the notebooks' closure (estimator + log-Gamma priors, E-SS+RD-SS.ipynb:167-173)
and exactly the wiring, data and seeds of tests/test_gpu_chains.py::
test_config1_ess_mh_chain_matches_oracle: Pima-shaped synthetic N=768, D=8 (the repo's
gpdemo.utils.synthetic_gp_data(768, 8, 1), pinned by a SHA-256 of X), ARD-SE, N_imp=64,
Gaussian random-walk MH with scales 0.05 and its log density, one RandomState(4321) for u,
proposals and accept draws, 8 samples from theta_init = (0, log sqrt(D), ...).

    python tests/golden/make_golden_config1.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE]

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402  (reference imports + adaptations)
from make_golden_fullsize import repo_data, x_digest  # noqa: E402


def main():
    n, d, s, n_sample = 768, 8, 64, 8
    X, y = repo_data('synthetic_gp_data', n, d, 1)
    P = d + 1
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    est = mg.ref_est.LogMarginalLikelihoodApproxPosteriorISEstimator(
        X, y, mg.kfunc('ard', 1e-8), mg.ref_lpa.laplace_approximation)

    def log_f_estimator(u, theta=None, cached_res=None):
        val, new_cache = est(u, theta, cached_res)
        lp = mg.ref_utils.log_gamma_log_pdf(theta[0], prior['a_sigma'], prior['b_sigma'])
        for k in range(1, P):
            lp += mg.ref_utils.log_gamma_log_pdf(theta[k], prior['a_tau'], prior['b_tau'])
        return val + lp, new_cache

    theta_init = np.r_[0.0, np.full(d, np.log(np.sqrt(d)))]
    prng = np.random.RandomState(4321)
    sampler = mg.ref_smp.APMEllSSPlusMHSampler(
        log_f_estimator, lambda xp, xc, sc: -0.5 * np.sum(((xp - xc) / sc) ** 2),
        lambda x, sc: x + sc * prng.normal(size=x.shape), np.full(P, 0.05),
        lambda: prng.normal(size=(n, s)), prng)
    est.reset_cubic_op_count()
    th, n_reject = sampler.get_samples(theta_init, n_sample)
    np.savez_compressed(os.path.join(HERE, 'config1_ref.npz'), thetas=th, n_reject=n_reject,
                        n_cubic_ops=est.n_cubic_ops, y=y, x_sha256=x_digest(X),
                        theta_init=theta_init)
    print('config1_ref.npz', th[-1], n_reject, est.n_cubic_ops)


if __name__ == '__main__':
    np.seterr(all='ignore')
    main()

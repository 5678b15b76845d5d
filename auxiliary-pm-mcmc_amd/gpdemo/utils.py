# -*- coding: utf-8 -*-
"""Host helpers of the experiments: log-Gamma priors, the adaptive-MH schedule, input
standardisation, synthetic data and the run-output format (reference gpdemo/utils.py)."""
import datetime
import json
import os

import numpy as np
from scipy.special import gammaln

__all__ = ['gamma_log_pdf', 'log_gamma_log_pdf', 'adapt_factor_func', 'normalise_inputs',
           'save_run', 'save_adaptive_run', 'plot_trace', 'log_prior_ard', 'log_prior_ard_batch',
           'synthetic_gp_data', 'load_uci_data']


def gamma_log_pdf(x, a, b):
    """log Gamma(x; shape a, rate b) (reference utils.py:19-36)."""
    return a * np.log(b) - gammaln(a) + (a - 1) * np.log(x) - b * x


def log_gamma_log_pdf(x, a, b):
    """Log density of x when exp(x) ~ Gamma(a, rate b) (reference utils.py:39-59)."""
    return a * np.log(b) - gammaln(a) + a * x - b * np.exp(x)


def adapt_factor_func(b, n_batch):
    """Adaptive-MH scale factor for batch b (Filippone & Girolami 2013; reference :62-83)."""
    return 5. - min(b + 1, n_batch / 5.) / (n_batch / 5.) * 3.9


def normalise_inputs(X):
    """Zero-mean, unit-sd features; returns (X_normalised, mean, sd) (reference :86-105)."""
    X_mn = X.mean(0)
    X_sd = X.std(0)
    return (X - X_mn[None]) / X_sd[None], X_mn, X_sd


def log_prior_ard(theta, prior):
    """Log-Gamma prior of the notebook closures (e.g. E-SS+RD-SS.ipynb:167-173) on
    theta[0] = log sigma (a_sigma, b_sigma) and every theta[k>=1] = log tau_k (a_tau, b_tau).
    The notebooks use the isotropic kernel (theta of length 2); for ARD the tau prior is
    applied to every length-scale (a build decision)."""
    lp = log_gamma_log_pdf(theta[0], prior['a_sigma'], prior['b_sigma'])
    for k in range(1, len(theta)):
        lp += log_gamma_log_pdf(theta[k], prior['a_tau'], prior['b_tau'])
    return lp


def load_uci_data(data_set, data_dir=None, normalise=True):
    """Load `<data_dir>/<data_set>_X.txt` and `_y.txt` the way every experiment notebook does
    (e.g. E-SS+RD-SS.ipynb cells at :85-87: np.genfromtxt, then normalise_inputs on X).
    `data_dir` defaults to $DATA_DIR/uci (notebook :39). Returns (X, y) or, with
    normalise=True, (X_normalised, y, X_mn, X_sd). Labels must be +-1 (probit likelihood);
    a ValueError names the offending file otherwise."""
    if data_dir is None:
        data_dir = os.path.join(os.environ['DATA_DIR'], 'uci')
    x_path = os.path.join(data_dir, data_set + '_X.txt')
    y_path = os.path.join(data_dir, data_set + '_y.txt')
    X = np.genfromtxt(x_path)
    y = np.genfromtxt(y_path)
    if X.ndim == 1:
        X = X[:, None]
    if y.ndim != 1 or y.shape[0] != X.shape[0]:
        raise ValueError('{0}: {1} labels for {2} inputs'.format(y_path, y.size, X.shape[0]))
    if not np.all((y == 1.) | (y == -1.)):
        raise ValueError('{0}: labels must be +1/-1'.format(y_path))
    if not normalise:
        return X, y
    X, X_mn, X_sd = normalise_inputs(X)
    return X, y, X_mn, X_sd


def log_prior_ard_batch(thetas, prior):
    """log_prior_ard of every row of `thetas` (chains x P) at once: the same terms, summed in
    the same order (theta[0] term, then += each length-scale term), vectorised over chains so a
    64-chain batch costs microseconds of host time instead of milliseconds."""
    th = np.atleast_2d(np.asarray(thetas, dtype=np.float64))
    lp = log_gamma_log_pdf(th[:, 0], prior['a_sigma'], prior['b_sigma'])
    if th.shape[1] > 1:
        terms = log_gamma_log_pdf(th[:, 1:], prior['a_tau'], prior['b_tau'])
        for k in range(terms.shape[1]):
            lp = lp + terms[:, k]
    return lp


def synthetic_gp_data(n, d, seed, kind='ard', jitter=1e-6):
    """Synthetic probit GP-classification data: X ~ N(0,1) then normalised;
    y = sign(f*) with f* a GP prior draw at log sigma = 0, log tau_k = log sqrt(d). The prior
    draw uses the numpy Cholesky on the host (data preparation, not the hot path)."""
    rng = np.random.RandomState(seed)
    X, _, _ = normalise_inputs(rng.normal(size=(n, d)))
    tau = np.sqrt(d)
    s = np.zeros((n, n))
    for k in range(d):
        diff = (X[:, k][:, None] - X[:, k][None, :]) / tau
        s += diff ** 2
    K = np.exp(-0.5 * s) + jitter * np.eye(n)
    f = np.linalg.cholesky(K).dot(rng.normal(size=n))
    y = np.where(f >= 0, 1., -1.)
    return X, y


def _perf_stats(n_reject, n_cubic_ops, comp_time):
    if hasattr(n_reject, '__len__'):
        return np.array([n for n in n_reject] + [n_cubic_ops, comp_time])
    return np.array([n_reject, n_cubic_ops, comp_time])


def _paths(output_dir, tag):
    stamp = datetime.datetime.now().strftime('%Y_%m_%d_%H_%M_%S_')
    return (os.path.join(output_dir, stamp + tag + '_results.npz'),
            os.path.join(output_dir, stamp + tag + '_params.json'))


def save_run(output_dir, tag, thetas, n_reject, n_cubic_ops, comp_time, run_params):
    """``<stamp><tag>_results.npz`` (thetas, n_reject_n_cubic_ops_comp_time) plus
    ``<stamp><tag>_params.json`` — the reference's output schema (utils.py:108-149)."""
    res, par = _paths(output_dir, tag)
    np.savez(res, thetas=thetas,
             n_reject_n_cubic_ops_comp_time=_perf_stats(n_reject, n_cubic_ops, comp_time))
    with open(par, 'w') as f:
        json.dump(run_params, f, indent=4, sort_keys=True)
    return res, par


def save_adaptive_run(output_dir, tag, adapt_thetas, adapt_prop_scales, adapt_accept_rates,
                      thetas, n_reject, n_cubic_ops, comp_time, run_params):
    """As :func:`save_run` plus the adaptive-phase arrays (reference utils.py:152-208)."""
    res, par = _paths(output_dir, tag)
    np.savez(res, adapt_thetas=adapt_thetas, adapt_prop_scales=adapt_prop_scales,
             adapt_accept_rates=adapt_accept_rates, thetas=thetas,
             n_reject_n_cubic_ops_comp_time=_perf_stats(n_reject, n_cubic_ops, comp_time))
    with open(par, 'w') as f:
        json.dump(run_params, f, indent=4, sort_keys=True)
    return res, par


def plot_trace(thetas, fig_size=(12, 8)):
    """Trace plot of log sigma and log tau (reference utils.py:211-242): returns
    ``(fig, ax1, ax2)`` with ax1 the log-variance and ax2 the log-length-scale axes (for ARD
    thetas ax2 shows the first length-scale, as the reference plots column 1)."""
    import matplotlib.pyplot as plt
    fig = plt.figure(figsize=fig_size)
    ax1 = fig.add_subplot(211)
    ax1.plot(thetas[:, 0])
    ax1.set_xlabel('Number of updates', fontsize=12)
    ax1.set_ylabel(r'$\log\,\sigma$', fontsize=18)
    ax2 = fig.add_subplot(212)
    ax2.plot(thetas[:, 1])
    ax2.set_xlabel('Number of updates', fontsize=12)
    ax2.set_ylabel(r'$\log\,\tau$', fontsize=18)
    return fig, ax1, ax2

# -*- coding: utf-8 -*-
"""Chain diagnostics used to report ESS/s on theta.

The reference's analysis (experiment_notebooks/Analyse results.ipynb:138-141) calls R's
``coda::effectiveSize`` and ``coda::gelman.diag``; R is not available, so both are restated
here from coda's published definitions (coda 0.19):

* ``effectiveSize(x) = n var(x) / spectrum0.ar(x)``, where ``spectrum0.ar`` fits an AR(p) model
  by Yule-Walker (``ar(x, aic=TRUE)``: order.max = min(n-1, floor(10 log10 n)), AIC order
  selection, var.pred rescaled by n / (n - (p+1))) and returns var.pred / (1 - sum(phi))^2;
  a series with zero residual sd about a linear trend gets spectrum 0 and ESS 0.
* ``gelman.diag`` point estimate (no autoburnin, no transform) of the potential scale
  reduction factor with the (df+3)/(df+1) correction.

No R fixture exists in the reference or here: these restatements are "parity unpinned"
against coda and are checked against closed-form AR(1) behaviour in tests/test_diagnostics.py.
"""
import numpy as np

__all__ = ['ar_yule_walker', 'spectrum0_ar', 'effective_size', 'gelman_rubin']


def ar_yule_walker(x, order_max=None):
    """R ``ar.yw`` (univariate, demean=TRUE, aic=TRUE): returns (coefs, var_pred, order)."""
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[0]
    if order_max is None:
        order_max = int(min(n - 1, np.floor(10 * np.log10(n))))
    xc = x - x.mean()
    r = np.array([xc[:n - k].dot(xc[k:]) / n for k in range(order_max + 1)])
    # Levinson-Durbin (R's eureka): prediction variances and coefficients for orders 1..p
    vars_ = np.empty(order_max)
    coefs = np.zeros((order_max, order_max))
    v = r[0]
    phi = np.zeros(0)
    for m in range(1, order_max + 1):
        k = (r[m] - phi.dot(r[m - 1:0:-1])) / v if m > 1 else r[1] / v
        phi = np.r_[phi - k * phi[::-1], k]
        v = v * (1 - k * k)
        coefs[m - 1, :m] = phi
        vars_[m - 1] = v
    var_pred = np.r_[r[0], vars_]
    with np.errstate(divide='ignore', invalid='ignore'):
        aic = n * np.log(var_pred) + 2 * np.arange(order_max + 1) + 2
    order = int(np.argmin(aic)) if np.isfinite(aic).any() else 0
    ar = coefs[order - 1, :order] if order else np.zeros(0)
    vp = var_pred[order] * n / (n - (order + 1))
    return ar, vp, order


def spectrum0_ar(x):
    """coda ``spectrum0.ar``: spectral density at frequency 0 of an AIC-selected AR fit."""
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[0]
    z = np.arange(1, n + 1, dtype=np.float64)
    A = np.stack([np.ones(n), z], 1)
    resid = x - A.dot(np.linalg.lstsq(A, x, rcond=None)[0])
    if np.allclose(resid.std(ddof=1), 0.0, atol=1.5e-8 * max(1.0, np.abs(x).max())):
        return 0.0, 0
    ar, vp, order = ar_yule_walker(x)
    return vp / (1. - ar.sum()) ** 2, order


def effective_size(x):
    """coda ``effectiveSize`` of each column of x (n_samples, n_dims) (or a 1-D chain)."""
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        x = x[:, None]
    out = np.empty(x.shape[1])
    for i in range(x.shape[1]):
        spec, _ = spectrum0_ar(x[:, i])
        out[i] = 0.0 if spec == 0 else x.shape[0] * x[:, i].var(ddof=1) / spec
    return out


def gelman_rubin(chains):
    """Potential scale reduction factor per dimension; chains: (m, n, d)."""
    ch = np.asarray(chains, dtype=np.float64)
    m, n = ch.shape[:2]
    means = ch.mean(1)
    W = ch.var(1, ddof=1).mean(0)
    B = n * means.var(0, ddof=1)
    var_plus = (n - 1) / n * W + B / n
    V = var_plus + B / (m * n)
    # degrees of freedom of V (Gelman & Rubin 1992), as in coda's gelman.diag
    s2 = ch.var(1, ddof=1)
    var_W = s2.var(0, ddof=1) / m
    var_B = 2 * B ** 2 / (m - 1)
    cov_WB = n / m * (np.array([np.cov(s2[:, k], means[:, k] ** 2)[0, 1] for k in range(ch.shape[2])])
                      - 2 * means.mean(0) * np.array([np.cov(s2[:, k], means[:, k])[0, 1]
                                                       for k in range(ch.shape[2])]))
    var_V = ((n - 1) / n) ** 2 * var_W + ((m + 1) / (m * n)) ** 2 * var_B + \
        2 * (m - 1) * (n - 1) / (m * n * n) * cov_WB
    df = 2 * V ** 2 / var_V
    return np.sqrt((df + 3) / (df + 1) * V / W)

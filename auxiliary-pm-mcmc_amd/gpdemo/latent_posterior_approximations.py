# -*- coding: utf-8 -*-
"""Laplace approximation of the latent posterior p(f | y, theta, X) for probit GP
classification, computed on the GPU (reference latent_posterior_approximations.py:22-124).

Same signature, return tuples, convergence rule (mean squared change of f below
``diff_f_tol``), iteration cap and exception as the reference. The covariance C and the LML
use the Newton quantities of the last iteration together with the updated f, as the
reference does (:107-110).
"""
import numpy as np

from . import _native

__all__ = ['MaximumIterationsExceededError', 'laplace_approximation']


class MaximumIterationsExceededError(Exception):
    """Raised when Newton's method fails to converge by the iteration limit."""


def laplace_approximation(K, y, calc_cov=True, calc_lml=False, diff_f_tol=1e-4, max_iters=1000):
    """Returns ``(f, C, lml, n_ops)``, ``(f, lml, n_ops)``, ``(f, C, n_ops)`` or ``(f, n_ops)``
    depending on the flags, with ``n_ops`` the reference's count of O(N^3) operations."""
    f, C, lml, n_iter, status = _native.laplace(K, y, calc_cov, calc_lml, diff_f_tol, max_iters)
    if status == _native.STATUS_MAXITER:
        raise MaximumIterationsExceededError(
            'Failed to converge in {0} iterations'.format(n_iter))
    if status != _native.STATUS_OK:
        raise np.linalg.LinAlgError('Cholesky factorisation of B failed (not positive definite)')
    if calc_cov and calc_lml:
        return f, C, lml, n_iter + 1
    if calc_lml:
        return f, lml, n_iter
    if calc_cov:
        return f, C, n_iter + 1
    return f, n_iter


# the estimators run this approximation fused on the device when they are handed this function
laplace_approximation.apm_fused = True

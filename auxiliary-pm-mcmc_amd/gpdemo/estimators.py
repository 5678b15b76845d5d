# -*- coding: utf-8 -*-
"""Estimators of log p(y | theta, X) for probit GP classification, evaluated on the MI355X.

Drop-in for the reference's ``gpdemo/estimators.py``: the three classes keep their constructor
arguments, ``__call__`` signatures, return values, ``n_cubic_ops`` accounting and exceptions.
The work runs in libapm.so (include/apm.h) in fp64 (Gram, Newton/Laplace, Cholesky factors)
with the importance-sampling product L.U in fp32 MFMA.

``cached_results`` / ``K_chol`` become :class:`DeviceCache` handles: opaque references to a
device-resident cache slot that is released when the handle is garbage-collected. Passing one
back skips the O(N^3) work exactly as the reference's tuple does.
"""
import numpy as np

from . import _native
from .latent_posterior_approximations import MaximumIterationsExceededError

__all__ = ['LogMarginalLikelihoodLaplaceEstimator', 'InvalidCovarianceMatrixError',
           'LogMarginalLikelihoodApproxPosteriorISEstimator',
           'LogMarginalLikelihoodPriorMCEstimator', 'DeviceCache', 'DeviceInvariantError']

_UBUF = 0  # single-chain estimators upload each call's draws into this device buffer


class InvalidCovarianceMatrixError(Exception):
    """Raised when the posterior approximation's covariance is not positive definite."""


class DeviceInvariantError(RuntimeError):
    """A device-side invariant of the theta-call failed (APM_STATUS_GUARD): the
    estimate is withheld rather than returned. No reference counterpart (the reference has no
    device); a sampler treats it like any other failed estimator call."""


class DeviceCache(object):
    """Handle to the per-theta state kept on the device (replaces the reference's
    ``(K_chol, C_chol, f_post)`` tuple / ``K_chol`` array). Iterating an IS cache reads the
    state back as that tuple (reference estimators.py:166-176) for inspection; the samplers only
    pass the handle back. The slot keeps C_chol and f_post; L_K = chol(K) is consumed by the
    posterior factor on the device, so iterating refactors K on the device
    (a PriorMC theta-call into a scratch slot) — all three factors are read back rounded to fp32
    like the slot itself. That refactor runs once per handle (memoised): an O(N^3) device call,
    so unpacking the tuple is not free the first time. ``numpy.asarray`` is defined for a PriorMC
    handle only (the reference's K_chol array); an IS handle is a tuple, not an array."""

    __slots__ = ('_ctx', 'slot', 'kind', '_owner', '_theta', '_kchol', '__weakref__')

    def __init__(self, ctx, slot, kind, owner=None, theta=None):
        self._ctx = ctx
        self.slot = slot
        self.kind = kind
        self._owner = owner  # the estimator (its kernel_func / X) for the K_chol refactor
        self._theta = None if theta is None else np.array(theta, dtype=np.float64)
        self._kchol = None

    def __del__(self):
        try:
            self._ctx.slots.release(self.slot)
        except Exception:
            pass

    def read(self):
        """(factor (n, n) lower, f_post (n,), g (n,), const) — factor rounded to fp32."""
        return self._ctx.slot_read(self.slot)

    def k_chol(self):
        """chol(K(theta)) (n, n) lower, computed on the device (fp32-rounded read-back)."""
        if self.kind == _native.EST_PRIORMC:
            return self.read()[0]
        if self._kchol is not None:  # a fresh array per call, as the reference's tuple element
            return self._kchol.copy()
        if self._owner is None or self._theta is None:
            raise ValueError('this cache does not record its theta')
        tmp = self._ctx.slots.acquire()
        try:
            _, st, _ = self._owner._theta_call(_native.EST_PRIORMC, self._ctx, self._theta,
                                               _UBUF, tmp)
            _raise_for_status(int(st[0]), self._ctx)
            self._kchol = self._ctx.slot_read(tmp)[0]
            return self._kchol.copy()
        finally:
            self._ctx.slots.release(tmp)

    def __iter__(self):
        L, f, _, _ = self.read()
        if self.kind == _native.EST_PRIORMC:  # the reference's K_chol is the array itself
            return iter(L)
        return iter((self.k_chol(), L, f))

    def __array__(self, dtype=None, copy=None):
        if self.kind != _native.EST_PRIORMC:
            raise TypeError('an importance-sampling cache is the tuple (K_chol, C_chol, f_post), '
                            'not an array: unpack it')
        L = self.read()[0]
        return L if dtype is None else L.astype(dtype)


def _kernel_spec(kernel_func):
    kind = getattr(kernel_func, 'native_kind', None)
    if kind is None:
        return _native.KERNEL_PRECOMPUTED, 1e-8
    return kind, getattr(kernel_func, 'epsilon', 1e-8)


def _raise_for_status(status, ctx, n_iter_cap=1000):
    if status == _native.STATUS_OK:
        return
    if status == _native.STATUS_CHOL_C:
        raise InvalidCovarianceMatrixError(
            'Posterior covariance matrix not PSD: sum of negative eigenvalues nan '
            '(Cholesky of C failed on the device)')
    if status == _native.STATUS_GUARD:
        raise DeviceInvariantError('a device-side invariant of the theta-call failed '
                                   '(apm_guard_read gives the residuals)')
    if status == _native.STATUS_MAXITER:
        raise MaximumIterationsExceededError('Failed to converge in {0} iterations'
                                             .format(n_iter_cap))
    what = 'K' if status == _native.STATUS_CHOL_K else 'B'
    raise np.linalg.LinAlgError('{0}-th leading minor not positive definite (Cholesky of {1} '
                                'on the device)'.format('?', what))


class _Problem(object):
    """Device contexts for one (X, y, kernel) problem, created lazily per number of draws."""

    def __init__(self, X, y, kernel_func, n_slots=8):
        self.X = X
        self.y = np.asarray(y, dtype=np.float64)
        self.kind, self.eps = _kernel_spec(kernel_func)
        self.n_slots = n_slots
        self._ctxs = {}

    @property
    def device_gram(self):
        return self.kind != _native.KERNEL_PRECOMPUTED

    def ctx(self, n_imp):
        c = self._ctxs.get(n_imp)
        if c is None:
            c = _native.Context(self.X, self.y, self.kind, self.eps, n_imp, max_batch=1,
                                n_slots=self.n_slots, n_ubufs=1)
            self._ctxs[n_imp] = c
        return c


class _EstimatorBase(object):
    def __init__(self, X, y, kernel_func):
        self.X = X
        self.y = y
        self.kernel_func = kernel_func
        self._prob = _Problem(X, y, kernel_func)
        self._K = None if self._prob.device_gram else np.empty((X.shape[0], X.shape[0]))
        self.n_cubic_ops = 0
        _native.load_library()  # fail loudly here, not at the first call

    def reset_cubic_op_count(self):
        """Reset the count of executed ops with order ``n_data**3`` cost."""
        self.n_cubic_ops = 0

    def _theta_call(self, est, ctx, theta, ubuf, slot):
        if self._prob.device_gram:
            return ctx.theta_eval(est, np.atleast_1d(theta)[None], [ubuf], [slot])
        self.kernel_func(self._K, self.X, theta)
        return ctx.theta_eval_K(est, self._K, ubuf, slot)


class LogMarginalLikelihoodLaplaceEstimator(_EstimatorBase):
    """Deterministic (biased) Laplace-approximation estimate of log p(y | theta, X)
    (reference estimators.py:19-82)."""

    def __call__(self, theta):
        ctx = self._prob.ctx(1)
        out, st, nops = self._theta_call(_native.EST_LAPLACE, ctx, theta, _UBUF, 0)
        _raise_for_status(int(st[0]), ctx)
        self.n_cubic_ops += int(nops[0])
        return float(out[0])


class LogMarginalLikelihoodApproxPosteriorISEstimator(_EstimatorBase):
    """Unbiased importance-sampling estimate of p(y | theta, X) with the Laplace posterior as
    proposal (reference estimators.py:90-241). ``ns``: (n_data, n_imp_sample) N(0,1) draws."""

    def __init__(self, X, y, kernel_func, post_approx_func):
        if not (getattr(post_approx_func, 'apm_fused', False) or
                getattr(post_approx_func, '__name__', '') == 'laplace_approximation'):
            raise NotImplementedError(
                'the device estimator fuses the Laplace approximation '
                '(gpdemo.latent_posterior_approximations.laplace_approximation); got {0!r}'
                .format(post_approx_func))
        super(LogMarginalLikelihoodApproxPosteriorISEstimator, self).__init__(X, y, kernel_func)
        self.post_approx_func = post_approx_func

    def __call__(self, ns, theta=None, cached_results=None):
        if theta is None and cached_results is None:
            raise ValueError('One of theta or cached_results must be provided')
        ns = np.asarray(ns, dtype=np.float64)
        if cached_results is None:
            ctx = self._prob.ctx(ns.shape[1])
            ctx.u_upload(_UBUF, ns)
            slot = ctx.slots.acquire()
            cache = DeviceCache(ctx, slot, _native.EST_IS, self, theta)
            out, st, nops = self._theta_call(_native.EST_IS, ctx, theta, _UBUF, slot)
            _raise_for_status(int(st[0]), ctx)
            self.n_cubic_ops += int(nops[0])
            return float(out[0]), cache
        ctx = cached_results._ctx
        if ns.shape[1] != ctx.n_imp:
            raise ValueError('cached results were computed for {0} importance samples, got {1}'
                             .format(ctx.n_imp, ns.shape[1]))
        ctx.u_upload(_UBUF, ns)
        out, st = ctx.u_eval([cached_results.slot], [_UBUF])
        _raise_for_status(int(st[0]), ctx)
        return float(out[0]), cached_results


class LogMarginalLikelihoodPriorMCEstimator(_EstimatorBase):
    """Unbiased simple Monte Carlo estimate of p(y | theta, X) with draws from the GP prior
    (reference estimators.py:244-325). Returns ``(log_estimate, K_chol)``; ``K_chol`` is a
    :class:`DeviceCache`."""

    def __call__(self, ns, theta=None, K_chol=None):
        if theta is None and K_chol is None:
            raise ValueError('One of theta or K_chol must be provided')
        ns = np.asarray(ns, dtype=np.float64)
        if K_chol is None:
            ctx = self._prob.ctx(ns.shape[1])
            ctx.u_upload(_UBUF, ns)
            slot = ctx.slots.acquire()
            cache = DeviceCache(ctx, slot, _native.EST_PRIORMC, self, theta)
            out, st, nops = self._theta_call(_native.EST_PRIORMC, ctx, theta, _UBUF, slot)
            _raise_for_status(int(st[0]), ctx)
            self.n_cubic_ops += int(nops[0])
            return float(out[0]), cache
        ctx = K_chol._ctx
        ctx.u_upload(_UBUF, ns)
        out, st = ctx.u_eval([K_chol.slot], [_UBUF])
        _raise_for_status(int(st[0]), ctx)
        return float(out[0]), K_chol

# -*- coding: utf-8 -*-
"""Pseudo-marginal and auxiliary pseudo-marginal (APM) samplers — host-side drivers.

Same classes, constructor/method signatures, return types and RNG consumption order as the
reference's ``auxpm/samplers.py`` so that existing experiment code runs unchanged; the
``log_f_estimator`` they call is where the GPU work happens (``gpdemo.estimators``).

Estimator protocol (reference samplers.py:279-297):
    PM-MH:  ``log_f = log_f_estimator(theta)``
    APM:    ``log_f, cached = log_f_estimator(u, theta[, cached])`` — ``cached`` is the opaque
            per-theta state; passing it back makes the call an O(N^2 S) u-call.

Cache protocol kept verbatim (reference :557-584, :994-1001, :1079-1086, :1154-1161): u-updates
reuse the current cache; MH theta-updates promote the proposal's cache on accept; slice
theta-updates overwrite the current cache on every estimator call (the last call of a slice
step is the accepted point).
"""
import numpy as np

from . import mcmc_updates as mcmc


def _theta_array(theta_init, n_sample, column=False):
    if hasattr(theta_init, 'shape'):
        return np.empty((n_sample, theta_init.shape[0]))
    return np.empty((n_sample, 1)) if column else np.empty(n_sample)


class BaseAdaptiveMHSampler(object):
    """MH-type sampler with batch-wise proposal-scale adaptation (reference samplers.py:14-156)."""

    def __init__(self, prop_scales):
        self.prop_scales = prop_scales

    def get_samples(self, theta_init, n_sample):
        raise NotImplementedError()

    def adaptive_run(self, theta_init, batch_size, n_batch, low_acc_thr, upp_acc_thr,
                     adapt_factor_func, print_details=False, reject_count_index=-1):
        """Run ``n_batch`` batches, dividing / multiplying ``self.prop_scales`` (in place, as the
        reference does) by ``adapt_factor_func(b, n_batch)`` when the batch accept rate falls
        below / above the thresholds. With several rejection counts, the one at
        ``reject_count_index`` drives adaptation (a zero index is ignored: reference :143).

        Returns ``(thetas, prop_scales_per_batch, accept_rates)``.
        """
        thetas = np.empty((n_batch * batch_size, theta_init.shape[0]))
        scales = np.empty((n_batch, self.prop_scales.shape[0]))
        rates = np.empty(n_batch)
        for b in range(n_batch):
            lo, hi = b * batch_size, (b + 1) * batch_size
            thetas[lo:hi], n_reject = self.get_samples(theta_init, batch_size)
            if hasattr(n_reject, '__len__') and reject_count_index:
                n_reject = n_reject[reject_count_index]
            rates[b] = 1. - (n_reject * 1. / batch_size)
            theta_init = thetas[hi - 1]
            factor = adapt_factor_func(b, n_batch)
            if rates[b] < low_acc_thr:
                self.prop_scales /= factor
            elif rates[b] > upp_acc_thr:
                self.prop_scales *= factor
            scales[b] = self.prop_scales
            if print_details:
                print('Batch {0}: accept rate {1}, adapt factor {2}'.format(b + 1, rates[b], factor))
        return thetas, scales, rates


class PMMHSampler(BaseAdaptiveMHSampler):
    """Standard pseudo-marginal Metropolis(-Hastings) (reference samplers.py:159-262).

    A fresh estimate is drawn at every proposal (``log_f_estimator(theta)``); the current
    state's estimate is recycled, as pseudo-marginal MH requires.
    """

    def __init__(self, log_f_estimator, log_prop_density, prop_sampler, prop_scales, prng):
        super(PMMHSampler, self).__init__(prop_scales)
        self.log_f_estimator = log_f_estimator
        self.do_metropolis_update = log_prop_density is None
        if not self.do_metropolis_update:
            self.log_prop_density = log_prop_density
        self.prop_sampler = prop_sampler
        self.prng = prng

    def get_samples(self, theta_init, n_sample):
        """Returns ``(thetas, n_reject)``."""
        thetas = _theta_array(theta_init, n_sample)
        thetas[0] = theta_init
        log_f = self.log_f_estimator(theta_init)
        n_reject = 0
        for s in range(1, n_sample):
            if self.do_metropolis_update:
                thetas[s], log_f, rej = mcmc.metropolis_step(
                    thetas[s - 1], log_f, self.log_f_estimator, self.prng, self.prop_sampler,
                    self.prop_scales)
            else:
                thetas[s], log_f, rej = mcmc.met_hastings_step(
                    thetas[s - 1], log_f, self.log_f_estimator, self.prng, self.prop_sampler,
                    self.prop_scales, self.log_prop_density)
            n_reject += bool(rej)
        return thetas, n_reject


class _APMMHMixin(object):
    """theta | u Metropolis(-Hastings) step shared by the two APM+MH samplers."""

    def _mh_theta(self, theta, log_f, u):
        holder = {}

        def log_f_theta(th):
            val, holder['cache'] = self.log_f_estimator(u, th)
            return val

        if self.do_metropolis_update:
            th, lf, rej = mcmc.metropolis_step(theta, log_f, log_f_theta, self.prng,
                                               self.prop_sampler, self.prop_scales)
        else:
            th, lf, rej = mcmc.met_hastings_step(theta, log_f, log_f_theta, self.prng,
                                                 self.prop_sampler, self.prop_scales,
                                                 self.log_prop_density)
        self._cached_res_prop = holder.get('cache')
        return th, lf, rej


class APMMetIndPlusMHSampler(_APMMHMixin, BaseAdaptiveMHSampler):
    """APM: Metropolis-independence on u, Metropolis(-Hastings) on theta (reference :265-418)."""

    def __init__(self, log_f_estimator, log_prop_density, prop_sampler, prop_scales, u_sampler,
                 prng):
        super(APMMetIndPlusMHSampler, self).__init__(prop_scales)
        self.log_f_estimator = log_f_estimator
        self.do_metropolis_update = log_prop_density is None
        if not self.do_metropolis_update:
            self.log_prop_density = log_prop_density
        self.prop_sampler = prop_sampler
        self.prop_scales = prop_scales
        self.u_sampler = u_sampler
        self.prng = prng

    def get_samples(self, theta_init, n_sample, u_init=None):
        """Returns ``(thetas, (n_reject_u, n_reject_theta))``."""
        thetas = _theta_array(theta_init, n_sample)
        thetas[0] = theta_init
        u = u_init if u_init is not None else self.u_sampler()
        log_f, cache = self.log_f_estimator(u, theta_init)
        n_rej_u = n_rej_th = 0
        for s in range(1, n_sample):
            th_prev = thetas[s - 1]
            u, log_f, rej = mcmc.metropolis_indepedence_step(
                u, log_f, lambda v: self.log_f_estimator(v, th_prev, cache)[0], self.prng,
                self.u_sampler)
            n_rej_u += bool(rej)
            thetas[s], log_f, rej = self._mh_theta(th_prev, log_f, u)
            if rej:
                n_rej_th += 1
            else:
                cache = self._cached_res_prop
        return thetas, (n_rej_u, n_rej_th)


class APMEllSSPlusMHSampler(_APMMHMixin, BaseAdaptiveMHSampler):
    """APM: elliptical slice sampling on u, Metropolis(-Hastings) on theta (reference :421-585)."""

    def __init__(self, log_f_estimator, log_prop_density, prop_sampler, prop_scales, u_sampler,
                 prng, max_slice_iters=1000):
        super(APMEllSSPlusMHSampler, self).__init__(prop_scales)
        self.log_f_estimator = log_f_estimator
        self.do_metropolis_update = log_prop_density is None
        if not self.do_metropolis_update:
            self.log_prop_density = log_prop_density
        self.prop_sampler = prop_sampler
        self.prop_scales = prop_scales
        self.prng = prng
        self.u_sampler = u_sampler
        self.max_slice_iters = max_slice_iters

    def elliptical_slice_sample_u_given_theta(self, u, log_f_est, log_f_func):
        nu = self.u_sampler()
        return mcmc.elliptical_slice_step(u, log_f_est, log_f_func, self.prng, nu,
                                          self.max_slice_iters)

    def get_samples(self, theta_init, n_sample, u_init=None):
        """Returns ``(thetas, n_reject_theta)``."""
        thetas = _theta_array(theta_init, n_sample)
        thetas[0] = theta_init
        u = u_init if u_init is not None else self.u_sampler()
        log_f, self._cached_res_curr = self.log_f_estimator(u, theta_init)
        n_reject = 0
        for s in range(1, n_sample):
            th_prev = thetas[s - 1]
            u, log_f = self.elliptical_slice_sample_u_given_theta(
                u, log_f, lambda v: self.log_f_estimator(v, th_prev, self._cached_res_curr)[0])
            thetas[s], log_f, rej = self._mh_theta(th_prev, log_f, u)
            if rej:
                n_reject += 1
            else:
                self._cached_res_curr = self._cached_res_prop
        return thetas, n_reject


class _SliceBase(object):
    def __init__(self, log_f_estimator, u_sampler, prng, max_steps_out=0, max_slice_iters=1000):
        self.log_f_estimator = log_f_estimator
        self.u_sampler = u_sampler
        self.prng = prng
        self.max_steps_out = max_steps_out
        self.max_slice_iters = max_slice_iters

    def slice_step(self, x_curr, log_f_curr, log_f_func, w):
        return mcmc.linear_slice_step(x_curr, log_f_curr, log_f_func, w, self.prng,
                                      self.max_steps_out, self.max_slice_iters)

    def slice_sample_theta_given_u(self, theta, log_f_est, u):
        raise NotImplementedError()

    def slice_sample_theta_gvn_u(self, theta, log_f_est, u):
        return self.slice_sample_theta_given_u(theta, log_f_est, u)

    def _estimate_and_cache(self, u, theta):
        """Estimator call during a slice theta-update: the cache always follows the last call."""
        val, self._cached_res_curr = self.log_f_estimator(u, theta)
        return val


class BaseAPMMetIndPlusSliceSampler(_SliceBase):
    """APM: Metropolis-independence on u, slice sampling on theta (reference :588-710)."""

    def get_samples(self, theta_init, n_sample, u_init=None):
        """Returns ``(thetas, n_reject_u)``."""
        thetas = _theta_array(theta_init, n_sample, column=True)
        thetas[0] = theta_init
        u = u_init if u_init is not None else self.u_sampler()
        log_f, self._cached_res_curr = self.log_f_estimator(u, theta_init)
        n_reject = 0
        for s in range(1, n_sample):
            th_prev = thetas[s - 1]
            u, log_f, rej = mcmc.metropolis_indepedence_step(
                u, log_f, lambda v: self.log_f_estimator(v, th_prev, self._cached_res_curr)[0],
                self.prng, self.u_sampler)
            n_reject += bool(rej)
            thetas[s], log_f = self.slice_sample_theta_gvn_u(thetas[s - 1].copy(), log_f, u)
        return thetas, n_reject


class BaseAPMEllSSPlusSliceSampler(_SliceBase):
    """APM: elliptical slice sampling on u, slice sampling on theta (reference :713-841)."""

    def elliptical_slice_sample_u_given_theta(self, u, log_f_est, log_f_func):
        nu = self.u_sampler()
        return mcmc.elliptical_slice_step(u, log_f_est, log_f_func, self.prng, nu,
                                          self.max_slice_iters)

    def get_samples(self, theta_init, n_sample, u_init=None):
        """Returns ``thetas`` only (as the reference, :841)."""
        thetas = _theta_array(theta_init, n_sample, column=True)
        thetas[0] = theta_init
        u = u_init if u_init is not None else self.u_sampler()
        log_f, self._cached_res_curr = self.log_f_estimator(u, theta_init)
        for s in range(1, n_sample):
            th_prev = thetas[s - 1]
            u, log_f = self.elliptical_slice_sample_u_given_theta(
                u, log_f, lambda v: self.log_f_estimator(v, th_prev, self._cached_res_curr)[0])
            thetas[s], log_f = self.slice_sample_theta_gvn_u(thetas[s - 1].copy(), log_f, u)
        return thetas


class APMMetIndPlusSeqSliceSampler(BaseAPMMetIndPlusSliceSampler):
    """MI on u; axis-aligned (sequential) linear slice sampling on each theta_j (reference :844-923)."""

    def __init__(self, log_f_estimator, u_sampler, prng, ws, max_steps_out=0,
                 max_slice_iters=1000):
        super(APMMetIndPlusSeqSliceSampler, self).__init__(
            log_f_estimator, u_sampler, prng, max_steps_out, max_slice_iters)
        self.ws = ws

    def slice_sample_theta_given_u(self, theta, log_f_est, u):
        for j in range(len(theta)):
            def log_f_j(x, j=j):
                return self._estimate_and_cache(u, np.r_[theta[:j], x, theta[j + 1:]])
            theta[j], log_f_est = self.slice_step(theta[j], log_f_est, log_f_j, self.ws[j])
        return theta, log_f_est


class _RandDirMixin(object):
    def slice_sample_theta_given_u(self, theta, log_f_est, u):
        d, w = self.slc_dir_and_w_sampler()
        x, log_f_est = self.slice_step(
            0., log_f_est, lambda x: self._estimate_and_cache(u, theta + x * d), w)
        return theta + x * d, log_f_est


class APMMetIndPlusRandDirSliceSampler(_RandDirMixin, BaseAPMMetIndPlusSliceSampler):
    """MI on u; random-direction linear slice sampling on theta (reference :926-1004)."""

    def __init__(self, log_f_estimator, u_sampler, prng, slc_dir_and_w_sampler,
                 max_steps_out=0, max_slice_iters=1000):
        super(APMMetIndPlusRandDirSliceSampler, self).__init__(
            log_f_estimator, u_sampler, prng, max_steps_out, max_slice_iters)
        self.slc_dir_and_w_sampler = slc_dir_and_w_sampler


class APMEllSSPlusRandDirSliceSampler(_RandDirMixin, BaseAPMEllSSPlusSliceSampler):
    """E-SS on u; random-direction linear slice sampling on theta (reference :1007-1089).

    This is the north-star configuration (BASELINE.json configs 3/4).
    """

    def __init__(self, log_f_estimator, u_sampler, prng, slc_dir_and_w_sampler,
                 max_steps_out=0, max_slice_iters=1000):
        super(APMEllSSPlusRandDirSliceSampler, self).__init__(
            log_f_estimator, u_sampler, prng, max_steps_out, max_slice_iters)
        self.slc_dir_and_w_sampler = slc_dir_and_w_sampler


class APMEllSSPlusEllSSSampler(BaseAPMEllSSPlusSliceSampler):
    """E-SS on u and E-SS on theta under a Gaussian theta prior (reference :1092-1165)."""

    def __init__(self, log_f_estimator, u_sampler, theta_sampler, prng, max_slice_iters=1000):
        super(APMEllSSPlusEllSSSampler, self).__init__(
            log_f_estimator, u_sampler, prng, None, max_slice_iters)
        self.theta_sampler = theta_sampler

    def slice_sample_theta_given_u(self, theta, log_f_est, u):
        nu = self.theta_sampler()
        return mcmc.elliptical_slice_step(
            theta, log_f_est, lambda th: self._estimate_and_cache(u, th), self.prng, nu,
            self.max_slice_iters)

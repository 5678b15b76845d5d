# -*- coding: utf-8 -*-
"""Single-transition MCMC kernels (host side of the APM driver).

API- and RNG-order-compatible with the reference's ``auxpm/mcmc_updates.py``: the same
functions, signatures, return values, exceptions and — because trajectories must be
reproducible from a seeded ``numpy.random.RandomState`` — the same sequence of ``prng`` draws
and the same floating-point expressions. Each function cites the reference lines it follows.
The per-step cost lives entirely in ``log_f_func`` (the GPU estimator); these loops only decide.
"""
import warnings

import numpy as np

__all__ = ['metropolis_step', 'met_hastings_step', 'metropolis_indepedence_step',
           'MaximumIterationsExceededError', 'elliptical_slice_step', 'linear_slice_step']


def metropolis_step(x_curr, log_f_curr, log_f_func, prng, prop_sampler, prop_scales):
    """Metropolis update with a symmetric proposal (reference mcmc_updates.py:14-76).

    Returns ``(x_next, log_f_next, rejected)``; accepts iff ``U < exp(log f(x') - log f(x))``.
    """
    x_prop = prop_sampler(x_curr, prop_scales)
    log_f_prop = log_f_func(x_prop)
    if prng.uniform() < np.exp(log_f_prop - log_f_curr):
        return x_prop, log_f_prop, False
    return x_curr, log_f_curr, True


def met_hastings_step(x_curr, log_f_curr, log_f_func, prng, prop_sampler, prop_params,
                      log_prop_density):
    """Metropolis-Hastings update (reference mcmc_updates.py:79-156).

    ``log_prop_density(x_to, x_from, params)``; returns ``(x_next, log_f_next, rejected)``.
    """
    x_prop = prop_sampler(x_curr, prop_params)
    log_f_prop = log_f_func(x_prop)
    log_q_fwd = log_prop_density(x_prop, x_curr, prop_params)
    log_q_bwd = log_prop_density(x_curr, x_prop, prop_params)
    p_acc = np.exp(log_f_prop + log_q_bwd - log_f_curr - log_q_fwd)
    if prng.uniform() < p_acc:
        return x_prop, log_f_prop, False
    return x_curr, log_f_curr, True


def metropolis_indepedence_step(x_curr, log_f_curr, log_f_func, prng, prop_sampler,
                                prop_params=None, log_prop_density=None):
    """Metropolis independence update (reference mcmc_updates.py:159-303; name kept verbatim).

    Without ``log_prop_density`` the proposal is the 'prior' factor of the target and cancels
    (the APM u-update); with it the usual independence-sampler ratio is used. As in the
    reference, the parameter tests are truthiness tests (``if prop_params:``).
    """
    x_prop = prop_sampler(prop_params) if prop_params else prop_sampler()
    log_f_prop = log_f_func(x_prop)
    if log_prop_density:
        if prop_params:
            log_q_fwd = log_prop_density(x_prop, prop_params)
            log_q_bwd = log_prop_density(x_curr, prop_params)
        else:
            log_q_fwd = log_prop_density(x_prop)
            log_q_bwd = log_prop_density(x_curr)
        p_acc = np.exp(log_f_prop + log_q_bwd - log_f_curr - log_q_fwd)
    else:
        p_acc = np.exp(log_f_prop - log_f_curr)
    if prng.uniform() < p_acc:
        return x_prop, log_f_prop, False
    return x_curr, log_f_curr, True


class MaximumIterationsExceededError(Exception):
    """A slice-sampling loop ran past its iteration cap (reference mcmc_updates.py:306-308)."""


def elliptical_slice_step(x_curr, log_f_curr, log_f_func, prng, gaussian_sample,
                          max_slice_iters=1000):
    """Elliptical slice sampling update (Murray, Adams & MacKay 2010; reference :311-400).

    Draw order: log-height uniform, initial angle uniform, then one uniform per shrink.
    Returns ``(x_next, log_f_next)``.
    """
    log_y = log_f_curr + np.log(prng.uniform())
    phi = prng.uniform() * 2. * np.pi
    lo, hi = phi - 2. * np.pi, phi
    it = 0
    while it < max_slice_iters:
        x_prop = x_curr * np.cos(phi) + gaussian_sample * np.sin(phi)
        log_f_prop = log_f_func(x_prop)
        if log_f_prop > log_y:
            return x_prop, log_f_prop
        if phi < 0:
            lo = phi
        elif phi > 0:
            hi = phi
        else:
            warnings.warn('Slice collapsed to current value')
            return x_curr, log_f_curr
        phi = lo + prng.uniform() * (hi - lo)
        it += 1
    raise MaximumIterationsExceededError(
        'Exceed maximum slice iterations: '
        'i={0}, phi_min={1}, phi_max={2}, log_f_prop={3}, log_f_curr={4}'
        .format(it, lo, hi, log_f_prop, log_f_curr))


def linear_slice_step(x_curr, log_f_curr, log_f_func, slice_width, prng, max_steps_out=0,
                      max_slice_iters=1000):
    """Slice sampling along a line with optional stepping out (Neal 2003; reference :403-519).

    Draw order: log-height uniform, bracket-offset uniform, [step-split uniform if
    ``max_steps_out > 0``], then one uniform per shrink. Returns ``(x_next, log_f_next)``.
    """
    log_y = np.log(prng.uniform()) + log_f_curr
    x_lo = x_curr - slice_width * prng.uniform()
    x_hi = x_lo + slice_width
    if max_steps_out > 0:
        n_down = np.round(prng.uniform() * max_steps_out)
        n_up = max_steps_out - n_down
        s = 0
        while s < n_down and log_y < log_f_func(x_lo):
            x_lo -= slice_width
            s += 1
        s = 0
        while s < n_up and log_y < log_f_func(x_hi):
            x_hi += slice_width
            s += 1
    it = 0
    while it < max_slice_iters:
        x_prop = x_lo + (x_hi - x_lo) * prng.uniform()
        log_f_prop = log_f_func(x_prop)
        if log_f_prop > log_y:
            return x_prop, log_f_prop
        if x_prop < x_curr:
            x_lo = x_prop
        elif x_prop > x_curr:
            x_hi = x_prop
        else:
            warnings.warn('Slice collapsed to current value')
            return x_curr, log_f_curr
        it += 1
    raise MaximumIterationsExceededError(
        'Exceed maximum slice iterations: '
        'i={0}, x_min={1}, x_max={2}, log_f_prop={3}, log_f_curr={4}'
        .format(it, x_lo, x_hi, log_f_prop, log_f_curr))

# -*- coding: utf-8 -*-
"""Squared-exponential Gram builders on the GPU (replace the reference's Cython kernels.pyx).

The two functions keep the reference signature ``f(K, X, theta, epsilon=1e-8)`` and fill the
caller-owned ``K`` in place (kernels.pyx:12-49, :52-90); ``theta`` entries beyond the ones the
kernel reads are ignored and a too-short ``theta`` raises ``IndexError`` as the bounds-checked
Cython does. :func:`make_kernel_func` returns the ``kernel_func(K, X, theta)`` callable the
estimators expect; the estimators recognise it and build K directly in device memory instead of
round-tripping it through the host.
"""
from . import _native

__all__ = ['isotropic_squared_exponential_kernel', 'diagonal_squared_exponential_kernel',
           'make_kernel_func', 'SEKernelFunc']


def isotropic_squared_exponential_kernel(K, X, theta, epsilon=1e-8):
    """K[i,j] = exp(theta[0]) exp(-|x_i - x_j|^2 / (2 exp(theta[1])^2)) + epsilon [i == j]."""
    _native.gram(_native.KERNEL_ISO, K, X, theta, epsilon)


def diagonal_squared_exponential_kernel(K, X, theta, epsilon=1e-8):
    """K[i,j] = exp(theta[0]) exp(-1/2 sum_k ((x_ik - x_jk) / exp(theta[k+1]))^2) + eps [i == j]."""
    _native.gram(_native.KERNEL_ARD, K, X, theta, epsilon)


class SEKernelFunc(object):
    """``kernel_func(K, X, theta)`` for the isotropic ('iso') or ARD ('ard') SE kernel."""

    def __init__(self, kind, epsilon=1e-8):
        if kind not in ('iso', 'ard'):
            raise ValueError("kind must be 'iso' or 'ard'")
        self.kind = kind
        self.epsilon = float(epsilon)
        self.native_kind = _native.KERNEL_ISO if kind == 'iso' else _native.KERNEL_ARD

    def __call__(self, K, X, theta):
        _native.gram(self.native_kind, K, X, theta, self.epsilon)

    def __repr__(self):
        return 'SEKernelFunc({0!r}, epsilon={1!r})'.format(self.kind, self.epsilon)


def make_kernel_func(kind, epsilon=1e-8):
    return SEKernelFunc(kind, epsilon)

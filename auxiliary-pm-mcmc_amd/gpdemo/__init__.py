# -*- coding: utf-8 -*-
"""GP probit-classification pieces of the APM hot path, backed by libapm.so (HIP, gfx950).

Module layout mirrors the reference's ``gpdemo`` package: ``kernels`` (Gram builders),
``latent_posterior_approximations`` (Laplace), ``estimators`` (log-marginal-likelihood
estimators), ``utils`` (priors, adaptation schedule, I/O)."""

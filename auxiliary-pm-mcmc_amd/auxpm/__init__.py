# -*- coding: utf-8 -*-
"""Host-side (auxiliary) pseudo-marginal MCMC samplers, API-compatible with the reference's
``auxpm`` package; the estimator they drive runs on the MI355X (``gpdemo.estimators``)."""

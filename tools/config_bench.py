"""GPU throughput of the batched drivers at BASELINE.json configs[0] and configs[1] (development
tool; bench.py measures the headline configs[2]/[3]):

* configs[0]: PM-MH, iso SE, Pima-shaped synthetic N=768 D=8, N_imp=1 (BatchedPMMHSampler,
  IS estimator; the notebook's Laplace adaptive phase is deterministic and not timed here);
* configs[1]: APM E-SS(u) + MH(theta), ARD SE, N=768 D=8, N_imp=64
  (BatchedAPMEllSSPlusMHSampler).

Each at 1 chain (the reference's per-chain protocol) and 64 chains per GPU. Prints one JSON line
of MCMC iterations/s (all chains) per config and batch.

    python tools/config_bench.py [--steps 30]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))
from auxpm.batched import BatchedAPMEllSSPlusMHSampler, BatchedPMMHSampler  # noqa: E402
from gpdemo.utils import synthetic_gp_data  # noqa: E402


def run(make, chains, steps, warm=5):
    smp = make(chains)
    th0 = smp.prior_draw()
    smp.get_samples(warm, th0)  # warm-up (and the first theta-call's one-off setup)
    t0 = time.perf_counter()
    th, nrej = smp.get_samples(steps + 1)
    el = time.perf_counter() - t0
    return {'chains': chains, 'iterations_per_s': chains * steps / el, 'seconds': el,
            'accept_rate': float(1 - nrej.mean() / steps), 'failed': int(smp.failed.sum()),
            'theta_calls': int(smp.n_theta_calls), 'u_calls': int(smp.n_u_calls)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=30)
    a = ap.parse_args()
    n, d = 768, 8
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    Xi, yi = synthetic_gp_data(n, d, 20151009, 'iso')
    Xa, ya = synthetic_gp_data(n, d, 20151009, 'ard')
    out = {'configs0_pmmh_iso_n768_nimp1': [], 'configs1_essmh_ard_n768_nimp64': []}
    for C in (1, 64):
        out['configs0_pmmh_iso_n768_nimp1'].append(run(
            lambda c: BatchedPMMHSampler(Xi, yi, c, 1, prior, prop_scales=[0.5, 0.5],
                                         kernel='iso', seed=1), C, a.steps))
        out['configs1_essmh_ard_n768_nimp64'].append(run(
            lambda c: BatchedAPMEllSSPlusMHSampler(Xa, ya, c, 64, prior, prop_scales=0.05,
                                                   seed=1), C, a.steps))
        print(json.dumps(out), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()

"""Development tool: the bench workload (configs[2], 64 chains per GPU) run as K cohorts of 64/K
chains, each its own device context (own HIP streams) driven by its own host thread, so that the
latency-bound phases of one cohort's theta-call (Newton TRSVs, dataflow panels, host round trips)
overlap the MFMA-bound phases of another's. Chain c always uses the streams of chain c of one
64-chain sampler (first_chain), so the trajectories are the same whatever K.

    python tools/cohort_bench.py --cohorts 1 2 4 --steps 20 --warmup 5
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def run(K, a, X, y):
    from auxpm.batched import BatchedAPMEllSSPlusRandDirSliceSampler
    prior = dict(a_tau=1., b_tau=1. / a.d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    C = a.chains // K
    smps = [BatchedAPMEllSSPlusRandDirSliceSampler(
        X, y, C, a.n_imp, prior, kernel='ard', epsilon=1e-8, w=1., max_steps_out=0,
        seed=a.seed, first_chain=q * C) for q in range(K)]
    th = None
    if a.stationary:  # the long-chain record's chain states (bench.stationary_states)
        th = np.load(a.stationary)[np.arange(a.chains) % 64]
    for q, s in enumerate(smps):
        s.initialise(None if th is None else th[q * C:(q + 1) * C])

    def par(fn):
        out = [None] * K
        ths = [threading.Thread(target=lambda q=q: out.__setitem__(q, fn(smps[q])))
               for q in range(K)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        return out
    par(lambda s: s.run_async(a.warmup))
    t0 = time.perf_counter()
    res = par(lambda s: s.run_async(a.steps, keep_going=True))
    el = time.perf_counter() - t0
    done = sum(int(r[1][~s.failed].sum()) for r, s in zip(res, smps))
    first = [list(map(float, res[q][0][c][0])) for q in range(K) for c in range(min(2, C))]
    for s in smps:
        s.ctx.close()
    return {'cohorts': K, 'transitions': done, 'elapsed_s': el, 'transitions_per_s': done / el,
            'first_theta_of_first_chains': first[:2]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cohorts', type=int, nargs='+', default=[1, 2])
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--chains', type=int, default=64)
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--d', type=int, default=32)
    ap.add_argument('--n-imp', type=int, default=256)
    ap.add_argument('--seed', type=int, default=20151009)
    ap.add_argument('--stationary', default=None,
                    help='start from these chain states (profiles/r04_stationary_thetas.npy)')
    a = ap.parse_args()
    from gpdemo.utils import synthetic_gp_data
    X, y = synthetic_gp_data(a.n, a.d, a.seed)
    for K in a.cohorts:
        r = run(K, a, X, y)
        print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()

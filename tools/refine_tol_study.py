"""Accuracy of the mixed-precision Newton modes at the long-chain record's stationary states
(development tool): the 64-chain IS theta-call with the default refinement tolerance and with
looser ones (APM_REFINE_TOL), each against the all-fp64 Newton iteration (APM_MIXED=0) on the same
states: per chain max |f_post - f_post64| / max |f_post64| (read from the slots of the first
--nread chains), max |d log f|, n_cubic_ops equality, refinement rounds per theta-call and the
theta-call time.

    python tools/refine_tol_study.py [--tols 1e-3 3e-3 1e-2] [--nread 16]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def run(env, th, X, y, nread, reps):
    from gpdemo import _native
    for k in ('APM_MIXED', 'APM_REFINE_TOL'):
        os.environ.pop(k, None)
    os.environ.update(env)
    nb = len(th)
    ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, 256, max_batch=nb, n_slots=nb,
                          n_ubufs=nb)
    idx = np.arange(nb)
    ctx.u_normal(idx, np.full(nb, 7), idx)
    ts = []
    for r in range(reps + 1):
        if r == 1:
            ctx.prof_read(_native.PROF_STATS, reset=True)
        t0 = time.perf_counter()
        out, st, nops = ctx.theta_eval(_native.EST_IS, th, idx, idx)
        if r:
            ts.append(time.perf_counter() - t0)
    rounds = ctx.prof_read(_native.PROF_STATS)[2] / max(reps, 1)
    fp = [ctx.slot_read(s)[1] for s in range(nread)]
    ctx.close()
    return out, st, nops, np.array(fp), 1e3 * np.median(ts) if ts else float('nan'), rounds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tols', nargs='+', default=['1e-3', '3e-3', '1e-2'])
    ap.add_argument('--nread', type=int, default=16)
    ap.add_argument('--reps', type=int, default=2)
    ap.add_argument('--theta-file', default=os.path.join(REPO, 'profiles',
                                                         'r04_stationary_thetas.npy'))
    a = ap.parse_args()
    from gpdemo import utils
    X, y = utils.synthetic_gp_data(4096, 32, 20151009)
    th = np.load(a.theta_file)[:64].astype(np.float64)
    o64, s64, n64, f64, t64, _ = run({'APM_MIXED': '0'}, th, X, y, a.nread, 1)
    print('all-fp64 Newton: theta-call {0:.1f} ms, status ok {1}'.format(t64, bool((s64 == 0).all())),
          flush=True)
    for tol in a.tols:
        o, s, n, f, t, rounds = run({'APM_REFINE_TOL': tol}, th, X, y, a.nread, a.reps)
        rel = np.abs(f - f64).max(1) / np.abs(f64).max(1)
        print('refine tol {0}: theta-call {1:.1f} ms  refinement rounds {2:.1f}  status ok {3}  '
              'n_cubic_ops equal {4}  max|dlogf| {5:.2e}  f_post rel err max {6:.2e} median {7:.2e}'
              .format(tol, t, rounds, bool((s == 0).all()), bool((n == n64).all()),
                      float(np.abs(o - o64).max()), float(rel.max()), float(np.median(rel))),
              flush=True)


if __name__ == '__main__':
    main()

"""APM_SKEW probe (development tool): the 64-chain stationary theta-call + cached u-call under each
APM_SKEW value, wall time per call, max |d log f| against the undelayed context, statuses and the
guard's residuals - evidence that the delay kernels ran and what a dropped wait does.

    python tools/skew_probe.py 0 1 2 3 4 5 [--calls 2]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('modes', nargs='+')
    ap.add_argument('--calls', type=int, default=2)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--env', nargs='*', default=[], help='VAR=value for every context')
    ap.add_argument('--pkg', default=None,
                    help='import gpdemo from this directory instead (another build\'s binding; '
                         'with APM_LIB naming its library)')
    a = ap.parse_args()
    if a.pkg:
        sys.path.insert(0, a.pkg)
    for kv in a.env:
        k, v = kv.split('=', 1)
        os.environ[k] = v
    from gpdemo import _native
    from gpdemo import utils
    X, y = utils.synthetic_gp_data(4096, 32, 20151009)
    B = a.batch
    th = np.load(os.path.join(REPO, 'tests', 'golden', 'stationary_thetas.npy'))[
        np.arange(B) % 64].astype(np.float64)
    base = None
    for m in a.modes:
        os.environ['APM_SKEW'] = m
        ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, 256, max_batch=B, n_slots=B,
                              n_ubufs=B)
        del os.environ['APM_SKEW']
        idx = np.arange(B)
        ctx.u_normal(idx, np.full(B, 7), idx)
        for r in range(a.calls):
            t0 = time.perf_counter()
            out, st, nops = ctx.theta_eval(_native.EST_IS, th, idx, idx)
            t1 = time.perf_counter()
            out2, st2 = ctx.u_eval(idx, idx)
            g = ctx.guard_read(B) if hasattr(ctx, 'guard_read') else np.zeros((B, 4))
            if base is None:
                base = (out.copy(), out2.copy())
            ok = st == 0
            silent = int((ok & ((out != base[0]) | (out2 != base[1]))).sum())
            d1 = np.abs(out - base[0])[ok].max() if ok.any() else np.nan
            d2 = np.abs(out2 - base[1])[ok].max() if ok.any() else np.nan
            print('APM_SKEW={0} call {1}: theta-call {2:.1f} ms  statuses {3}  silent {10}  max|d| ok chains '
                  'theta {4:.3e} u {5:.3e}  guard max r1 {6:.2e} r2 {7:.2e} r3 {8:.2e} r4 {9:.2e}'.format(
                      m, r, 1e3 * (t1 - t0), dict(zip(*np.unique(st, return_counts=True))), d1,
                      d2, np.nanmax(g[:, 0]), np.nanmax(g[:, 1]), np.nanmax(g[:, 2]),
                      np.nanmax(g[:, 3]), silent), flush=True)
        ctx.close()


if __name__ == '__main__':
    main()

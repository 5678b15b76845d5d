"""Determinism check of the 64-chain stationary theta-call (development tool). Every call
evaluates the same 64 (theta, u) pairs, but call r of a context assigns pair k to chain position
(k + 7 r) mod 64 (its slot, workspace rows and U buffer move with it), so a read of any state a
previous call left behind - in a workspace, a slot, a progress word, a cache line - changes a
value instead of returning identical bytes. Each value is compared with pair k's value from the
first call of the first context; the guard's residuals and the device counters are printed.

    python tools/det_check.py [--contexts 3] [--calls 4] [--env APM_SKEW=1 ...]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--contexts', type=int, default=3)
    ap.add_argument('--calls', type=int, default=4)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--env', nargs='*', default=[],
                    help='VAR=value settings for every context after the first')
    ap.add_argument('--theta-file', default=os.path.join(REPO, 'tests', 'golden',
                                                         'stationary_thetas.npy'))
    a = ap.parse_args()
    from gpdemo import _native
    from gpdemo import utils
    X, y = utils.synthetic_gp_data(4096, 32, 20151009)
    B = a.batch
    th = np.load(a.theta_file)[np.arange(B) % 64].astype(np.float64)
    ref = None
    bad = 0
    for ci in range(a.contexts):
        for kv in (a.env if ci else []):
            k, v = kv.split('=', 1)
            os.environ[k] = v
        ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, 256, max_batch=B, n_slots=B,
                              n_ubufs=B)
        idx = np.arange(B)
        ctx.u_normal(idx, np.full(B, 7), idx)  # U buffer k: pair k's draws
        for r in range(a.calls):
            pos = (idx + 7 * (r + ci)) % B      # chain position of pair k
            order = np.argsort(pos)             # pair evaluated at each position
            out, st, nops = ctx.theta_eval(_native.EST_IS, th[order], order, idx)
            out2, st2 = ctx.u_eval(idx, order)
            g = ctx.guard_read(B)
            v1, v2, nk = np.empty(B), np.empty(B), np.empty(B, dtype=np.int64)
            v1[order], v2[order], nk[order] = out, out2, nops
            if ref is None:
                ref = (v1.copy(), v2.copy(), nk.copy())
            d, d2 = np.abs(v1 - ref[0]), np.abs(v2 - ref[1])
            ctrs = [ctx.prof_read(k)[1] for k in (_native.PROF_STATS, _native.PROF_DF_TIMEOUTS,
                                                   _native.PROF_TRSV_TIMEOUTS, _native.PROF_GUARD)]
            same = (d == 0).all() and (d2 == 0).all() and (nk == ref[2]).all()
            print('context {0} call {1}: max|d| theta {2:.3e} u {3:.3e}  status ok {4}  bitwise {5}'
                  '  counters [reruns, df, trsv, guard] {6}  guard max r1 {7:.2e} r2 {8:.2e} '
                  'r3 {9:.2e} r4 {10:.2e}'.format(ci, r, d.max(), d2.max(),
                                      bool((st == 0).all() and (st2 == 0).all()), bool(same), ctrs,
                                      g[:, 0].max(), g[:, 1].max(), g[:, 2].max(),
                                      g[:, 3].max()), flush=True)
            if not same:
                bad += 1
                for k in np.nonzero((d > 0) | (d2 > 0) | (nk != ref[2]))[0][:8]:
                    print('   pair {0} at position {1}: theta-call {2!r} vs {3!r}, u-call {4!r} vs '
                          '{5!r}, nops {6} vs {7}'.format(k, pos[k], v1[k], ref[0][k], v2[k],
                                                         ref[1][k], nk[k], ref[2][k]), flush=True)
        ctx.close()
    print('differing calls:', bad)
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main())

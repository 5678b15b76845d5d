"""Determinism check of the 64-chain stationary theta-call (development tool): for each value of an
APM_* knob (one context each, created in turn in one process) every call's per-chain estimates
are compared with the first call's of the first context; a differing call prints the chains, their
values and the device counters.

    python tools/det_check.py APM_OVERLAP_K 1 0 1 0 --calls 4
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('var')
    ap.add_argument('values', nargs='+')
    ap.add_argument('--calls', type=int, default=4)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--prof', action='store_true',
                    help='HIP-event profiling on from the second call (as tools/ab_knob.py)')
    ap.add_argument('--theta-file', default=os.path.join(REPO, 'profiles',
                                                         'r04_stationary_thetas.npy'))
    a = ap.parse_args()
    from gpdemo import _native
    from gpdemo import utils
    X, y = utils.synthetic_gp_data(4096, 32, 20151009)
    th = np.load(a.theta_file)[np.arange(a.batch) % 64].astype(np.float64)
    ref = None
    bad = 0
    for ci, v in enumerate(a.values):
        os.environ[a.var] = v
        ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, 256, max_batch=a.batch,
                              n_slots=a.batch, n_ubufs=a.batch)
        idx = np.arange(a.batch)
        ctx.u_normal(idx, np.full(a.batch, 7), idx)
        for r in range(a.calls):
            if a.prof and r == 1:
                for k in range(_native.PROF_NKINDS):
                    ctx.prof_read(k, reset=True)
                ctx.prof_enable(1)
            out, st, nops = ctx.theta_eval(_native.EST_IS, th, idx, idx)
            out2, st2 = ctx.u_eval(idx, idx)
            if ref is None:
                ref = (out.copy(), out2.copy(), nops.copy())
            d = np.abs(out - ref[0])
            d2 = np.abs(out2 - ref[1])
            ctrs = [ctx.prof_read(k)[1] for k in (_native.PROF_STATS, _native.PROF_DF_TIMEOUTS,
                                                   _native.PROF_TRSV_TIMEOUTS)]
            ok = d.max() <= 1e-3 and d2.max() <= 1e-3 and (nops == ref[2]).all()
            print('context {0} ({1}={2}) call {3}: max|d| theta {4:.3e} u {5:.3e}  status ok {6}  '
                  'nops equal {7}  counters {8}'.format(ci, a.var, v, r, d.max(), d2.max(),
                                                        bool((st == 0).all() and (st2 == 0).all()),
                                                        bool((nops == ref[2]).all()), ctrs),
                  flush=True)
            if not ok:
                bad += 1
                for b in np.nonzero((d > 1e-3) | (d2 > 1e-3) | (nops != ref[2]))[0]:
                    print('   chain {0}: theta-call {1!r} vs {2!r}, u-call {3!r} vs {4!r}, nops {5} '
                          'vs {6}, status {7} {8}'.format(b, out[b], ref[0][b], out2[b], ref[1][b],
                                                          nops[b], ref[2][b], st[b], st2[b]),
                          flush=True)
        ctx.close()
    print('differing calls:', bad)
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main())

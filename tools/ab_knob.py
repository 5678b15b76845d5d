"""A/B of a context knob on one box, in one process (development tool): the 64-chain theta-call
(and the cached u-call) at the long-chain record's stationary states under each value of an
APM_* environment variable (read by apm_create), timed over --reps calls after one warm-up call,
with the outputs compared against the first value's: max |d log f|, n_cubic_ops and status equal,
and a per-phase kernel-time split from the library's profiling counters.

    python tools/ab_knob.py APM_H3 0 1 [--reps 3] [--batch 64]
"""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('var')
    ap.add_argument('values', nargs='+')
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--theta-file', default=os.path.join(REPO, 'profiles',
                                                         'r04_stationary_thetas.npy'))
    a = ap.parse_args()
    from gpdemo import _native
    from gpdemo import utils
    X, y = utils.synthetic_gp_data(4096, 32, 20151009)
    th = np.load(a.theta_file)[np.arange(a.batch) % 64].astype(np.float64)
    base = None
    for v in a.values:
        os.environ[a.var] = v
        ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, 256, max_batch=a.batch,
                              n_slots=a.batch, n_ubufs=a.batch)
        idx = np.arange(a.batch)
        ctx.u_normal(idx, np.full(a.batch, 7), idx)
        ts, tu = [], []
        for r in range(a.reps + 1):
            if r == 1:
                for k in range(_native.PROF_NKINDS):
                    ctx.prof_read(k, reset=True)
                ctx.prof_enable(1)
            t0 = time.perf_counter()
            out, st, nops = ctx.theta_eval(_native.EST_IS, th, idx, idx)
            t1 = time.perf_counter()
            out2, st2 = ctx.u_eval(idx, idx)
            t2 = time.perf_counter()
            if r:
                ts.append(t1 - t0)
                tu.append(t2 - t1)
        prof = {k: ctx.prof_read(getattr(_native, 'PROF_' + k)) for k in
                ('CHOL_UPDATE32_OUTER', 'CHOL_UPDATE_OUTER', 'UGEMM', 'POST32_OUTER')}
        ctrs = [ctx.prof_read(k)[1] for k in (_native.PROF_STATS, _native.PROF_DF_TIMEOUTS,
                                               _native.PROF_TRSV_TIMEOUTS)]
        nref = ctx.prof_read(_native.PROF_STATS)[2] / a.reps  # refinement rounds per theta-call
        ctx.close()
        h = hashlib.sha1(out.tobytes()).hexdigest()[:12]
        line = '{0}={1}: theta-call {2:.2f} ms (min {3:.2f})  u-call {4:.3f} ms  hash {5}  ' \
               'status ok {6}  reruns/df/trsv timeouts {7}  refinement rounds {8:.1f}'.format(
                   a.var, v, 1e3 * np.median(ts), 1e3 * min(ts), 1e3 * np.median(tu), h,
                   bool((st == 0).all() and (st2 == 0).all()), ctrs, nref)
        if base is None:
            base = (out, out2, nops)
        else:
            line += '  max|dlogf| theta {0:.2e} u {1:.2e}  nops equal {2}'.format(
                float(np.abs(out - base[0]).max()), float(np.abs(out2 - base[1]).max()),
                bool((nops == base[2]).all()))
        print(line, flush=True)
        for k, (ms, cnt, wk) in prof.items():
            if cnt:
                print('    {0:22s} {1:8.2f} ms / {2:4d} launches  {3:7.1f} TFLOP/s'.format(
                    k, ms / a.reps, cnt // a.reps, wk / (ms * 1e-3) / 1e12), flush=True)


if __name__ == '__main__':
    main()

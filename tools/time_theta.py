"""Quick timing of the batched theta-call / u-call at a given size (development tool)."""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))
from gpdemo import _native  # noqa: E402
from gpdemo import utils  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--n', type=int, default=4096)
ap.add_argument('--d', type=int, default=32)
ap.add_argument('--s', type=int, default=256)
ap.add_argument('--batch', type=int, default=1)
ap.add_argument('--reps', type=int, default=3)
ap.add_argument("--no-prof", action="store_true")
ap.add_argument("--theta0", type=float, default=0.0, help="log signal variance of the thetas")
ap.add_argument("--theta-file", default=None,
                help=".npy of (batch, D+1) thetas, e.g. profiles/r04_stationary_thetas.npy (the "
                     "long-chain record's 64 chains at 9000 transitions: the stationary regime)")
a = ap.parse_args()

X, y = utils.synthetic_gp_data(a.n, a.d, 20151009)
ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, a.s, max_batch=a.batch,
                      n_slots=a.batch, n_ubufs=a.batch)
ctx.u_normal(np.arange(a.batch), np.full(a.batch, 7), np.arange(a.batch))
th = np.tile(np.r_[a.theta0, np.full(a.d, np.log(np.sqrt(a.d)))], (a.batch, 1))
th += np.random.RandomState(0).normal(scale=0.1, size=th.shape)
if a.theta_file:
    th = np.load(a.theta_file)[:a.batch].astype(np.float64)
    assert th.shape == (a.batch, a.d + 1)
for r in range(a.reps):
    if r == min(1, a.reps - 1) and not a.no_prof:  # rep 0 is cold (tile lists, first launches): not profiled
        for k in range(_native.PROF_NKINDS):
            ctx.prof_read(k, reset=True)
        ctx.prof_enable(2)
    t0 = time.perf_counter()
    out, st, nops = ctx.theta_eval(_native.EST_IS, th, np.arange(a.batch), np.arange(a.batch))
    t1 = time.perf_counter()
    out2, st2 = ctx.u_eval(np.arange(a.batch), np.arange(a.batch))
    t2 = time.perf_counter()
    print('rep {0}: theta-call {1:.2f} ms  u-call {2:.3f} ms  logf {3}  status {4}  ops {5}'
          .format(r, 1e3 * (t1 - t0), 1e3 * (t2 - t1), out[:2], st[:2], nops[:2]), flush=True)
print('newton iterations per chain (sorted):', sorted((np.asarray(nops) - 3).tolist()))
print('hash theta-call {0} u-call {1}'.format(hashlib.sha1(out.tobytes()).hexdigest()[:16],
                                            hashlib.sha1(out2.tobytes()).hexdigest()[:16]))
for k, name in ((0, 'gram'), (1, 'chol_update'), (2, 'ugemm'), (3, 'chol_update32'),
                (5, 'upd32_outer'), (6, 'upd64_outer'), (8, 'post32_outer')):
    ms, cnt, wk = ctx.prof_read(k)
    rate = wk / (ms * 1e-3) if ms > 0 else 0
    print('{0:12s} total {1:9.3f} ms  launches {2:6d}  avg {3:8.4f} ms  {4:.3f} {5}/s'.format(
        name, ms, cnt, ms / max(cnt, 1), rate / 1e12, 'TB' if k == 0 else 'TFLOP'))
print('posterior bottom blocks recomputed in fp64:', ctx.prof_read(_native.PROF_POST64_RERUNS)[1])

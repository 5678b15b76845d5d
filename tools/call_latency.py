"""Per-call host latency of the C-ABI at the bench size (development tool): a 1-chain u_combine
(tiny kernel + sync), a 1-chain and a 32-chain u_eval (N=4096, S=256), repeated."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))
from gpdemo import _native, utils  # noqa: E402

X, y = utils.synthetic_gp_data(4096, 32, 20151009)
C = 32
ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, 256, max_batch=C, n_slots=C, n_ubufs=2 * C)
idx = np.arange(C)
ctx.u_normal(idx, np.full(C, 3), idx)
th = np.tile(np.r_[0.0, np.full(32, np.log(np.sqrt(32)))], (C, 1))
ctx.theta_eval(_native.EST_IS, th, idx, idx)
res = {}
for name, fn in (
        ('u_combine_1', lambda: ctx.u_combine([C], [0], [1], [0.6], [0.8])),
        ('u_eval_1', lambda: ctx.u_eval([0], [0])),
        ('u_eval_32', lambda: ctx.u_eval(idx, idx)),
        ('prof_marker', lambda: ctx.prof_marker(0))):
    for _ in range(20):
        fn()
    t0 = time.perf_counter()
    for _ in range(200):
        fn()
    res[name] = (time.perf_counter() - t0) / 200 * 1e6
print('APM_SCHED={0}: '.format(os.environ.get('APM_SCHED', 'default')) +
      '  '.join('{0} {1:.1f} us'.format(k, v) for k, v in res.items()), flush=True)

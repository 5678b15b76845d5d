"""k_ugemm (C_chol.U + probit epilogue) in isolation: cached u-calls at several batch sizes after
one batched theta-call at the bench shape (N=4096, D=32, S=256). HIP-event time per launch and
fp32-MFMA TFLOP/s (N(N+1)S flops per chain). Development tool: A/B two builds with APM_LIB.

    python tools/ugemm_bench.py [--batches 1,8,21,64 --reps 20]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))
from gpdemo import _native  # noqa: E402
from gpdemo import utils  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--n', type=int, default=4096)
ap.add_argument('--d', type=int, default=32)
ap.add_argument('--s', type=int, default=256)
ap.add_argument('--batches', default='1,8,21,64')
ap.add_argument('--reps', type=int, default=20)
a = ap.parse_args()
B = 64
X, y = utils.synthetic_gp_data(a.n, a.d, 20151009)
ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, a.s, max_batch=B, n_slots=B, n_ubufs=B)
ctx.u_normal(np.arange(B), np.full(B, 7), np.arange(B))
th = np.tile(np.r_[0.0, np.full(a.d, np.log(np.sqrt(a.d)))], (B, 1))
th += np.random.RandomState(0).normal(scale=0.1, size=th.shape)
out, st, _ = ctx.theta_eval(_native.EST_IS, th, np.arange(B), np.arange(B))
assert (st == 0).all()
ref = None
for nb in [int(x) for x in a.batches.split(',')]:
    idx = np.arange(nb)
    ctx.u_eval(idx, idx)  # warm
    ctx.prof_read(_native.PROF_UGEMM, reset=True)
    ctx.prof_enable(True)
    for _ in range(a.reps):
        o, _ = ctx.u_eval(idx, idx)
    ctx.prof_enable(False)
    ms, cnt, fl = ctx.prof_read(_native.PROF_UGEMM, reset=True)
    if nb == B:
        ref = o
    print('batch {0:3d}: {1:8.1f} us/launch  {2:6.1f} TFLOP/s  logf[0] {3:.6f}'.format(
        nb, 1e3 * ms / cnt, fl / (ms * 1e-3) / 1e12, o[0]), flush=True)
print('checksum', float(np.sum(ref)))

"""Development experiment: how far does the IS estimate move when the posterior factor
C_chol = L_K U^-T is formed in fp32 arithmetic (SYRK M = I + L_K^T W L_K,
chol of J M J, the triangular solve) instead of fp64?  fp32 LAPACK/BLAS stands in for the
device's fp16x3 updates + fp32 panels. Uses the oracle (development tool, not product).

    python tools/exp_post32.py --n 4096
"""
import argparse
import os
import sys
import time

import numpy as np
import scipy.linalg as la

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'oracle'))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def post32(K_chol, W):
    L32 = K_chol.astype(np.float32)
    Y = L32 * np.sqrt(W).astype(np.float32)[:, None]         # W^1/2 L_K
    M = np.eye(K_chol.shape[0], dtype=np.float32) + Y.T.dot(Y)
    Lp = la.cholesky(M[::-1, ::-1], lower=True)
    U = Lp[::-1, ::-1]
    C = la.solve_triangular(U, L32.T, lower=False).T
    return C.astype(np.float64), 2. * np.log(Lp.diagonal().astype(np.float64)).sum()


def main():
    import apm_oracle as orc
    from gpdemo.utils import synthetic_gp_data
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--d', type=int, default=32)
    ap.add_argument('--s', type=int, default=256)
    a = ap.parse_args()
    X, y = synthetic_gp_data(a.n, a.d, 20151009)
    base = np.log(np.sqrt(a.d))
    rng = np.random.RandomState(7)
    thetas = [np.r_[0.0, np.full(a.d, base)], np.r_[1.0, np.full(a.d, base + 2.0)],
              np.r_[0.7, base + rng.normal(scale=0.5, size=a.d)]]
    for s0 in (2.0, 3.2, 4.5, 6.0):
        thetas.append(np.r_[s0, base + rng.normal(scale=0.7, size=a.d)])
    U = np.random.RandomState(1).normal(size=(a.n, a.s))
    K = np.empty((a.n, a.n))
    for th in thetas:
        t0 = time.time()
        orc.ard_se_kernel(K, X, th)
        st = orc.theta_state_pushthrough(K.copy(), y)
        K_chol = la.cholesky(K, lower=True)
        ref = orc.is_estimate_consistent(y, st, U)
        r32 = orc.is_estimate_consistent(y, st, U, C_chol=st['C_chol'].astype(np.float32).astype(np.float64))
        C32, ld32 = post32(K_chol, st['W'])
        st2 = dict(st, logdet_B=ld32)
        e32 = orc.is_estimate_consistent(y, st, U, C_chol=C32)
        e32ld = orc.is_estimate_consistent(y, st2, U, C_chol=C32)
        rel = np.abs(C32 - st['C_chol']).max() / np.abs(st['C_chol']).max()
        print('th0 %.2f trC %.3g  ref %.6f  store32 %+.2e  arith32 %+.2e  (+ld32 %+.2e)  '
              'relmax %.2e  %.0fs' % (th[0], (st['C_chol'] ** 2).sum(), ref, r32 - ref, e32 - ref,
                                      e32ld - ref, rel, time.time() - t0), flush=True)


if __name__ == '__main__':
    main()

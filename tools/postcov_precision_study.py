"""Which parts of the posterior-covariance factor need fp64?

The device forms C_chol = L_K U^-T with M = I + L_K^T W L_K = U U^T (postcov.hip, all fp64:
~3.3 N^3/3 flops per chain beyond chol(K), the largest fp64 MFMA block of a theta-call). M is as
well conditioned as the Newton matrix B (same eigenvalues), so this study evaluates the IS
estimate (the device's self-consistent form, apm_oracle.is_estimate_consistent) with the pieces
after chol(K) in float32 (LAPACK spotrf / strsm on float32 arrays), against the float64
push-through statement and the reference route (chol(K - V^T V)), on the bench's data at the
parity thetas, with S = 256 standard-normal draws:

  f64     : everything float64 (apm_oracle.theta_state_pushthrough)
  m64_u32 : M formed in float64, its UL factor and the TRSM L_K U^-T in float32, log|M| from the
            float32 factor
  m32_u32 : also Y = W^1/2 L_K and M = I + Y^T Y in float32
  m32_u32_ld64 : m32_u32 with log|B| taken from the float64 route (isolates the log-det error)
  trsm32  : M and its UL factor in float64 (log|M| exact), only the TRSM L_K U^-T in float32 -
            the bottom block of the stacked factorisation [[J M J],[L_K J]]

    python tools/postcov_precision_study.py [--n 2048]
"""
import argparse
import os
import sys

import numpy as np
import scipy.linalg as la

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))


def state32(K_chol, st, m_fp32):
    W = st['W']
    if m_fp32:
        Y = (K_chol.astype(np.float32).T * np.sqrt(W).astype(np.float32)[None])  # L_K^T W^1/2
        M = np.eye(K_chol.shape[0], dtype=np.float32) + Y.dot(Y.T)
    else:
        M = (np.eye(K_chol.shape[0]) + (K_chol.T * W[None]).dot(K_chol)).astype(np.float32)
    Lp = la.cholesky(M[::-1, ::-1], lower=True)
    U = Lp[::-1, ::-1]
    C_chol = la.solve_triangular(U, K_chol.T.astype(np.float32), lower=False).T
    logdet = 2. * np.log(Lp.diagonal().astype(np.float64)).sum()
    out = dict(st)
    out['C_chol'] = C_chol.astype(np.float64)
    out['logdet_B'] = logdet
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=2048)
    ap.add_argument('--d', type=int, default=32)
    ap.add_argument('--theta', type=int, nargs='*', default=[0, 1, 3])
    ap.add_argument('--log-sigma', type=float, nargs='*', default=[None],
                    help='override theta[0] (the posterior of the bench sits near 3.2)')
    a = ap.parse_args()
    import apm_oracle as orc
    from gpdemo.utils import synthetic_gp_data
    z = np.load(os.path.join(REPO, 'tests', 'golden', 'config2_ref.npz'))
    X, y = synthetic_gp_data(a.n, a.d, int(z['data_seed']))
    kf = orc.make_kernel_func('ard', 1e-8)
    rng = np.random.RandomState(5)
    ns = rng.normal(size=(a.n, 256))
    for ti, ls in [(t, l) for t in a.theta for l in a.log_sigma]:
        th = z['thetas'][ti][:a.d + 1].copy()
        if ls is not None:
            th[0] = ls
        K = np.empty((a.n, a.n))
        kf(K, X, th)
        st = orc.theta_state_pushthrough(K, y)
        ref = orc.theta_state_reformulated(K, y)
        K_chol = la.cholesky(K, lower=True)
        v64 = orc.is_estimate_consistent(y, st, ns)
        vref = orc.is_estimate_consistent(y, ref, ns)
        res = {'ref_route': vref - v64}
        for name, m32 in (('m64_u32', False), ('m32_u32', True)):
            s32 = state32(K_chol, st, m32)
            res[name] = orc.is_estimate_consistent(y, s32, ns) - v64
            res[name + '_logdet'] = s32['logdet_B'] - st['logdet_B']
            s32['logdet_B'] = st['logdet_B']
            res[name + '_ld64'] = orc.is_estimate_consistent(y, s32, ns) - v64
            rel = np.abs(s32['C_chol'] - st['C_chol']).max() / np.abs(st['C_chol']).max()
            res[name + '_Cchol_rel'] = rel
        W, st_U = st['W'], None
        M = np.eye(a.n) + (K_chol.T * W[None]).dot(K_chol)
        U = la.cholesky(M[::-1, ::-1], lower=True)[::-1, ::-1]
        Cc = la.solve_triangular(U.astype(np.float32), K_chol.T.astype(np.float32), lower=False).T
        s3 = dict(st)
        s3['C_chol'] = Cc.astype(np.float64)
        res['trsm32'] = orc.is_estimate_consistent(y, s3, ns) - v64
        res['trace_C'] = float((st['C_chol'] ** 2).sum())
        print('theta %d log_sigma %.2f  log f %.6f  ' % (ti, th[0], v64) +
              '  '.join('%s %.2e' % (k, v) for k, v in res.items()), flush=True)


if __name__ == '__main__':
    main()

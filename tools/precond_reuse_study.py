"""How far does the Newton matrix move between iterations?

For the bench's data (configs[2]: N=4096 D=32 ARD) at the parity thetas, run the reference Newton
iteration (latent_posterior_approximations.py:85-99, restated in float64 numpy) and, for each
iteration k >= 2, the spectrum of B_j^-1 B_k for the last factored matrix B_j (j = k-1, k-2):
Richardson (iterative refinement) contracts the error by max|1 - lambda| per step, PCG by
(sqrt(kappa)-1)/(sqrt(kappa)+1). Also the iteration count and diff sequence.

    python tools/preconds_reuse_study.py [--n 4096]
"""
import argparse
import os
import sys

import numpy as np
import scipy.linalg as la
from scipy.special import log_ndtr

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--d', type=int, default=32)
    ap.add_argument('--theta', type=int, nargs='*', default=[0, 1, 3])
    a = ap.parse_args()
    import apm_oracle as orc
    from gpdemo.utils import synthetic_gp_data
    z = np.load(os.path.join(REPO, 'tests', 'golden', 'config2_ref.npz'))
    X, y = synthetic_gp_data(a.n, a.d, int(z['data_seed']))
    kf = orc.make_kernel_func('ard', 1e-8)
    for ti in a.theta:
        th = z['thetas'][ti][:a.d + 1]
        K = np.empty((a.n, a.n))
        kf(K, X, th)
        f = np.zeros(a.n)
        Bs, diffs = [], []
        for i in range(100):
            v = np.exp(-0.5 * f ** 2 - log_ndtr(y * f) - 0.5 * np.log(2 * np.pi))
            g = v * y
            W = v ** 2 + g * f
            s = W ** 0.5
            B = np.eye(a.n) + s[:, None] * K * s[None, :]
            Bs.append(B)
            L = la.cholesky(B, lower=True)
            b = W * f + g
            aa = b - s * la.cho_solve((L, True), s * K.dot(b))
            fn = K.dot(aa)
            diff = np.mean((fn - f) ** 2)
            diffs.append(diff)
            f = fn
            if diff < 1e-4:
                break
        print('theta %d: %d iterations, diffs %s' % (ti, len(Bs), ' '.join('%.1e' % d for d in diffs)))
        for k in range(1, len(Bs)):
            for j in (k - 1, k - 2):
                if j < 0:
                    continue
                Lj = la.cholesky(Bs[j], lower=True)
                M = la.solve_triangular(Lj, la.solve_triangular(Lj, Bs[k], lower=True).T, lower=True)
                lam = la.eigvalsh(M)
                rho = np.abs(1 - lam).max()
                kap = lam.max() / lam.min()
                pcg = (np.sqrt(kap) - 1) / (np.sqrt(kap) + 1)
                print('  B_%d with factor of B_%d: lambda [%.4f, %.4f] richardson rho %.3e  '
                      'pcg rate %.3e  cond(B_k) %.2e' % (k + 1, j + 1, lam.min(), lam.max(), rho,
                                                         pcg, np.linalg.cond(Bs[k])))


if __name__ == '__main__':
    main()

"""Can the Newton solves use explicit inverses of 512-wide diagonal blocks?

The device solves B x = r with the fp32 factor L of B (chol32.hip) by substitution over 64-wide
blocks (inverses of the 64x64 diagonal tiles, fp64 vectors), then refines once in fp64. A solve
over 512-wide blocks against fp32 explicit inverses of the 512x512 diagonal blocks would have 8
instead of 64 dependent steps. This study (numpy; the bench's data, Newton matrices of the
reference iteration at the parity thetas) compares, per Newton iteration, the refinement
contraction rho = |x - x1| / |x - x0| and the relative error of the refined x1 for both solves
on the same fp32 factor (LAPACK spotrf of B rounded to fp32).

    python tools/trsv_inverse_study.py [--n 2048 --block 512]
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


def block_inverses(L32, w):
    """fp32 inverses of the w x w diagonal blocks of the fp32 factor (strtri-like)."""
    n = L32.shape[0]
    return [la.solve_triangular(L32[i:i + w, i:i + w], np.eye(w, dtype=np.float32),
                                lower=True).astype(np.float32) for i in range(0, n, w)]


def fwd(L32, inv, w, r):
    """L y = r by blocks of w: y_J = inv_J (r_J - sum_I<J L_JI y_I), fp64 accumulation."""
    y = np.zeros_like(r)
    for J, i in enumerate(range(0, len(r), w)):
        t = r[i:i + w] - L32[i:i + w, :i].astype(np.float64).dot(y[:i])
        y[i:i + w] = inv[J].astype(np.float64).dot(t)
    return y


def bwd(L32, inv, w, r):
    n = len(r)
    z = np.zeros_like(r)
    for J in reversed(range(n // w)):
        i = J * w
        t = r[i:i + w] - L32[i + w:, i:i + w].astype(np.float64).T.dot(z[i + w:])
        z[i:i + w] = inv[J].astype(np.float64).T.dot(t)
    return z


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=2048)
    ap.add_argument('--d', type=int, default=32)
    ap.add_argument('--block', type=int, default=512)
    ap.add_argument('--theta', type=int, nargs='*', default=[0, 1, 3])
    a = ap.parse_args()
    import apm_oracle as orc
    from gpdemo.utils import synthetic_gp_data
    z = np.load(os.path.join(REPO, 'tests', 'golden', 'config2_ref.npz'))
    X, y = synthetic_gp_data(a.n, a.d, int(z['data_seed']))
    kf = orc.make_kernel_func('ard', 1e-8)
    worst = {64: 0., a.block: 0.}
    for ti in a.theta:
        th = z['thetas'][ti][:a.d + 1]
        K = np.empty((a.n, a.n))
        kf(K, X, th)
        f = np.zeros(a.n)
        for it in range(100):
            v = np.exp(-0.5 * f ** 2 - log_ndtr(y * f) - 0.5 * np.log(2 * np.pi))
            g = v * y
            W = v ** 2 + g * f
            s = W ** 0.5
            B = np.eye(a.n) + s[:, None] * K * s[None, :]
            rhs = s * K.dot(W * f + g)
            x = la.solve(B, rhs, assume_a='pos')
            L32 = la.cholesky(B.astype(np.float32), lower=True)
            row = []
            for w in (64, a.block):
                inv = block_inverses(L32, w)
                x0 = bwd(L32, inv, w, fwd(L32, inv, w, rhs))
                res = rhs - B.dot(x0)
                x1 = x0 + bwd(L32, inv, w, fwd(L32, inv, w, res))
                rho = np.abs(x - x1).max() / np.abs(x - x0).max()
                e1 = np.abs(x - x1).max() / np.abs(x).max()
                worst[w] = max(worst[w], e1)
                row.append('w=%d: x0 err %.1e rho %.1e x1 err %.1e' % (
                    w, np.abs(x - x0).max() / np.abs(x).max(), rho, e1))
            print('theta %d it %d cond %.1e | %s' % (ti, it + 1, np.linalg.cond(B), ' | '.join(row)),
                  flush=True)
            aa = W * f + g - s * x
            fn = K.dot(aa)
            diff = np.mean((fn - f) ** 2)
            f = fn
            if diff < 1e-4:
                break
    print('worst refined error by block width:', worst)


if __name__ == '__main__':
    main()

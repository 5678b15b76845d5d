"""Richardson refinement with the previous Newton iteration's factor, W-rescaled.

For the bench data at a stationary theta (row argv[1] of tests/golden/stationary_thetas.npy), the
reference Newton iteration restated in numpy; per iteration the relative error of 8 refinement
steps preconditioned by E^-1 B_old^-1 E^-1 (E = W^1/2 / W_old^1/2) and by B_old^-1 alone."""
import sys, numpy as np, scipy.linalg as la
from scipy.special import log_ndtr
sys.path[:0] = ['/root/repo/auxiliary-pm-mcmc_amd', '/root/repo']
from gpdemo.utils import synthetic_gp_data
from oracle.apm_oracle import ard_se_kernel
n, d = 4096, 32
X, y = synthetic_gp_data(n, d, 20151009)
th = np.load('/root/repo/tests/golden/stationary_thetas.npy')[int(sys.argv[1]) if len(sys.argv) > 1 else 45]
K = np.empty((n, n)); ard_se_kernel(K, X, th)
f = np.zeros(n); prev = None; i = 0
while True:
    v = np.exp(-0.5 * f**2 - log_ndtr(y * f) - 0.5 * np.log(2 * np.pi))
    g = v * y; W = v**2 + g * f; Ws = W**0.5
    B = np.eye(n) + Ws[:, None] * K * Ws[None, :]
    L = la.cholesky(B, lower=True)
    b = W * f + g; rhs = Ws * K.dot(b)
    xs = la.cho_solve((L, True), rhs)
    if prev is not None:
        Lo, Wso = prev
        E = Ws / Wso
        out = []
        for scaled in (True, False):
            x = np.zeros(n); errs = []
            for k in range(8):
                r = rhs - (x + Ws * K.dot(Ws * x))
                dx = la.cho_solve((Lo, True), r / E if scaled else r) / (E if scaled else 1)
                x = x + dx
                errs.append(np.linalg.norm(x - xs) / np.linalg.norm(xs))
            out.append(errs)
        print('it %d  max|Wo/W-1| %.3g  scaled %s' % (i, np.max(np.abs(1 / E**2 - 1)),
              ' '.join('%.1e' % e for e in out[0])))
        print('      %s unscaled %s' % (' ' * 18, ' '.join('%.1e' % e for e in out[1])))
    prev = (L, Ws)
    a = b - Ws * xs
    fn = K.dot(a); diff = np.mean((fn - f)**2); f = fn; i += 1
    print('  iter %d diff %.3e' % (i, diff))
    if diff < 1e-4: break

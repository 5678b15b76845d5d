"""ORACLE / TEST INFRASTRUCTURE ONLY — CPU restatement of the reference hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline. The
product (``auxiliary-pm-mcmc_amd/``) never imports it and has no CPU fallback.

Every function restates the reference algorithm in the reference's own operation
order (numpy float64, scipy LAPACK), citing the file:line it follows. The oracle is
pinned against golden vectors produced by the reference itself
(``tests/golden/make_golden.py``, fixtures ``tests/golden/*.npz``), see
``tests/test_oracle_golden.py``.

Besides the literal restatement this module also holds
:func:`is_estimate_reformulated`, a float64 statement of the algebraically
identical form of the importance-sampling estimator that the HIP path computes
(DESIGN.md §3). ``tests/test_oracle_golden.py`` checks that it equals the
reference form on the golden vectors, which is what justifies the GPU's form.
"""
import ctypes
import os

import numpy as np
import scipy.linalg as la
from scipy.special import gammaln, log_ndtr, logsumexp

_HERE = os.path.dirname(os.path.abspath(__file__))


class MaximumIterationsExceededError(Exception):
    """Mirror of gpdemo/latent_posterior_approximations.py:17-19."""


class InvalidCovarianceMatrixError(Exception):
    """Mirror of gpdemo/estimators.py:85-87."""


# ----------------------------------------------------------------------------- Gram


def iso_se_kernel(K, X, theta, epsilon=1e-8):
    """gpdemo/kernels.pyx:12-49 (isotropic SE), vectorised over (i, j), k-loop kept in order."""
    sigma = np.exp(theta[0])
    tau = np.exp(theta[1])
    s = np.zeros((X.shape[0], X.shape[0]))
    for k in range(X.shape[1]):
        d = X[:, k][:, None] - X[:, k][None, :]
        s += d ** 2
    K[...] = sigma * np.exp(-s / (2. * tau ** 2))
    K[np.diag_indices_from(K)] = sigma + epsilon


def ard_se_kernel(K, X, theta, epsilon=1e-8):
    """gpdemo/kernels.pyx:52-90 (diagonal / ARD SE), k-loop kept in order."""
    sigma = np.exp(theta[0])
    s = np.zeros((X.shape[0], X.shape[0]))
    for k in range(X.shape[1]):
        d = (X[:, k][:, None] - X[:, k][None, :]) / np.exp(theta[k + 1])
        s += d ** 2
    K[...] = sigma * np.exp(-s / 2.)
    K[np.diag_indices_from(K)] = sigma + epsilon


_CLIB = None


def _clib():
    global _CLIB
    if _CLIB is None:
        path = os.path.join(_HERE, 'liboracle_gram.so')
        if not os.path.exists(path):
            raise OSError('oracle C Gram not built: run `make -C oracle`')
        lib = ctypes.CDLL(path)
        for name in ('oracle_iso_se_kernel', 'oracle_ard_se_kernel'):
            fn = getattr(lib, name)
            fn.restype = None
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_double]
        _CLIB = lib
    return _CLIB


def c_gram(kind, K, X, theta, epsilon=1e-8):
    """Single-threaded C Gram (oracle/gram.c), same op order as kernels.pyx."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    theta = np.ascontiguousarray(theta, dtype=np.float64)
    assert K.flags.c_contiguous and K.dtype == np.float64
    n, d = X.shape
    fn = _clib().oracle_iso_se_kernel if kind == 'iso' else _clib().oracle_ard_se_kernel
    fn(K.ctypes.data, n, X.ctypes.data, d, n, d, theta.ctypes.data, float(epsilon))


def make_kernel_func(kind, epsilon=1e-8, impl='c'):
    """kernel_func(K, X, theta) as built in the notebooks (e.g. Pseudo-Marginal MH.ipynb:165-167)."""
    if impl == 'c':
        return lambda K, X, theta: c_gram(kind, K, X, theta, epsilon)
    fn = iso_se_kernel if kind == 'iso' else ard_se_kernel
    return lambda K, X, theta: fn(K, X, theta, epsilon)


# ----------------------------------------------------------------------------- priors / utils


def log_gamma_log_pdf(x, a, b):
    """gpdemo/utils.py:39-59."""
    return a * np.log(b) - gammaln(a) + a * x - b * np.exp(x)


def normalise_inputs(X):
    """gpdemo/utils.py:86-105."""
    X_mn = X.mean(0)
    X_sd = X.std(0)
    return (X - X_mn[None]) / X_sd[None], X_mn, X_sd


# ----------------------------------------------------------------------------- Laplace


def laplace_approximation(K, y, calc_cov=True, calc_lml=False, diff_f_tol=1e-4,
                          max_iters=1000, return_internals=False):
    """gpdemo/latent_posterior_approximations.py:22-124, same op order.

    Newton loop :85-99; LML :103-106 and C :107-112 use the L, W, a of the LAST
    iteration (computed at the previous f) together with the updated f.
    ``return_internals`` additionally returns a dict with W_diag, L, a, b (the
    quantities the GPU reformulation consumes).
    """
    f = np.zeros(y.shape[0])
    converged = False
    i = 0
    while not converged and i < max_iters:
        v = np.exp(-0.5 * f ** 2 - log_ndtr(y * f) - 0.5 * np.log(2 * np.pi))
        grad = v * y
        W_diag = v ** 2 + grad * f
        W_diag_sqrt = W_diag ** 0.5
        W_sqrt_K = (W_diag_sqrt * K).T
        B = np.eye(y.shape[0]) + W_sqrt_K * W_diag_sqrt
        L = la.cholesky(B, lower=True)
        b = W_diag * f + grad
        a = b - (W_diag_sqrt * la.cho_solve((L, True), W_sqrt_K.dot(b)))
        f_ = K.dot(a)
        diff = np.mean((f_ - f) ** 2)
        converged = diff < diff_f_tol
        f = f_
        i += 1
    if not converged:
        raise MaximumIterationsExceededError('Failed to converge in {0} iterations'.format(i))
    out = [f]
    if calc_cov:
        B_inv_W_sqrt_K = la.cho_solve((L, True), W_sqrt_K)
        C = K - W_sqrt_K.T.dot(B_inv_W_sqrt_K)
        out.append(C)
    if calc_lml:
        lml = (-0.5 * a.dot(f) + log_ndtr(y * f).sum() - np.log(L.diagonal()).sum())
        out.append(lml)
    out.append(i + 1 if calc_cov else i)
    if return_internals:
        out.append(dict(W_diag=W_diag, L=L, a=a, b=b, n_iter=i))
    return tuple(out)


# ----------------------------------------------------------------------------- estimators


def is_estimate(X, y, kernel_func, ns, theta=None, cached_results=None, K_work=None):
    """gpdemo/estimators.py:152-241 (ApproxPosteriorIS), same op order.

    Returns (log_estimate, (K_chol, C_chol, f_post), cubic_ops_added).
    """
    if theta is None and cached_results is None:
        raise ValueError('One of theta or cached_results must be provided')
    cubic = 0
    if cached_results is None:
        K = np.empty((X.shape[0], X.shape[0])) if K_work is None else K_work
        kernel_func(K, X, theta)
        K_chol = la.cholesky(K, lower=True)
        f_post, C, cubic_ops = laplace_approximation(K, y)
        try:
            C_chol = la.cholesky(C, lower=True)
        except la.LinAlgError:
            e, _ = la.eigh(C)
            raise InvalidCovarianceMatrixError(
                'Posterior covariance matrix not PSD: sum of negative eigenvalues {0}'
                .format(e[e <= 0].sum()))
        cubic = cubic_ops + 2
    else:
        K_chol, C_chol, f_post = cached_results
    n_imp = ns.shape[1]
    f_s = f_post[None] + C_chol.dot(ns).T
    q_K = (la.cho_solve((K_chol, True), f_s.T) * f_s.T).sum(0)
    log_p_f = -0.5 * q_K - np.log(K_chol.diagonal()).sum()
    log_p_y = log_ndtr(f_s * y).sum(-1)
    f_zm = f_s - f_post[None]
    q_C = (la.cho_solve((C_chol, True), f_zm.T) * f_zm.T).sum(0)
    log_q = -0.5 * q_C - np.log(C_chol.diagonal()).sum()
    lw = log_p_y + log_p_f - log_q
    return logsumexp(lw) - np.log(n_imp), (K_chol, C_chol, f_post), cubic


def priormc_estimate(X, y, kernel_func, ns, theta=None, K_chol=None, K_work=None):
    """gpdemo/estimators.py:286-325 (PriorMC), same op order."""
    if theta is None and K_chol is None:
        raise ValueError('One of theta or K_chol must be provided')
    cubic = 0
    if K_chol is None:
        K = np.empty((X.shape[0], X.shape[0])) if K_work is None else K_work
        kernel_func(K, X, theta)
        K_chol = la.cholesky(K, lower=True)
        cubic = 1
    f_s = K_chol.dot(ns).T
    log_p_y = log_ndtr(f_s * y[None]).sum(-1)
    return logsumexp(log_p_y) - np.log(ns.shape[1]), K_chol, cubic


def laplace_estimate(X, y, kernel_func, theta, K_work=None):
    """gpdemo/estimators.py:65-82 (Laplace LML)."""
    K = np.empty((X.shape[0], X.shape[0])) if K_work is None else K_work
    kernel_func(K, X, theta)
    f_post, lml, cubic = laplace_approximation(K, y, calc_cov=False, calc_lml=True)
    return lml, cubic


# ----------------------------------------------------------------------------- GPU form (fp64)


def theta_state_reformulated(K, y):
    """Per-theta state of the reformulated IS estimator.

    With W, L (= chol(B), B = I + W^1/2 K W^1/2) of the last Newton iteration and
    f_post the updated mode, C = (K^-1 + W)^-1 exactly, hence
      log|C| - log|K| = -log|B|,
      f^T K^-1 f = ||C_chol^-1 f||^2 - f^T W f,
    and with g = C_chol^-1 f_post and f_s = f_post + C_chol u_s:
      log w_s = sum_n [log Phi(y_n f_sn) + 1/2 W_n f_sn^2] - g^T u_s - 1/2 ||g||^2 - 1/2 log|B|.
    """
    f_post, C, n_ops, st = laplace_approximation(K, y, return_internals=True)
    C_chol = la.cholesky(C, lower=True)
    g = la.solve_triangular(C_chol, f_post, lower=True)
    logdet_B = 2. * np.log(st['L'].diagonal()).sum()
    return dict(C_chol=C_chol, f_post=f_post, W=st['W_diag'], g=g, logdet_B=logdet_B,
                n_ops=n_ops, a=st['a'])


def theta_state_pushthrough(K, y):
    """The reformulated state with C_chol formed the way the device forms it (DESIGN.md §3.1
    step 3, postcov.hip) instead of chol(K - V^T V) (estimators.py:206-209, lpa.py:111-112):
    C = (K^-1 + W)^-1 = L_K M^-1 L_K^T with M = I + L_K^T W L_K (W of the last Newton iteration),
    M = U U^T by the "UL" Cholesky (U = J chol(J M J) J upper, J the index reversal), so
    C_chol = L_K U^-T (lower, positive diagonal) and log|B| = log|M|. M is SPD for any W >= 0,
    so this never raises where the reference's chol(C) does (InvalidCovarianceMatrixError at
    extreme theta, tests/golden/errors.npz icm_*); chol(K) failing still raises LinAlgError."""
    K_chol = la.cholesky(K, lower=True)
    f_post, _, n_ops, st = laplace_approximation(K, y, return_internals=True)
    W = st['W_diag']
    M = np.eye(K.shape[0]) + (K_chol.T * W[None]).dot(K_chol)
    Lp = la.cholesky(M[::-1, ::-1], lower=True)
    U = Lp[::-1, ::-1]                                   # upper, M = U U^T
    C_chol = la.solve_triangular(U, K_chol.T, lower=False).T   # (U^-1 L_K^T)^T = L_K U^-T
    g = la.solve_triangular(C_chol, f_post, lower=True)
    logdet_M = 2. * np.log(Lp.diagonal()).sum()
    return dict(C_chol=C_chol, f_post=f_post, W=W, g=g, logdet_B=logdet_M, n_ops=n_ops,
                a=st['a'])


def is_estimate_reformulated(y, state, ns):
    """IS log-estimate from the reformulated per-theta state (float64 statement of the GPU math)."""
    f_s = state['f_post'][:, None] + state['C_chol'].dot(ns)          # (N, S)
    t = log_ndtr(y[:, None] * f_s) + 0.5 * state['W'][:, None] * f_s ** 2
    g = state['g']
    lw = t.sum(0) - g.dot(ns) - 0.5 * g.dot(g) - 0.5 * state['logdet_B']
    return logsumexp(lw) - np.log(ns.shape[1])


def is_estimate_consistent(y, state, ns, C_chol=None):
    """The device's self-consistent form of estimators.py:221-241 (ugemm.hip):
    the reference's log p(y|f) + log p(f) - log q(f) evaluated at f_s = f_post + C_chol u_s with
    K^-1 = C^-1 - W and |C| / |K| = 1 / |B| substituted and the quadratic forms expanded around
    f_post, so that nothing but f_s enters per sample:
      log w_s = sum_n [log Phi(y_n f_sn) + 1/2 W_n f_sn^2 - z_n f_sn] + 1/2 f_post^T z
                - 1/2 log|B|,   z = C^-1 f_post = a + W f_post  (f_post = K a, lpa.py:95).
    C_chol: the factor to form f_s with (default: the state's; the GPU passes its fp32 one)."""
    L = state['C_chol'] if C_chol is None else C_chol
    f_post, W = state['f_post'], state['W']
    z = state['a'] + W * f_post
    f_s = f_post[:, None] + L.dot(ns)                                  # (N, S)
    t = log_ndtr(y[:, None] * f_s) + (0.5 * W[:, None] * f_s - z[:, None]) * f_s
    lw = t.sum(0) + 0.5 * f_post.dot(z) - 0.5 * state['logdet_B']
    return logsumexp(lw) - np.log(ns.shape[1])


# ----------------------------------------------------------------------------- CPU baseline wrapper


class ISEstimatorCPU(object):
    """CPU port of LogMarginalLikelihoodApproxPosteriorISEstimator (estimators.py:90-241)
    for the bench's cpu_baseline leg: same op order, C Gram + scipy LAPACK."""

    def __init__(self, X, y, kernel_func):
        self.X, self.y, self.kernel_func = X, y, kernel_func
        self._K = np.empty((X.shape[0], X.shape[0]))
        self.n_cubic_ops = 0

    def __call__(self, ns, theta=None, cached_results=None):
        val, cache, cubic = is_estimate(self.X, self.y, self.kernel_func, ns, theta,
                                        cached_results, K_work=self._K)
        self.n_cubic_ops += cubic
        return val, cache


# ----------------------------------------------------------------------------- device RNG (f2)


PHILOX_KAT = (  # Random123 kat_vectors (Salmon et al., SC'11): counter[4], key[2] -> out[4]
    ((0, 0, 0, 0, 0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 6, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
)


def philox4x32_10(ctr, key):
    """Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; Random123's philox4x32_R with R = 10)
    on rows of uint32 counters (n, 4) and keys (n, 2): the published algorithm the batched
    driver's device draws use (the reference draws u with numpy's MT19937 instead, so this
    stream is pinned by the published known-answer vectors, PHILOX_KAT)."""
    c = np.array(ctr, dtype=np.uint64).reshape(-1, 4)
    k = np.array(key, dtype=np.uint64).reshape(-1, 2)
    m = np.uint64(0xffffffff)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[:, 0]
        p1 = np.uint64(0xCD9E8D57) * c[:, 2]
        n0 = (p1 >> np.uint64(32)) ^ c[:, 1] ^ k[:, 0]
        n2 = (p0 >> np.uint64(32)) ^ c[:, 3] ^ k[:, 1]
        c = np.stack([n0 & m, p1 & m, n2 & m, p0 & m], 1)
        k = np.stack([(k[:, 0] + np.uint64(0x9E3779B9)) & m,
                      (k[:, 1] + np.uint64(0xBB67AE85)) & m], 1)
    return c.astype(np.uint32)


def u_normal(seed, counter, n, s):
    """The (n, s) N(0, 1) draws of apm_u_normal for one (seed, counter) (ugemm.hip k_u_normal):
    Philox block q = counter (q, ctr_lo, ctr_hi, q >> 32), key (seed_lo, seed_hi); its 4 words
    give 2 Box-Muller pairs u = (w + 0.5) 2^-32 (formed in fp32 as on the device),
    z = sqrt(-2 log u1) (cos, sin)(2 pi u2); element 4q + h. Transcendentals in float64 here
    (the device's are fp32: compare to ~1e-6)."""
    tot = n * s
    q = np.arange((tot + 3) // 4, dtype=np.uint64)
    ctr = np.stack([q & np.uint64(0xffffffff), np.full_like(q, counter & 0xffffffff),
                    np.full_like(q, counter >> 32), q >> np.uint64(32)], 1)
    key = np.tile(np.array([seed & 0xffffffff, seed >> 32], dtype=np.uint64), (q.shape[0], 1))
    w = philox4x32_10(ctr, key)
    # u exactly as the device forms it in fp32: ((float)w + 0.5f) * 2^-32
    u = ((w.astype(np.float32) + np.float32(0.5)) * np.float32(2.3283064365386963e-10)
         ).astype(np.float64)
    z = np.empty((q.shape[0], 4))
    for h in range(2):
        r = np.sqrt(-2. * np.log(u[:, 2 * h]))
        ang = (np.float32(6.283185307179586) * u[:, 2 * h + 1].astype(np.float32)).astype(
            np.float64)  # the fp32 angle of the device's sincosf
        z[:, 2 * h] = r * np.cos(ang)
        z[:, 2 * h + 1] = r * np.sin(ang)
    return z.reshape(-1)[:tot].reshape(n, s)

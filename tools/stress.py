"""BASELINE.json configs[4]: synthetic N=16384, D=64, N_imp=1024 — the tiled-Cholesky / fp32-MFMA
L.U roofline stress on one MI355X (ApproxPosteriorIS theta-calls and cached u-calls of a batch of
independent chains, no sampler).

    python tools/stress.py [--n 16384 --d 64 --s 1024 --batch 8 --reps 2] [--check 1]

Prints one JSON line: theta-call / u-call wall time per batch, per-kernel HIP-event timings and
rooflines (same accounting as bench.py), and with --check 1 the full-size parity of chain 0
against the oracle (CPU restatement of estimators.py:152-241 in the reference's op order, scipy
LAPACK on the host cores) on identical (theta, u): theta-call value, cached u-call value, f_post
and C_chol. Memory: ~12 GB of HBM per chain at N=16384 (K, the 2N x 2N work matrix, one slot);
the --check leg needs ~20 GB of host memory and a few minutes of CPU.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'auxiliary-pm-mcmc_amd'), os.path.join(REPO, 'oracle')]
from gpdemo import _native  # noqa: E402
from gpdemo.utils import normalise_inputs  # noqa: E402

PEAK = {'gram': (8.0, 'TB/s', 'hbm'), 'chol_update': (78.6, 'TFLOP/s', 'mfma'),
        'ugemm': (157.3, 'TFLOP/s', 'mfma'),
        # fp16x3 Newton updates: fp32-equivalent flops against the fp16 peak / 3
        'chol_update32': (2516.6 / 3, 'TFLOP/s', 'mfma')}


def stress_data(n, d, seed):
    """synthetic_gp_data's recipe (X ~ N(0,1) normalised, y = sign of a GP prior draw at
    log tau_k = log sqrt(d)), with the squared distances from one BLAS product so that data
    preparation at N=16384 takes seconds (host data preparation, not the measured path)."""
    rng = np.random.RandomState(seed)
    X, _, _ = normalise_inputs(rng.normal(size=(n, d)))
    Z = X / np.sqrt(d)
    sq = (Z * Z).sum(1)
    K = Z.dot(Z.T)
    K *= -2.
    K += sq[:, None]
    K += sq[None, :]
    np.maximum(K, 0., out=K)
    K *= -0.5
    np.exp(K, out=K)
    K[np.diag_indices(n)] += 1e-6
    f = np.linalg.cholesky(K).dot(rng.normal(size=n))
    del K
    return X, np.where(f >= 0, 1., -1.)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=16384)
    ap.add_argument('--d', type=int, default=64)
    ap.add_argument('--s', type=int, default=1024)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--reps', type=int, default=2)
    ap.add_argument('--check', type=int, default=0)
    ap.add_argument('--seed', type=int, default=20151009)
    a = ap.parse_args()

    t0 = time.perf_counter()
    X, y = stress_data(a.n, a.d, a.seed)
    t_data = time.perf_counter() - t0
    B = a.batch
    ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, a.s, max_batch=B, n_slots=B,
                          n_ubufs=B + 1)
    rng = np.random.RandomState(a.seed + 1)
    th = np.tile(np.r_[0.0, np.full(a.d, np.log(np.sqrt(a.d)))], (B, 1))
    th += rng.normal(scale=0.1, size=th.shape)
    U0 = rng.normal(size=(a.n, a.s))  # chain 0's draws come from the host (oracle check)
    ctx.u_upload(0, U0)
    if B > 1:
        ctx.u_normal(np.arange(1, B), np.full(B - 1, 7), np.arange(1, B))
    U1 = rng.normal(size=(a.n, a.s))
    ctx.u_upload(B, U1)
    idx = np.arange(B)
    reps = []
    for r in range(a.reps):
        if r == a.reps - 1:
            for k in range(5):
                ctx.prof_read(k, reset=True)
            ctx.prof_enable(2)
        t0 = time.perf_counter()
        out, st, nops = ctx.theta_eval(_native.EST_IS, th, idx, idx)
        t1 = time.perf_counter()
        out2, st2 = ctx.u_eval(idx, idx)
        t2 = time.perf_counter()
        reps.append({'theta_call_ms': 1e3 * (t1 - t0), 'u_call_ms': 1e3 * (t2 - t1)})
        print('rep {0}: theta-call {1:.1f} ms, u-call {2:.2f} ms, status {3}'
              .format(r, 1e3 * (t1 - t0), 1e3 * (t2 - t1), st.tolist()), file=sys.stderr,
              flush=True)
    ctx.prof_enable(False)
    _, n_rerun, n_refine = ctx.prof_read(_native.PROF_STATS, reset=True)
    kern = {}
    for k, name in enumerate(('gram', 'chol_update', 'ugemm', 'chol_update32')):
        ms, cnt, wk = ctx.prof_read(k)
        if not cnt:
            continue
        peak, unit, bound = PEAK[name]
        ach = wk / (ms * 1e-3) / 1e12
        kern[name] = {'launches': cnt, 'total_ms': ms, 'avg_launch_us': 1e3 * ms / cnt,
                      'achieved': ach, 'peak': peak, 'unit': unit, 'bound': bound,
                      'frac': ach / peak}
    res = {'config': 'BASELINE.json configs[4]: synthetic N={0} D={1} N_imp={2}, ARD-SE, '
                     'ApproxPosteriorIS theta-call + cached u-call, {3} chains batched'
                     .format(a.n, a.d, a.s, B),
           'n': a.n, 'd': a.d, 'n_imp': a.s, 'batch': B, 'data_prep_s': t_data,
           'theta_call_ms': reps[-1]['theta_call_ms'], 'u_call_ms': reps[-1]['u_call_ms'],
           'theta_calls_per_s': B / (reps[-1]['theta_call_ms'] * 1e-3),
           'status': st.tolist(), 'n_cubic_ops': nops.tolist(), 'log_f': out.tolist(),
           'newton_refinement_steps': int(n_refine), 'newton_fp64_reruns': int(n_rerun),
           'kernels': kern}

    if a.check:
        import threading
        import apm_oracle as orc
        done = threading.Event()

        def heartbeat():  # gpurun treats 3 silent minutes as a hang
            t = time.perf_counter()
            while not done.wait(30.):
                print('oracle check running, {0:.0f} s'.format(time.perf_counter() - t),
                      file=sys.stderr, flush=True)
        threading.Thread(target=heartbeat, daemon=True).start()
        ctx.u_upload(0, U1)  # u-call of chain 0 with the second host draw set
        o_u, _ = ctx.u_eval([0], [0])
        L, f, g, cst = ctx.slot_read(0)
        kf = orc.make_kernel_func('ard', 1e-8)
        t0 = time.perf_counter()
        r1, rc, cubic = orc.is_estimate(X, y, kf, U0, th[0])
        t1 = time.perf_counter()
        r2, _, _ = orc.is_estimate(X, y, kf, U1, None, rc)
        t2 = time.perf_counter()
        tol = lambda r: 2e-3 + 2e-5 * abs(r)  # noqa: E731  
        dC = np.abs(L - rc[1]).max() / np.abs(rc[1]).max()
        df = np.abs(f - rc[2]).max() / max(1., np.abs(rc[2]).max())
        res['check'] = {
            'oracle_theta_call': r1, 'gpu_theta_call': out[0], 'd_theta_call': out[0] - r1,
            'oracle_u_call': r2, 'gpu_u_call': float(o_u[0]), 'd_u_call': float(o_u[0]) - r2,
            'tolerance_theta_call': tol(r1), 'tolerance_u_call': tol(r2),
            'C_chol_max_abs_err_rel_to_max': dC, 'f_post_max_err': df,
            'n_cubic_ops_oracle': int(cubic), 'n_cubic_ops_gpu': int(nops[0]),
            'oracle_theta_call_s': t1 - t0, 'oracle_u_call_s': t2 - t1,
            'pass': bool(abs(out[0] - r1) <= tol(r1) and abs(o_u[0] - r2) <= tol(r2)
                         and int(cubic) == int(nops[0]) and df < 1e-8 and dC < 1e-5)}
        done.set()
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == '__main__':
    main()

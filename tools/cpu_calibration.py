"""Calibrate the CPU baseline: the oracle's restatement (oracle/apm_oracle.py: C Gram + scipy
LAPACK, the reference's op order) against the reference itself (imported from /root/reference,
kernels.pyx compiled by `make -C oracle ref`), both on this container's cores, at the bench size
(N=4096, D=32, N_imp=256, ARD: theta-call and cached u-call) and at configs[0] (PM-MH, iso,
N=768, D=8, N_imp=1: iterations/s of the notebook's PM-MH main phase).

Build container only (the reference does not exist on the GPU box). Writes
profiles/r02_cpu_calibration.json, which bench.py attaches to its cpu_baseline (SURVEY.md §8d:
port/reference ratio, target 0.8-1.25).

    python tools/cpu_calibration.py [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tests', 'golden'), os.path.join(REPO, 'oracle')]
import make_golden as mg  # noqa: E402  (imports the reference, read-only, no bytecode)
import apm_oracle as orc  # noqa: E402


def _repo_utils():
    """this repo's gpdemo/utils.py (the name `gpdemo` is the reference's package here)"""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        'apm_repo_utils', os.path.join(REPO, 'auxiliary-pm-mcmc_amd', 'gpdemo', 'utils.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


synthetic_gp_data = _repo_utils().synthetic_gp_data


def timed(fn, reps):
    ts = []
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--out', default=os.path.join(REPO, 'profiles', 'r02_cpu_calibration.json'))
    a = ap.parse_args()
    from threadpoolctl import threadpool_info
    blas = max([i.get('num_threads', 1) for i in threadpool_info()
                if i.get('user_api') == 'blas'] or [1])
    res = {'host': 'build container', 'cores_visible': len(os.sched_getaffinity(0)),
           'blas_threads': blas, 'reps': a.reps}
    # bench size (configs[2])
    n, d, s = 4096, 32, 256
    X, y = synthetic_gp_data(n, d, 20151009)
    th = np.r_[0.0, np.full(d, np.log(np.sqrt(d)))]
    ns = np.random.RandomState(0).normal(size=(n, s))
    ref = mg.ref_est.LogMarginalLikelihoodApproxPosteriorISEstimator(
        X, y, mg.kfunc('ard', 1e-8), mg.ref_lpa.laplace_approximation)
    port = orc.ISEstimatorCPU(X, y, orc.make_kernel_func('ard', 1e-8, impl='c'))
    out = {}
    for name, e in (('reference', ref), ('port', port)):
        tt, tts, (v, cache) = timed(lambda: e(ns, th), a.reps)
        tu, tus, _ = timed(lambda: e(ns, None, cache), a.reps)
        out[name] = {'theta_call_s': tt, 'theta_call_s_all': tts, 'u_call_s': tu,
                     'u_call_s_all': tus, 'value': float(v)}
    res['configs2'] = dict(out, workload='ApproxPosteriorIS ARD N=4096 D=32 N_imp=256',
                           ratio_port_over_reference_theta_call=out['port']['theta_call_s'] /
                           out['reference']['theta_call_s'],
                           ratio_port_over_reference_u_call=out['port']['u_call_s'] /
                           out['reference']['u_call_s'])
    # configs[0]: PM-MH iso N=768 D=8 N_imp=1, theta-call per iteration (fresh u each)
    X1, y1 = synthetic_gp_data(768, 8, 20151009, 'iso')
    th1 = np.r_[0.0, np.log(np.sqrt(8.))]
    ref1 = mg.ref_est.LogMarginalLikelihoodApproxPosteriorISEstimator(
        X1, y1, mg.kfunc('iso', 1e-8), mg.ref_lpa.laplace_approximation)
    port1 = orc.ISEstimatorCPU(X1, y1, orc.make_kernel_func('iso', 1e-8, impl='c'))
    rng = np.random.RandomState(1)
    c0 = {}
    for name, e in (('reference', ref1), ('port', port1)):
        t, ts, _ = timed(lambda: e(rng.normal(size=(768, 1)), th1), 5 * a.reps)
        c0[name] = {'theta_call_s': t, 'iters_per_s': 1.0 / t}
    res['configs0'] = dict(c0, workload='PM-MH iteration = one ApproxPosteriorIS theta-call, '
                                        'iso N=768 D=8 N_imp=1',
                           ratio_port_over_reference=c0['port']['theta_call_s'] /
                           c0['reference']['theta_call_s'])
    json.dump(res, open(a.out, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()

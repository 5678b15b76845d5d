"""Long-chain ESS / R-hat record (Analyse results.ipynb:138-141, E-SS+RD-SS.ipynb:64):
C independent APM E-SS(u) + RD-SS(theta) chains at BASELINE configs[2] (N=4096 D=32 ARD, N_imp=256)
on one MI355X, 500 warm-up transitions per chain discarded, >= 2000 kept; coda effectiveSize and
gelman.diag restated (auxpm/diagnostics.py) on the kept draws; wall time of the kept segment.

    python tools/ess_long.py [--chains 16 --warmup 500 --keep 2000] > out.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--chains', type=int, default=16)
    ap.add_argument('--warmup', type=int, default=500)
    ap.add_argument('--keep', type=int, default=2000)
    ap.add_argument('--chunk', type=int, default=100)
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--d', type=int, default=32)
    ap.add_argument('--n-imp', type=int, default=256)
    ap.add_argument('--seed', type=int, default=20151009)
    a = ap.parse_args()
    from auxpm.batched import BatchedAPMEllSSPlusRandDirSliceSampler
    from auxpm.diagnostics import effective_size, gelman_rubin
    from gpdemo.utils import synthetic_gp_data
    X, y = synthetic_gp_data(a.n, a.d, a.seed)
    prior = dict(a_tau=1., b_tau=1. / a.d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    smp = BatchedAPMEllSSPlusRandDirSliceSampler(
        X, y, a.chains, a.n_imp, prior, kernel='ard', epsilon=1e-8, w=1., max_steps_out=0,
        seed=a.seed + 1)
    smp.initialise()
    series = [[] for _ in range(a.chains)]
    t_start = time.perf_counter()
    t_keep = None
    total = a.warmup + a.keep
    have = 0
    while have < total:
        if have == a.warmup:
            t_keep = time.perf_counter()
        step = min(a.chunk, (a.warmup if have < a.warmup else total) - have)
        tr, done = smp.run_async(step)
        for c in range(a.chains):
            series[c].extend(tr[c])
        have += step
        print('{0} / {1} transitions per chain, {2:.0f} s'.format(
            have, total, time.perf_counter() - t_start), file=sys.stderr, flush=True)
    wall_keep = time.perf_counter() - t_keep
    live = [c for c in range(a.chains) if not smp.failed[c]]
    kept = np.stack([np.array(series[c][a.warmup:total]) for c in live])   # (C, keep, P)
    ess = np.stack([effective_size(kept[q]) for q in range(len(live))])     # (C, P)
    rhat = gelman_rubin(kept)
    out = {
        'what': 'long-chain ESS / R-hat at BASELINE configs[2] (SURVEY.md §8d protocol)',
        'config': {'n_data': a.n, 'n_features': a.d, 'n_imp': a.n_imp, 'chains': a.chains,
                   'warmup_discarded': a.warmup, 'kept_per_chain': a.keep, 'seed': a.seed},
        'failed_chains': int(smp.failed.sum()),
        'wall_s_kept_segment': wall_keep,
        'transitions_per_s_kept_segment': len(live) * a.keep / wall_keep,
        'ess_min_per_chain_mean': float(ess.min(1).mean()),
        'ess_min_per_chain_median': float(np.median(ess.min(1))),
        'ess_mean_per_chain_mean': float(ess.mean(1).mean()),
        'ess_per_transition_min_component': float(ess.min(1).mean() / a.keep),
        'ess_per_sec_min_component': float(ess.min(1).sum() / wall_keep),
        'ess_per_sec_mean_component': float(ess.mean(1).sum() / wall_keep),
        'rhat_max': float(rhat.max()), 'rhat_median': float(np.median(rhat)),
        'rhat_theta0_log_sigma': float(rhat[0]),
        'posterior_mean_log_sigma': float(kept[:, :, 0].mean()),
        'method': 'coda effectiveSize / gelman.diag restatements (auxpm/diagnostics.py); ESS per '
                  'chain = min (or mean) over the theta components; ESS/s = sum over chains / '
                  'wall time of the kept segment',
    }
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()

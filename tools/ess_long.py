"""Long-chain ESS / R-hat record (Analyse results.ipynb:138-141, E-SS+RD-SS.ipynb:64):
C independent APM E-SS(u) + RD-SS(theta) chains at BASELINE configs[2] (N=4096 D=32 ARD, N_imp=256)
on one MI355X, `--warmup` transitions per chain discarded; coda effectiveSize and gelman.diag
restated (auxpm/diagnostics.py) on the kept draws, with the R-hat trajectory over the run.

The run is split into segments of at most `--max-seconds` of sampling (one gpurun call each):
every segment writes the chains' checkpoint (auxpm.batched ``checkpoint``: host state + the u
history, no u arrays) and its own theta draws (float32) to `--out-dir`; the next segment is started
with `--resume-dir` pointing at a directory holding all earlier segments' files, rebuilds u on the
device, checks that the recomputed current estimates equal the saved ones, and continues the same
chains. The summary covers every segment so far.

    python tools/ess_long.py --chains 64 --max-seconds 1000 --out-dir gpurun_out/ess_seg0
    python tools/ess_long.py --chains 64 --resume-dir ess_state --out-dir gpurun_out/ess_seg1
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def lib_digest(native):
    """SHA-256 (16 hex) of the libapm.so this segment ran on."""
    import hashlib
    path = os.path.abspath(native.LIB_PATH)
    if not os.path.exists(path):
        return {'path': os.path.relpath(path, REPO), 'sha16': None}
    with open(path, 'rb') as f:
        return {'path': os.path.relpath(path, REPO), 'sha16': hashlib.sha256(f.read()).hexdigest()[:16]}


def library_rate(meta):
    """Sampling throughput of the segments run on the newest library (meta 'libs' lists the
    last segments' libraries): the stationary transitions/s of that build."""
    libs = meta.get('libs') or []
    if not libs or libs[-1].get('sha16') is None:
        return {}
    sha = libs[-1]['sha16']
    k0 = len(meta['seg_walls']) - len(libs)
    idx = [k0 + i for i, l in enumerate(libs) if l.get('sha16') == sha]
    t = sum(meta['seg_transitions'][i] for i in idx)
    w = sum(meta['seg_walls'][i] for i in idx)
    return {'latest_library': {'sha16': sha, 'segments': idx, 'transitions': int(t),
                               'wall_s': w, 'transitions_per_s': t / w if w > 0 else None}}


def load_series(dirs):
    """All segments' draws per chain, in segment order: a list of (T_c, P) float64 arrays
    (segments run in the 'finish' throughput mode hold ragged rows, padded with NaN)."""
    files = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, 'series_seg*.npy')):
            files[os.path.basename(f)] = f
    parts = [np.load(files[k]) for k in sorted(files)]
    if not parts:
        return None, 0
    chains = []
    for c in range(parts[0].shape[0]):
        rows = [p[c][~np.isnan(p[c]).any(axis=1)] for p in parts]
        chains.append(np.concatenate(rows, axis=0).astype(np.float64))
    return chains, len(parts)


def summarise(chains, live, warmup, seg_walls, seg_transitions, cfg):
    from auxpm.diagnostics import effective_size, gelman_rubin
    T = min(chains[c].shape[0] for c in live)  # common length of the live chains
    series = np.stack([chains[c][:T] for c in range(len(chains)) if c in set(live)])
    kept = series[:, warmup:T]
    keep = kept.shape[1]
    traj = []
    step = 500
    for L in list(range(step, keep, step)) + [keep]:
        r = gelman_rubin(kept[:, :L])
        traj.append({'kept_per_chain': int(L), 'transitions_per_chain': int(warmup + L),
                     'rhat_max': float(r.max()), 'rhat_median': float(np.median(r))})
    ess = np.stack([effective_size(kept[q]) for q in range(kept.shape[0])])  # (C, P)
    rhat = gelman_rubin(kept)
    crossed = next((t['transitions_per_chain'] for t in traj if t['rhat_max'] < 1.1), None)
    wall = float(sum(seg_walls))
    ntr = int(sum(seg_transitions))
    tps = ntr / wall if wall > 0 else None
    ept_min = float(ess.min(1).mean() / keep)
    ept_mean = float(ess.mean(1).mean() / keep)
    # the same per chain over all of its draws (chains that ran ahead in the 'finish' mode)
    full = [chains[c][warmup:] for c in live]
    ept_all = float(np.mean([effective_size(x).min() / x.shape[0] for x in full]))
    seg_tps = [t / w if w > 0 else None for t, w in zip(seg_transitions, seg_walls)]
    return {
        'what': 'long-chain ESS / R-hat at BASELINE configs[2] (SURVEY.md §8d protocol), '
                'checkpointed segments on one MI355X',
        'transitions_per_s_by_segment': seg_tps,
        'config': cfg,
        'segments': len(seg_walls),
        'failed_chains': int(len(chains) - len(live)),
        'transitions_per_chain': int(T), 'warmup_discarded': int(warmup), 'kept_per_chain': int(keep),
        'transitions_per_chain_max': int(max(chains[c].shape[0] for c in live)),
        'sampling_wall_s': wall,
        'transitions_per_s_sampling': tps,
        'ess_min_per_chain_mean': float(ess.min(1).mean()),
        'ess_min_per_chain_median': float(np.median(ess.min(1))),
        'ess_mean_per_chain_mean': float(ess.mean(1).mean()),
        'ess_per_transition_min_component': ept_min,
        'ess_per_transition_mean_component': ept_mean,
        'ess_per_transition_min_component_worst_chain': float(ess.min(1).min() / keep),
        'ess_per_transition_min_component_all_draws': ept_all,
        'kept_per_chain_all_draws_mean': float(np.mean([x.shape[0] for x in full])),
        'ess_per_sec_min_component': ept_min * tps if tps else None,
        'ess_per_sec_mean_component': ept_mean * tps if tps else None,
        'rhat_max': float(rhat.max()), 'rhat_median': float(np.median(rhat)),
        'rhat_argmax_component': int(rhat.argmax()),
        'rhat_theta0_log_sigma': float(rhat[0]),
        'rhat_below_1p1_at_transitions_per_chain': crossed,
        'rhat_trajectory': traj,
        'posterior_mean_log_sigma': float(kept[:, :, 0].mean()),
        'method': 'coda effectiveSize / gelman.diag restatements (auxpm/diagnostics.py) on the '
                  'kept draws of every live chain; ESS per transition = mean over chains of the '
                  'min (or mean) over the 33 theta components of ESS / kept length; ESS/s = that '
                  'x the sampling throughput (all chains, all segments: transitions / wall)',
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--chains', type=int, default=64)
    ap.add_argument('--warmup', type=int, default=500)
    ap.add_argument('--target', type=int, default=9000, help='transitions per chain in total')
    ap.add_argument('--chunk', type=int, default=100)
    ap.add_argument('--max-seconds', type=float, default=1000.)
    ap.add_argument('--resume-dir', default=None)
    ap.add_argument('--out-dir', default=None)
    ap.add_argument('--summarise', default=None, metavar='DIR',
                    help='no sampling: rewrite DIR/summary.json from every series_seg*.npy, '
                         'meta.json and state.npz in DIR (CPU only; a resume directory may hold '
                         'the state alone, so that only it travels to the GPU box)')
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--d', type=int, default=32)
    ap.add_argument('--n-imp', type=int, default=256)
    ap.add_argument('--seed', type=int, default=20151009)
    ap.add_argument('--restore-tol', type=float, default=1e-9,
                    help='largest |d log f| accepted on resume (a different build of libapm.so '
                         'continues the chains with its own rounding: ~1e-5 nats)')
    a = ap.parse_args()
    cfg = {'n_data': a.n, 'n_features': a.d, 'n_imp': a.n_imp, 'chains': a.chains,
           'seed': a.seed, 'kernel': 'ard', 'epsilon': 1e-8, 'w': 1., 'max_steps_out': 0}
    if a.summarise:
        with open(os.path.join(a.summarise, 'meta.json')) as f:
            meta = json.load(f)
        chains, _ = load_series([a.summarise])
        with np.load(os.path.join(a.summarise, 'state.npz')) as z:
            failed = z['failed'] if 'failed' in z.files else np.zeros(len(chains), bool)
        live = [c for c in range(len(chains)) if not failed[c]]
        out = summarise(chains, live, a.warmup, meta['seg_walls'], meta['seg_transitions'], cfg)
        out['restore_max_abs_dlogf'] = meta['restore_dlogf']
        out['segment_libs'] = meta.get('libs')
        out.update(library_rate(meta))
        with open(os.path.join(a.summarise, 'summary.json'), 'w') as f:
            json.dump(out, f, indent=1)
        print(json.dumps({k: out[k] for k in ('transitions_per_chain', 'rhat_max', 'rhat_median',
                                              'ess_per_transition_min_component')}))
        return
    from auxpm.batched import BatchedAPMEllSSPlusRandDirSliceSampler
    from gpdemo.utils import synthetic_gp_data
    os.makedirs(a.out_dir, exist_ok=True)
    t_start = time.perf_counter()
    X, y = synthetic_gp_data(a.n, a.d, a.seed)
    prior = dict(a_tau=1., b_tau=1. / a.d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    smp = BatchedAPMEllSSPlusRandDirSliceSampler(
        X, y, a.chains, a.n_imp, prior, kernel='ard', epsilon=1e-8, w=1., max_steps_out=0,
        seed=a.seed + 1)
    dirs = [a.resume_dir] if a.resume_dir else []
    prev, n_seg = load_series(dirs)
    have = np.zeros(a.chains, dtype=np.int64) if prev is None else \
        np.array([x.shape[0] for x in prev], dtype=np.int64)
    meta = {'seg_walls': [], 'seg_transitions': []}
    restore_dlogf = None
    if a.resume_dir:
        with np.load(os.path.join(a.resume_dir, 'state.npz')) as z:
            ck = {k: z[k] for k in z.files}
        with open(os.path.join(a.resume_dir, 'meta.json')) as f:
            meta = json.load(f)
        n_seg = len(meta['seg_walls'])  # (a state-only directory holds no series files)
        ck_have = np.broadcast_to(np.asarray(ck['transitions_per_chain'], np.int64), have.shape)
        if prev is None:  # a state-only resume directory
            have = ck_have.copy()
        if not np.array_equal(ck_have, have):
            raise RuntimeError('checkpoint at {0} transitions, series hold {1}'.format(
                ck_have.tolist(), have.tolist()))
        restore_dlogf = smp.restore(ck)
        print('resumed at {0} transitions per chain; max |d log f| on restore {1:.3g} ({2:.0f} s)'
              .format(int(have.min()), restore_dlogf, time.perf_counter() - t_start),
              file=sys.stderr, flush=True)
        if not restore_dlogf <= a.restore_tol:
            raise RuntimeError('restored chains differ from the checkpoint: {0}'.format(restore_dlogf))
    else:
        smp.initialise()
    seg = [[] for _ in range(a.chains)]
    t0 = time.perf_counter()
    done_here = np.zeros(a.chains, dtype=np.int64)
    last = 0.0  # duration of the previous chunk: no chunk is started that would overrun
    cur = have.copy()

    def slowest():  # the live chains' smallest count (failed chains stop where they failed)
        live = ~smp.failed
        return int(cur[live].min()) if live.any() else a.target
    while slowest() < a.target and time.perf_counter() - t0 + last < a.max_seconds:
        tc = time.perf_counter()
        # every chain to (at least) the slowest one's count + chunk: chains that are ahead keep
        # working while the batch waits for the slowest ('finish' throughput mode)
        step = np.maximum(min(slowest() + a.chunk, a.target) - cur, 0)
        beat = [time.perf_counter()]

        def heartbeat(done):  # a line a minute inside long chunks (gpurun's hang detection)
            if time.perf_counter() - beat[0] > 60:
                beat[0] = time.perf_counter()
                print('  ... chunk: {0} of {1} chains at their target'.format(
                    int((done >= step).sum()), len(done)),
                      file=sys.stderr, flush=True)
        tr, done = smp.run_async(step, keep_going='finish', on_round=heartbeat)
        for c in range(a.chains):
            seg[c].extend(tr[c])
        done_here += done
        cur = have + done_here
        last = time.perf_counter() - tc
        print('{0} .. {1} / {2} transitions per chain, segment {3:.0f} s'.format(
            int(cur.min()), int(cur.max()), a.target, time.perf_counter() - t0),
            file=sys.stderr, flush=True)
    wall = time.perf_counter() - t0
    live = [c for c in range(a.chains) if not smp.failed[c]]
    meta['seg_walls'].append(wall)
    meta['seg_transitions'].append(int(done_here[live].sum()))
    meta.setdefault('restore_dlogf', []).append(restore_dlogf)
    from gpdemo import _native
    meta.setdefault('libs', []).append(lib_digest(_native))
    arr = np.full((a.chains, max(1, max(len(x) for x in seg)), smp.P), np.nan, dtype=np.float32)
    for c in range(a.chains):
        if seg[c]:
            arr[c, :len(seg[c])] = np.array(seg[c], dtype=np.float32)
    np.save(os.path.join(a.out_dir, 'series_seg{0:02d}.npy'.format(n_seg)), arr)
    ck = smp.checkpoint()
    ck['transitions_per_chain'] = (have + done_here).astype(np.int64)
    np.savez(os.path.join(a.out_dir, 'state.npz'), **ck)
    with open(os.path.join(a.out_dir, 'meta.json'), 'w') as f:
        json.dump(meta, f)
    if a.resume_dir and prev is None:  # state-only resume: the summary needs every segment
        print('segment {0} written; merge it into the full directory and run --summarise'.format(
            n_seg), file=sys.stderr, flush=True)
        return
    chains, _ = load_series(dirs + [a.out_dir])
    out = summarise(chains, live, a.warmup, meta['seg_walls'], meta['seg_transitions'], cfg)
    out['restore_max_abs_dlogf'] = meta['restore_dlogf']
    out['segment_libs'] = meta.get('libs')
    out.update(library_rate(meta))
    with open(os.path.join(a.out_dir, 'summary.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ('transitions_per_chain', 'rhat_max', 'rhat_median',
                                          'ess_per_transition_min_component',
                                          'transitions_per_s_sampling')}), flush=True)


if __name__ == '__main__':
    main()

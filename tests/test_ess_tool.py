"""tools/ess_long.py bookkeeping on the CPU (no GPU): a stand-in sampler with the batched
driver's interface (run_async in the 'finish' mode returns ragged per-chain traces) drives a first
segment, a resume from a state-only directory (what travels to the GPU box), the merge and the
--summarise pass; the summary covers every chain's series at the common length."""
import json
import os
import runpy
import shutil
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(REPO, 'tools', 'ess_long.py')


class _Stand(object):
    """AR(1) chains with the batched sampler's surface (initialise / run_async / checkpoint /
    restore / failed / theta / P)."""

    def __init__(self, X, y, C, S, prior, **kw):
        self.n_chains, self.P = C, X.shape[1] + 1
        self.rng = np.random.RandomState(kw['seed'])
        self.failed = np.zeros(C, bool)
        self.theta = np.zeros((C, self.P))

    def initialise(self):
        pass

    def checkpoint(self):
        return {'theta': self.theta.copy(), 'failed': self.failed.copy(),
                'rng': np.array(self.rng.get_state()[1])}

    def restore(self, ck):
        self.theta = np.array(ck['theta'])
        return 0.0

    def run_async(self, n_steps, keep_going=False, on_round=None):
        assert keep_going == 'finish'
        n = np.broadcast_to(np.asarray(n_steps), (self.n_chains,))
        done = n + self.rng.randint(0, 4, self.n_chains)  # chains ahead keep working
        tr = []
        for c in range(self.n_chains):
            t = []
            for _ in range(done[c]):
                self.theta[c] = 0.9 * self.theta[c] + self.rng.normal(size=self.P)
                t.append(self.theta[c].copy())
            tr.append(t)
        if on_round:
            on_round(done)
        return tr, done


def _run(monkeypatch, *args):
    import auxpm.batched as B
    import gpdemo.utils as U
    monkeypatch.setattr(B, 'BatchedAPMEllSSPlusRandDirSliceSampler', _Stand)
    monkeypatch.setattr(U, 'synthetic_gp_data', lambda n, d, s: (np.zeros((n, d)), np.zeros(n)))
    monkeypatch.setattr(sys, 'argv', ['ess_long.py', '--chains', '5', '--chunk', '40',
                                      '--warmup', '30', '--n', '8', '--d', '3'] + list(args))
    runpy.run_path(TOOL, run_name='__main__')


def test_segments_state_only_resume_and_summary(monkeypatch, tmp_path):
    pytest.importorskip('scipy')
    s0, push, s1, full = (str(tmp_path / x) for x in ('s0', 'push', 's1', 'full'))
    _run(monkeypatch, '--target', '120', '--out-dir', s0)
    os.makedirs(push)
    for f in ('state.npz', 'meta.json'):
        shutil.copy(os.path.join(s0, f), push)
    _run(monkeypatch, '--target', '300', '--resume-dir', push, '--out-dir', s1)
    assert sorted(os.listdir(s1)) == ['meta.json', 'series_seg01.npy', 'state.npz']
    shutil.copytree(s0, full)
    for f in os.listdir(s1):
        shutil.copy(os.path.join(s1, f), full)
    _run(monkeypatch, '--summarise', full)
    out = json.load(open(os.path.join(full, 'summary.json')))
    lens = [np.load(os.path.join(full, f)) for f in ('series_seg00.npy', 'series_seg01.npy')]
    per_chain = [sum(int((~np.isnan(a[c]).any(1)).sum()) for a in lens) for c in range(5)]
    with np.load(os.path.join(full, 'state.npz')) as z:
        assert list(z['transitions_per_chain']) == per_chain
    assert out['segments'] == 2 and out['transitions_per_chain'] == min(per_chain) >= 300
    assert out['transitions_per_chain_max'] == max(per_chain)
    assert out['kept_per_chain'] == min(per_chain) - 30
    assert out['rhat_trajectory'][-1]['kept_per_chain'] == out['kept_per_chain']
    assert 0 < out['ess_per_transition_min_component'] <= out['ess_per_transition_mean_component']
    # a checkpoint that does not match the series it is resumed with is refused
    with open(os.path.join(push, 'meta.json')) as f:
        json.load(f)
    bad = str(tmp_path / 'bad')
    shutil.copytree(s0, bad)
    shutil.copy(os.path.join(s1, 'state.npz'), bad)
    with pytest.raises(RuntimeError):
        _run(monkeypatch, '--target', '400', '--resume-dir', bad, '--out-dir', str(tmp_path / 'x'))

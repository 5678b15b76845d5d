"""The N>1 path of bench.py on hardware: two ranks under torch.distributed.run (gloo bookkeeping,
one process per rank, each with its own device context and chain seeds), both pinned to the
box's single GPU with APM_DEVICE=0 (on an 8-GPU node each rank takes GPU LOCAL_RANK). The rank-0
JSON line must aggregate both ranks: n_gpus 2, transitions summed, no failed chain, and a
max-over-ranks time. Also BASELINE.json configs[3]'s per-rank share (64 chains at N=4096 per
GPU) for ranks 0..7 is exercised by the bench itself; here the 8 rank seeds are checked for
disjoint streams and one chain of two different ranks' batches for state consistency."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import apm_oracle as orc

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_on_one_gpu(gpu_available):
    env = dict(os.environ, APM_DEVICE='0', MASTER_ADDR='127.0.0.1')
    out = subprocess.run(
        [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
         '--master-addr', '127.0.0.1', '--master-port', '29561', os.path.join(REPO, 'bench.py'),
         '--gpus', '2', '--steps', '4', '--warmup', '1', '--chains', '4', '--n-data', '1024',
         '--n-features', '8', '--n-imp', '32', '--cpu-baseline', '0'],
        capture_output=True, text=True, env=env, timeout=500, cwd=REPO)
    assert out.returncode == 0, out.stdout[-4000:] + out.stderr[-2000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith('{')][-1])
    assert line['n_gpus'] == 2 and line['config']['global_batch'] == 8
    assert line['failed_chains'] == 0
    assert line['transitions_timed'] >= 2 * 4 * 4
    assert line['value'] > 0 and line['ms_per_step'] > 0
    assert line['ess_sample']['chains'] == 8
    # both ranks' GPU values checked against rank 0's oracle (gathered over gloo)
    assert line['parity']['pass'] and line['parity']['checked_ranks'] == 2
    assert line['parity']['vs_reference']['used'] is False  # N=1024: not the fixture's workload
    assert [r['rank'] for r in line['ranks']] == [0, 1]
    assert sum(r['transitions'] for r in line['ranks']) == line['transitions_timed']


def test_config3_rank_shares_consistent(gpu_available):
    """Two of configs[3]'s eight per-GPU shares (ranks 0 and 7: 64 chains each at N=4096, D=32,
    N_imp=256, the bench's data and rank seeds): one initial theta-call and one transition of
    every chain, finite and failure-free, and chain 0 of each share consistent with the oracle
    (its u downloaded from the device)."""
    import bench
    from auxpm.batched import BatchedAPMEllSSPlusRandDirSliceSampler, chain_streams
    from gpdemo.utils import synthetic_gp_data
    n, d, s = 4096, 32, 256
    X, y = synthetic_gp_data(n, d, 20151009)
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    keys = [chain_streams(bench.chain_seed(20151009, r), 64)[1] for r in range(8)]
    assert len(set(np.concatenate(keys).tolist())) == 8 * 64
    kf = orc.make_kernel_func('ard', 1e-8)
    for rank in (0, 7):
        smp = BatchedAPMEllSSPlusRandDirSliceSampler(
            X, y, 64, s, prior, kernel='ard', epsilon=1e-8, w=1., max_steps_out=0,
            seed=bench.chain_seed(20151009, rank), device=0)
        smp.initialise()
        traces, done = smp.run_async(1)
        assert not smp.failed.any() and (done == 1).all()
        assert np.isfinite(smp.log_f).all()
        c = 0
        U = smp.ctx.u_download(smp.ub_u[c])
        v, _, _ = orc.is_estimate(X, y, kf, U, smp.theta[c])
        lp = smp.log_prior(smp.theta[c][None])[0]
        assert abs(smp.log_f[c] - (v + lp)) <= 5e-4, (rank, smp.log_f[c], v + lp)
        smp.ctx.close()

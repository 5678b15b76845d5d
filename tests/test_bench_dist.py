"""The bench's N>1 bookkeeping (barrier, max-over-ranks time, sum of units) over gloo,
world_size 2, on CPU — the multi-GPU path has no data-path collective, only these."""
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dist_bookkeeping_gloo_world2(tmp_path):
    script = tmp_path / 'w.py'
    script.write_text(textwrap.dedent('''
        import os, sys, time
        sys.path.insert(0, {repo!r})
        import bench
        d = bench.Dist(backend='gloo')
        work = lambda: time.sleep(0.05 * (d.rank + 1))
        el = bench.timed_region(d, work, 2)
        tot = d.sum(10 * (d.rank + 1))
        if d.rank == 0:
            print('RESULT', el, tot, d.world)
        d.close()
    ''').format(repo=REPO))
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    out = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
                          '--nproc-per-node=2', '--master-addr', '127.0.0.1', '--master-port',
                          '29533', str(script)], capture_output=True, text=True, env=env,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith('RESULT')][0].split()
    el, tot, world = float(line[1]), float(line[2]), int(line[3])
    assert world == 2 and tot == 30.0
    assert el >= 0.19  # max over ranks: rank 1 sleeps 2 x 0.1 s


def test_rank_streams_disjoint_gloo_world2(tmp_path):
    """Each rank of `bench.py --gpus 2` drives device LOCAL_RANK with its own sampler seed
    (bench.chain_seed): the ranks' device indices differ and their 64 chains' Philox keys and
    host RandomState streams are disjoint (gathered over gloo)."""
    script = tmp_path / 's.py'
    script.write_text(textwrap.dedent('''
        import os, sys
        sys.path[:0] = [{repo!r}, os.path.join({repo!r}, 'auxiliary-pm-mcmc_amd')]
        import numpy as np, torch, torch.distributed as tdist
        import bench
        from auxpm.batched import chain_streams
        d = bench.Dist()
        prngs, keys = chain_streams(bench.chain_seed(20151009, d.rank), 64)
        first = np.array([r.randint(2 ** 31) for r in prngs], dtype=np.int64)
        mine = torch.tensor(np.r_[d.local_rank, keys.view(np.int64), first])
        allv = [torch.zeros_like(mine) for _ in range(d.world)]
        tdist.all_gather(allv, mine)
        if d.rank == 0:
            a, b = allv[0].numpy(), allv[1].numpy()
            print('RESULT', a[0], b[0], len(set(a[1:65]) & set(b[1:65])),
                  len(set(a[1:65])), len(set(a[65:]) & set(b[65:])), d.backend)
        d.close()
    ''').format(repo=REPO))
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    out = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
                          '--nproc-per-node=2', '--master-addr', '127.0.0.1', '--master-port',
                          '29534', str(script)], capture_output=True, text=True, env=env,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    r = [l for l in out.stdout.splitlines() if l.startswith('RESULT')][0].split()
    assert (r[1], r[2]) == ('0', '1')       # one GPU per rank
    assert r[3] == '0' and r[4] == '64'     # 64 distinct Philox keys per rank, none shared
    assert r[5] == '0'                      # host streams start differently on every chain
    assert r[6] == 'gloo'                   # bookkeeping never creates an RCCL communicator


def test_world8_devices_and_streams_gloo(tmp_path):
    """The 8-GPU layout of `bench.py --gpus 8` rehearsed on CPU over gloo, world size 8: each
    rank maps LOCAL_RANK to its own device (bench.rank_device: 8 distinct devices), the 8 x 64
    chains' Philox keys and host streams are pairwise disjoint, and the helpers the rank-0 line
    is built with (Dist.all_gather of the per-rank records, Dist.broadcast of the oracle values,
    max-over-ranks time, sums) agree on every rank."""
    script = tmp_path / 'w8.py'
    script.write_text(textwrap.dedent('''
        import os, sys, time
        sys.path[:0] = [{repo!r}, os.path.join({repo!r}, 'auxiliary-pm-mcmc_amd')]
        import numpy as np
        import bench
        from auxpm.batched import chain_streams
        d = bench.Dist()
        dev = bench.rank_device(d)
        prngs, keys = chain_streams(bench.chain_seed(20151009, d.rank), 64)
        first = np.array([r.randint(2 ** 31) for r in prngs], dtype=np.float64)
        rec = np.r_[d.rank, dev, keys.astype(np.float64), first]
        allr = d.all_gather(rec)
        orc = d.broadcast(np.arange(3.) * (d.rank + 1))  # rank 0's values everywhere
        el = bench.timed_region(d, lambda: time.sleep(0.02 * (d.rank + 1)), 1)
        tot = d.sum(64)
        if d.rank == 0:
            k = allr[:, 2:66]
            f = allr[:, 66:]
            print('RESULT', len(set(allr[:, 1].astype(int))), sorted(allr[:, 0].astype(int).tolist()),
                  len(set(k.ravel())), len(set(f.ravel())), orc.tolist(), el >= 0.16, tot,
                  d.backend)
        d.close()
    ''').format(repo=REPO))
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', OMP_NUM_THREADS='1')
    env.pop('APM_DEVICE', None)
    out = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
                          '--nproc-per-node=8', '--master-addr', '127.0.0.1', '--master-port',
                          '29535', str(script)], capture_output=True, text=True, env=env,
                         timeout=400)
    assert out.returncode == 0, out.stderr[-2000:]
    r = [l for l in out.stdout.splitlines() if l.startswith('RESULT')][0]
    assert r.startswith('RESULT 8 [0, 1, 2, 3, 4, 5, 6, 7] 512 512 [0.0, 1.0, 2.0] True 512.0 gloo'), r

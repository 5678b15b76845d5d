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

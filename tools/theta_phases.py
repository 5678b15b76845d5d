"""Phase timeline of the last theta-call in a rocprofv3 kernel trace of tools/time_theta.py
(development tool): Gram, Newton loop (main stream), concurrent chol(K) (second stream = the
other queue), posterior-covariance factor, slot write + L.U; wall time of each phase and the
summed kernel time per queue inside it.

usage: theta_phases.py kernel_trace.csv
"""
import collections
import csv
import sys


def main(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                     r['Kernel_Name'].split('(')[0].replace('void ', ''), r.get('Queue_Id', '0')))
    rows.sort()
    g = [i for i, r in enumerate(rows) if r[2].startswith('k_gram')][-1]
    rows = rows[g:]
    main_q = rows[0][3]
    t0 = rows[0][0]
    last_newton = max(i for i, r in enumerate(rows) if r[2].startswith('k_newton_check'))
    first_post = min(i for i, r in enumerate(rows) if i > last_newton and r[3] == main_q)
    slot = min(i for i, r in enumerate(rows) if 'slot_write' in r[2])
    end = max(i for i, r in enumerate(rows) if r[2].startswith('k_lme'))
    other = [r for r in rows if r[3] != main_q]
    phases = [('gram', rows[0][0], rows[0][1]),
              ('newton (main stream)', rows[1][0], rows[last_newton][1]),
              ('posterior factor', rows[first_post][0], rows[slot][0]),
              ('slot + L.U + LME', rows[slot][0], rows[end][1])]
    print('theta-call wall {0:.2f} ms'.format((rows[end][1] - t0) / 1e6))
    for name, a, b in phases:
        busy = collections.defaultdict(float)
        for s, e, n, q in rows:
            lo, hi = max(s, a), min(e, b)
            if hi > lo:
                busy['main' if q == main_q else 'stream2'] += (hi - lo) / 1e6
        print('{0:24s} {1:8.2f} ms  [{2:8.2f} .. {3:8.2f}]  kernel-ms main {4:7.2f} stream2 {5:7.2f}'
              .format(name, (b - a) / 1e6, (a - t0) / 1e6, (b - t0) / 1e6, busy['main'],
                      busy['stream2']))
    if other:
        print('stream2: first {0:.2f} ms, last end {1:.2f} ms, {2} kernels'.format(
            (other[0][0] - t0) / 1e6, (max(r[1] for r in other) - t0) / 1e6, len(other)))
    # Newton iterations: from one k_newton_prep to the next (the last ends at the last check)
    preps = [r[0] for r in rows[:last_newton + 1] if r[2].startswith('k_newton_prep')]
    ends = preps[1:] + [rows[last_newton][1]]
    print('newton iterations (ms): ' + ' '.join('{0:.1f}'.format((e - a) / 1e6)
                                                for a, e in zip(preps, ends)))
    post = collections.defaultdict(lambda: [0.0, 0])
    for s, e, n, q in rows[first_post:slot]:
        post[n][0] += (e - s) / 1e6
        post[n][1] += 1
    print('posterior factor kernels (main stream, ms / launches):')
    for n, (v, c) in sorted(post.items(), key=lambda x: -x[1][0])[:8]:
        print('  {0:40s} {1:8.2f} ms {2:5d}'.format(n[:40], v, c))
    top = collections.defaultdict(float)
    for s, e, n, q in rows[:end + 1]:
        top[(n, 'main' if q == main_q else 's2')] += (e - s) / 1e6
    for (n, q), v in sorted(top.items(), key=lambda x: -x[1])[:14]:
        print('  {0:40s} {1:5s} {2:8.2f} ms'.format(n[:40], q, v))


if __name__ == '__main__':
    main(sys.argv[1])

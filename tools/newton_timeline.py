"""Kernel timeline of one Newton iteration of the last theta-call in a rocprofv3 kernel trace of
tools/time_theta.py (development tool): every dispatch from the iteration's k_newton_prep to the
next, in start order, with its queue, start offset and duration (us), then per queue the busy
time and the summed time per kernel. Queues are numbered in order of first appearance in the
theta-call (0 = the main stream).

usage: newton_timeline.py kernel_trace.csv [--iter 3] [--max-rows 400]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--iter', type=int, default=3)
    ap.add_argument('--max-rows', type=int, default=400)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                     r['Kernel_Name'].split('(')[0].replace('void ', ''), r.get('Queue_Id', '0')))
    rows.sort()
    g = [i for i, r in enumerate(rows) if r[2].startswith('k_gram')][-1]
    rows = rows[g:]
    qid = {}
    for r in rows:
        qid.setdefault(r[3], len(qid))
    preps = [i for i, r in enumerate(rows) if r[2].startswith('k_newton_prep')]
    if a.iter + 1 >= len(preps):
        raise SystemExit('only {0} Newton iterations in the trace'.format(len(preps)))
    t0, t1 = rows[preps[a.iter]][0], rows[preps[a.iter + 1]][0]
    sel = [r for r in rows if r[0] < t1 and r[1] > t0]
    print('iteration {0}: {1:.1f} us, {2} dispatches'.format(a.iter, (t1 - t0) / 1e3, len(sel)))
    for k, (s, e, n, q) in enumerate(sel[:a.max_rows]):
        print('{0:9.1f} {1:8.1f}  q{2}  {3}'.format((s - t0) / 1e3, (e - s) / 1e3, qid[q], n[:60]))
    busy = collections.defaultdict(float)
    per = collections.defaultdict(lambda: [0.0, 0])
    for s, e, n, q in sel:
        lo, hi = max(s, t0), min(e, t1)
        busy[qid[q]] += (hi - lo) / 1e3
        per[(qid[q], n)][0] += (hi - lo) / 1e3
        per[(qid[q], n)][1] += 1
    for q in sorted(busy):
        print('queue {0}: busy {1:.1f} us of {2:.1f}'.format(q, busy[q], (t1 - t0) / 1e3))
    for (q, n), (v, c) in sorted(per.items(), key=lambda x: -x[1][0])[:20]:
        print('  q{0} {1:50s} {2:9.1f} us {3:5d}'.format(q, n[:50], v, c))


if __name__ == '__main__':
    main()

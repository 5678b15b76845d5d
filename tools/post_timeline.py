"""Kernel timeline of the posterior phase of the last theta-call in a rocprofv3 kernel trace of
tools/time_theta.py (development tool): every dispatch from the last k_newton_check of the call
to its k_lme, in start order, with queue, start offset and duration (us); then per queue the busy
time and the summed time per kernel.

usage: post_timeline.py kernel_trace.csv [--max-rows 400]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
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
    last = [i for i, r in enumerate(rows) if r[2].startswith('k_newton_check')][-1]
    end = [i for i, r in enumerate(rows) if r[2].startswith('k_lme')]
    end = end[0] if end else len(rows) - 1
    win = rows[last:end + 1]
    t0, t1 = win[0][0], max(r[1] for r in win)
    print('posterior phase: %.1f us, %d dispatches' % ((t1 - t0) / 1e3, len(win)))
    for r in win[:a.max_rows]:
        print('  %9.1f %9.1f  q%d  %s' % ((r[0] - t0) / 1e3, (r[1] - r[0]) / 1e3, qid[r[3]], r[2]))
    busy = collections.defaultdict(float)
    per = collections.defaultdict(lambda: [0.0, 0])
    for r in win:
        busy[qid[r[3]]] += (r[1] - r[0]) / 1e3
        k = (qid[r[3]], r[2])
        per[k][0] += (r[1] - r[0]) / 1e3
        per[k][1] += 1
    for q in sorted(busy):
        print('queue %d: busy %.1f us of %.1f' % (q, busy[q], (t1 - t0) / 1e3))
    for (q, k), (t, n) in sorted(per.items(), key=lambda x: -x[1][0]):
        print('  q%d %-50s %9.1f us %5d' % (q, k, t, n))


if __name__ == '__main__':
    main()

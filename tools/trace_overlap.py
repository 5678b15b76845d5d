"""Timeline analysis of a rocprofv3 kernel trace (development tool).

Prints per-kernel busy time, the wall time of the union of all kernels, and how much of each
kernel's time runs concurrently with some other kernel (lookahead overlap check).
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main(path, t_from=None):
    rows = []
    if path.endswith('.db'):  # rocprofv3 default (rocpd sqlite) output
        con = sqlite3.connect(path)
        for s, e, n in con.execute('select start, end, name from kernels'):
            rows.append((int(s), int(e), n.split('(')[0]))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r['Kernel_Name'].split('(')[0]
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), name))
    rows.sort()
    if t_from is not None:
        t0 = rows[0][0]
        rows = [r for r in rows if r[0] - t0 >= t_from]
    busy = defaultdict(int)
    for s, e, n in rows:
        busy[n] += e - s
    # union wall time
    wall, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                wall += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    wall += cur_e - cur_s
    # overlap of each kernel with any other kernel (sweep)
    ev = []
    for i, (s, e, n) in enumerate(rows):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    active = set()
    over = defaultdict(int)
    last = None
    for t, typ, i in ev:
        if last is not None and len(active) > 1:
            for j in active:
                over[rows[j][2]] += t - last
        last = t
        if typ == 1:
            active.add(i)
        else:
            active.discard(i)
    span = rows[-1][1] - rows[0][0]
    print('span {0:.3f} ms, union busy {1:.3f} ms, sum of kernel time {2:.3f} ms'.format(
        span / 1e6, wall / 1e6, sum(busy.values()) / 1e6))
    for n, b in sorted(busy.items(), key=lambda x: -x[1]):
        print('{0:28s} {1:10.3f} ms  overlapped {2:6.1f}%'.format(n, b / 1e6, 100.0 * over[n] / b))


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)

"""GPU idle time inside the bench's timed window of a rocprofv3 kernel trace (development tool):
the window is bracketed by the k_apm_marker<1>/<2> kernels (apm_prof_marker); prints busy and
idle time and the kernels that most often follow an idle gap."""
import collections
import csv
import sys


def main(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                     r['Kernel_Name'].split('(')[0]))
    rows.sort()
    m1 = [r for r in rows if 'marker<1>' in r[2]][0][0]
    m2 = [r for r in rows if 'marker<2>' in r[2]][0][1]
    w = [r for r in rows if r[0] >= m1 and r[1] <= m2]
    busy, gaps = 0, []
    cs, ce = w[0][0], w[0][1]
    for s, e, n in w[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print('window {0:.1f} ms  busy {1:.1f} ms  idle {2:.1f} ms ({3:.1%})'.format(
        (m2 - m1) / 1e6, busy / 1e6, (m2 - m1 - busy) / 1e6, 1 - busy / (m2 - m1)))
    g, gc = collections.Counter(), collections.Counter()
    for d, n in gaps:
        g[n] += d
        gc[n] += 1
    for n, d in g.most_common(12):
        print('  before {0:32s} {1:8.2f} ms  {2:6d} gaps  avg {3:7.1f} us'.format(
            n[:32], d / 1e6, gc[n], d / gc[n] / 1e3))


if __name__ == '__main__':
    main(sys.argv[1])

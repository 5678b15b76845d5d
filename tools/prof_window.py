"""Per-kernel statistics of the bench's timed region from rocprofv3 outputs (profiles/ helper).

The bench brackets its timed region with the empty kernels k_apm_marker<1> / <2>
(apm_prof_marker). Given a --kernel-trace CSV this prints/writes per-kernel dispatch count and
average duration inside the window (to compare with bench.py's HIP-event averages); given the
counter_collection CSVs of separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes it writes
per-dispatch HBM traffic, corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of 16-byte-per-lane reads
(x2 here); WRITE_SIZE is exact for 16-byte-per-lane stores (8-byte stores are uncalibrated).

Given the counter_collection CSV of a `--pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE` pass it
also writes per-kernel MFMA utilisation: SQ_VALU_MFMA_BUSY_CYCLES sums the busy cycles of every
MFMA over all 1024 SIMDs, GRBM_GUI_ACTIVE sums the dispatch's active cycles over the 8 XCDs
(MI355X_MICROARCH.md: DVFS note), so util = MFMA_BUSY / (1024 x GRBM_GUI_ACTIVE / 8). Counter
passes serialise dispatches (no overlap with the concurrent chol(K) stream).

usage: prof_window.py trace.csv [--fetch fetch.csv --write write.csv] [--mfma mfma.csv]
                      [--out out.json]
"""
import argparse
import collections
import csv
import json


def window(rows, key_name, key_start, key_end):
    rows = sorted(rows, key=lambda r: int(r[key_start]))
    lo = hi = None
    for r in rows:
        n = r[key_name]
        if 'k_apm_marker<1>' in n and lo is None:
            lo = int(r[key_end])
        if 'k_apm_marker<2>' in n:
            hi = int(r[key_start])
    if lo is None or hi is None:
        raise SystemExit('markers k_apm_marker<1>/<2> not found')
    return [r for r in rows if lo <= int(r[key_start]) and int(r[key_end]) <= hi]


def short(n):
    return n.split('(')[0].replace('void ', '')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--fetch')
    ap.add_argument('--write')
    ap.add_argument('--mfma')
    ap.add_argument('--out')
    ap.add_argument('--csrc-sha16', help='bench.csrc_sha16() of the profiled build')
    ap.add_argument('--commit', help='git describe of the profiled tree (build container)')
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    win = window(rows, 'Kernel_Name', 'Start_Timestamp', 'End_Timestamp')
    st = collections.defaultdict(lambda: [0, 0])
    for r in win:
        s = st[short(r['Kernel_Name'])]
        s[0] += 1
        s[1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    total = sum(v[1] for v in st.values())
    out = {'csrc_sha16': a.csrc_sha16, 'commit': a.commit, 'timed_window_kernels': {
        k: {'dispatches': v[0], 'avg_us': v[1] / v[0] / 1e3, 'share': v[1] / total}
        for k, v in sorted(st.items(), key=lambda x: -x[1][1])}}
    for k, v in list(out['timed_window_kernels'].items())[:12]:
        print('{0:28s} {1:7d} {2:10.1f} us {3:6.1%}'.format(k, v['dispatches'], v['avg_us'],
                                                          v['share']))
    if a.fetch and a.write:
        traffic = {}
        for path, cname in ((a.fetch, 'FETCH_SIZE'), (a.write, 'WRITE_SIZE')):
            crow = [r for r in csv.DictReader(open(path)) if r['Counter_Name'] == cname]
            cw = window(crow, 'Kernel_Name', 'Start_Timestamp', 'End_Timestamp')
            agg = collections.defaultdict(lambda: [0, 0.0])
            for r in cw:
                g = agg[short(r['Kernel_Name'])]
                g[0] += 1
                g[1] += float(r['Counter_Value'])
            for k, (n, tot) in agg.items():
                traffic.setdefault(k, {})[cname] = {'dispatches': n, 'avg_kib': tot / n}
        for k, d in traffic.items():
            if 'FETCH_SIZE' in d and 'WRITE_SIZE' in d:
                d['read_bytes_per_dispatch'] = 2.0 * d['FETCH_SIZE']['avg_kib'] * 1024
                d['write_bytes_per_dispatch'] = d['WRITE_SIZE']['avg_kib'] * 1024
                d['traffic_bytes_per_dispatch'] = (d['read_bytes_per_dispatch'] +
                                                   d['write_bytes_per_dispatch'])
        out['pmc_traffic'] = traffic
        out['pmc_correction'] = ('read = 2 x FETCH_SIZE (KiB, gfx950 half-count of 16 B/lane '
                                 'reads), write = WRITE_SIZE (KiB); MI355X_MICROARCH.md HBM')
    if a.mfma:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        rows = list(csv.DictReader(open(a.mfma)))
        win = window(rows, 'Kernel_Name', 'Start_Timestamp', 'End_Timestamp')
        disp = collections.defaultdict(set)
        for r in win:
            k = short(r['Kernel_Name'])
            per[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add(r.get('Dispatch_Id', r['Start_Timestamp']))
        util = {}
        for k, d in per.items():
            busy, act = d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0), d.get('GRBM_GUI_ACTIVE', 0.0)
            if act > 0 and busy > 0:
                util[k] = {'dispatches': len(disp[k]), 'mfma_busy_cycles': busy,
                           'mfma_busy_cycles_per_dispatch': busy / len(disp[k]),
                           'grbm_gui_active': act, 'mfma_util': busy / (1024.0 * act / 8.0)}
        out['pmc_mfma'] = dict(sorted(util.items(), key=lambda x: -x[1]['mfma_busy_cycles']))
        out['pmc_mfma_formula'] = ('SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 '
                                   'XCDs), summed over the timed window\'s dispatches')
        for k, v in list(out['pmc_mfma'].items())[:8]:
            print('mfma {0:28s} {1:6d} util {2:6.1%}'.format(k, v['dispatches'], v['mfma_util']))
    if a.out:
        json.dump(out, open(a.out, 'w'), indent=1)


if __name__ == '__main__':
    main()

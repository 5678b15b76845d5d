"""Per-kernel averages of rocprofv3 counter passes (development helper, tools/r05_pmc_newton.sh).

Reads one or more `--pmc ... --kernel-trace` counter_collection CSVs and prints, for the kernels
whose name contains one of the given substrings, the dispatch count and the per-dispatch mean of
every counter; with a kernel_trace CSV also the mean duration. Derived figures (MI355X_MICROARCH.md):
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8); HBM read bytes =
2 x FETCH_SIZE KiB (gfx950 half-count of 16-B/lane reads), write bytes = WRITE_SIZE KiB; LDS
conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES (disjoint: parked / issue-stalled / issuing).

usage: pmc_kernels.py --match k_chol_update32_t128 [--trace trace.csv] pass1.csv [pass2.csv ...]
       [--min-us 300] [--json out.json]
"""
import argparse
import collections
import csv
import json


def short(n):
    return n.split('(')[0].replace('void ', '')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csvs', nargs='+')
    ap.add_argument('--match', action='append', required=True)
    ap.add_argument('--trace')
    ap.add_argument('--min-us', type=float, default=0.0,
                    help='only dispatches at least this long (kernel trace of the same pass)')
    ap.add_argument('--json')
    a = ap.parse_args()
    out = {}
    for path in a.csvs:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        dur = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            k = short(r['Kernel_Name'])
            if not any(m in k for m in a.match):
                continue
            t = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 \
                if 'End_Timestamp' in r and r['End_Timestamp'] else None
            if t is not None and t < a.min_us:
                continue
            d = r.get('Dispatch_Id', r.get('Correlation_Id', r['Start_Timestamp']))
            per[k][r['Counter_Name']] += float(r['Counter_Value'])
            if d not in disp[k]:
                disp[k].add(d)
                if t is not None:
                    dur[k] += t
        for k, cs in per.items():
            n = len(disp[k])
            e = out.setdefault(k, {'dispatches': {}, 'per_dispatch': {}, 'avg_us': {}})
            e['dispatches'][path] = n
            if dur[k]:
                e['avg_us'][path] = dur[k] / n
            for c, v in cs.items():
                e['per_dispatch'][c] = v / n
    for k, e in out.items():
        p = e['per_dispatch']
        der = {}
        if p.get('GRBM_GUI_ACTIVE') and 'SQ_VALU_MFMA_BUSY_CYCLES' in p:
            der['mfma_busy'] = p['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024.0 * p['GRBM_GUI_ACTIVE'] / 8)
        if 'FETCH_SIZE' in p:
            der['hbm_read_bytes'] = 2.0 * p['FETCH_SIZE'] * 1024
        if 'WRITE_SIZE' in p:
            der['hbm_write_bytes'] = p['WRITE_SIZE'] * 1024
        if p.get('SQ_LDS_IDX_ACTIVE'):
            der['lds_conflict_share'] = p.get('SQ_LDS_BANK_CONFLICT', 0.0) / p['SQ_LDS_IDX_ACTIVE']
        if p.get('SQ_WAVE_CYCLES'):
            for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS',
                      'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS', 'SQ_BUSY_CYCLES'):
                if c in p:
                    der[c.lower() + '_share'] = p[c] / p['SQ_WAVE_CYCLES']
        if p.get('TCC_HIT_sum') is not None and p.get('TCC_MISS_sum'):
            der['l2_hit'] = p['TCC_HIT_sum'] / (p['TCC_HIT_sum'] + p['TCC_MISS_sum'])
        if p.get('SQ_INSTS_MFMA'):
            for c in ('SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_SALU'):
                if c in p:
                    der[c.lower() + '_per_mfma'] = p[c] / p['SQ_INSTS_MFMA']
        e['derived'] = der
        print('==', k, e['dispatches'], {q: round(v, 1) for q, v in e['avg_us'].items()})
        for c, v in sorted(p.items()):
            print('   {0:28s} {1:16.4g}'.format(c, v))
        for c, v in der.items():
            print('   * {0:26s} {1:16.4g}'.format(c, v))
    if a.json:
        json.dump(out, open(a.json, 'w'), indent=1)


if __name__ == '__main__':
    main()

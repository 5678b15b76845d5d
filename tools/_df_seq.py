"""Per-dispatch durations of k_chol_panel_df32 in kernel-trace order (one theta-call's panels):
development tool for the dataflow-panel analysis."""
import csv
import sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
df = [r for r in rows if 'k_chol_panel_df32' in r['Kernel_Name']]
up = [r for r in rows if 'k_chol_update32_t128' in r['Kernel_Name']]
print('df32 launches', len(df), 'update32 launches', len(up))
last = df[-48 * 2:] if len(df) > 96 else df
for i, r in enumerate(last):
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    print('%3d grid %8s  %7.1f us' % (i, r.get('Grid_Size_X', r.get('Grid_Size', '?')), d))

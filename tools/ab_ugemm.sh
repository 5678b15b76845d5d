# A/B of k_ugemm between two builds (tools/_oldlib/libapm_<A>.so, _<B>.so): HIP-event timing per
# batch size, then one FETCH_SIZE pass each (k_ugemm dispatches only, KiB x2 per gfx950 rule)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
A=$1; B=$2
for v in $A $B $A $B; do
  echo "== $v"; APM_LIB=tools/_oldlib/libapm_$v.so timeout -k 10 120 python3 -u tools/ugemm_bench.py
done
for v in $A $B; do
  rm -rf /tmp/pmc_$v
  APM_LIB=tools/_oldlib/libapm_$v.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_$v -o run -- python3 tools/ugemm_bench.py --reps 3 > /dev/null 2>&1
  F=$(find /tmp/pmc_$v -name '*counter_collection.csv' | head -1)
  python3 - "$F" "$v" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_ugemm' in r['Kernel_Name'] and r['Counter_Name'] == 'FETCH_SIZE']
by = collections.defaultdict(list)
for r in rows:
    by[int(r['Grid_Size'])].append(2 * 1024 * float(r['Counter_Value']))
for g, v in sorted(by.items()):
    print(sys.argv[2], 'grid', g, 'dispatches', len(v), 'fetch MB/dispatch %.1f' % (sum(v) / len(v) / 1e6))
PY
done

# Same-box A/B of stationary 64-chain theta-calls (development tool): for each variant
# "name|library|VAR=value ..." (empty library = the in-tree build), tools/time_theta.py under a
# kernel trace; prints the variant's theta-call times, value hashes and the kernels matching
# $AB_KERNELS (a regex, default: every kernel above 1 % of the total).
#   bash tools/ab_theta.sh 'head|tools/_headlib/libapm.so|' 'new||APM_X=1' ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/ab_theta.txt; : > $OUT
for spec in "$@"; do
  IFS='|' read -r name lib envs <<< "$spec"
  rm -rf /tmp/abt_$name
  ( if [ -n "$lib" ]; then export APM_LIB=$lib; fi
    for kv in $envs; do export "$kv"; done
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/abt_$name -o run \
      -- python3 tools/time_theta.py --batch 64 --reps 4 --no-prof \
      --theta-file tests/golden/stationary_thetas.npy > gpurun_out/abt_$name.log 2>&1 ) || exit 1
  F=$(find /tmp/abt_$name -name '*kernel_stats.csv' | head -1)
  { echo "== $name ($spec)"; grep -E "^rep|^hash" gpurun_out/abt_$name.log
    python3 - "$F" <<'PY'
import csv, os, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
pat = os.environ.get('AB_KERNELS')
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    share = float(r['TotalDurationNs']) / tot
    if (pat and re.search(pat, r['Name'])) or (not pat and share > 0.01):
        print('  %-60s %5s calls %9.1f us avg %6.2f %%' % (r['Name'][:60], r['Calls'],
              float(r['AverageNs']) / 1e3, 100 * share))
PY
  } >> $OUT
done
cat $OUT

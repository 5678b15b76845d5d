cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in new old new old; do
  if [ $v = old ]; then export APM_T128=0 APM_LEFT=0 APM_OUTER=4; else unset APM_T128 APM_LEFT APM_OUTER; fi
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --cpu-baseline 0 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value'],2), round(d['wall_split_s']['theta_call'],2), d['theta_calls_per_transition'])"
done > gpurun_out/ab.log

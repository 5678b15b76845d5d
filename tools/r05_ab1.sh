# Round-5 A/B on one MI355X: the stationary bench with 1 and 2 cohorts per GPU (short, no CPU
# baseline / parity / ESS extension)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
for K in 1 2 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 --parity 0 --ess-min 0 --ess-burn 0 --cohorts $K > $O/coh$K.json 2> $O/coh$K.err || exit $?
  python -c "import json; l=json.load(open('$O/coh$K.json')); print('cohorts', $K, 'value', round(l['value'],1), 'prior', round(l['value_prior_init']['value'],1), 'thcall', round(l['theta_call_ms_mean'],1))"
done


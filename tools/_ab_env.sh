# in-situ A/B of an env knob (VAR=a vs VAR=b) on the current build: GPU tests first, then
# time_theta + bench alternated
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; A=$2; B=$3; STEPS=${4:-30}
[ -n "$SKIPTESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
[ -n "$SKIPTESTS" ] || tail -1 gpurun_out/gpu_tests.log
for v in $A $B $A $B; do
  env $VAR=$v timeout -k 10 200 python -u tools/time_theta.py --batch 64 --reps 3 2>&1 | grep "rep 2\|update32 " | sed "s/^/$VAR=$v /"
  env $VAR=$v timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 5 --cpu-baseline 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$VAR=$v', round(d['value'],2), d['newton_refinement_steps'], d['newton_fp64_reruns'], {k: round(d[k]['achieved'],1) for k in d if k.startswith('roofline')})"
done

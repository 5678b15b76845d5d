# in-situ A/B/C of three libapm builds (tools/_oldlib/libapm_<X>.so): tests with each non-head build first
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in $2 $3; do
  APM_LIB=tools/_oldlib/libapm_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$v.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/gpu_tests_$v.log)"
done
for v in $1 $2 $3 $1 $2 $3; do
  APM_LIB=tools/_oldlib/libapm_$v.so timeout -k 10 200 python -u tools/time_theta.py --batch 64 --reps 3 2>&1 | grep "rep 2" | sed "s/^/$v /"
  APM_LIB=tools/_oldlib/libapm_$v.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', round(d['value'],2), d['newton_refinement_steps'], d['newton_fp64_reruns'])"
done

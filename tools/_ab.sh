# in-situ A/B of two libapm builds (tools/_oldlib/libapm_<A>.so vs _<B>.so): tests with B, then bench alternated
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
A=$1; B=$2; STEPS=${3:-30}
APM_LIB=tools/_oldlib/libapm_$B.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in $A $B $A $B; do
  APM_LIB=tools/_oldlib/libapm_$v.so timeout -k 10 200 python -u tools/time_theta.py --batch 64 --reps 3 2>&1 | grep "rep 2" | sed "s/^/$v /"
  APM_LIB=tools/_oldlib/libapm_$v.so timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 5 --cpu-baseline 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', round(d['value'],2), {k: round(d[k]['achieved'],1) for k in d if k.startswith('roofline')})"
done

set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for L in new old new old; do
  unset APM_LIB
  if [ $L = old ]; then export APM_LIB=$PWD/tools/_oldlib/libapm.so; fi
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/ab_$L.json 2> gpurun_out/ab.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$L.json'));print('$L', round(d['value'],2), d['parity']['pass'], round(d['roofline_lu']['avg_launch_us'],1), round(d['roofline_lu']['frac'],3), d['wall_split_s'])"
done

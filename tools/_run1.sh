set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py -x -v --timeout 500 --timeout-method thread > gpurun_out/t_knobs.txt 2>&1 || { tail -30 gpurun_out/t_knobs.txt; exit 1; }
tail -3 gpurun_out/t_knobs.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.err
python3 -c "import json;d=json.loads(open('gpurun_out/bench20.json').read().strip().splitlines()[-1]);print(d['value'], d['parity']['pass'], d['pmc_provenance']['stale'], d['ess_per_sec'])"

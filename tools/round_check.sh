# Full round check of HEAD on one MI355X: GPU tests, smoke, default bench, then the rocprofv3
# kernel-trace/stats summary and the FETCH_SIZE / WRITE_SIZE PMC passes of a short bench.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
bash tools/profile_round.sh

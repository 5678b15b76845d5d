# GPU tests (whole -m gpu suite, new full-size parity tests included), smoke, and the bench
# under the driver's own invocation (--steps 20 --warmup 5).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.err

set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1 || { tail -30 gpurun_out/gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/gpu_tests_final.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
cat gpurun_out/smoke_final.log

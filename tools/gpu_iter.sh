cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -3 gpurun_out/gpu_tests.log
grep -q " passed" gpurun_out/gpu_tests.log && ! grep -q "failed\|error" gpurun_out/gpu_tests.log || exit 1
for v in 1 0 1 0; do
  echo "== OVERLAP_K=$v"; APM_OVERLAP_K=$v timeout -k 10 200 python -u tools/time_theta.py --batch 64 --reps 3 2>&1 | grep -v amdgpu | grep "rep 2" || exit 1
done > gpurun_out/tt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tt_trace -o run -- python3 tools/time_theta.py --batch 64 --reps 2 > gpurun_out/tt_trace.log 2>&1

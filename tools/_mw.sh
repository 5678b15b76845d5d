set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 90 python -u tools/time_theta.py --batch 8 --reps 2 2>&1 | grep "rep"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in 0 1 0 1; do
  APM_TRSV_MW=$v timeout -k 10 200 python -u tools/time_theta.py --batch 64 --reps 3 2>&1 | grep "rep 2" | sed "s/^/MW=$v /"
done

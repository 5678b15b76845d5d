set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in 0 1; do
  rm -rf gpurun_out/ph_o$v
  APM_OVERLAP_K=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ph_o$v -o run -- python3 tools/time_theta.py --batch 64 --reps 2 > /dev/null 2>&1
  T=$(find gpurun_out/ph_o$v -name '*kernel_trace.csv' | head -1)
  echo "== OVERLAP_K=$v"; python3 tools/theta_phases.py $T
  find gpurun_out/ph_o$v -name '*.csv' -delete
done

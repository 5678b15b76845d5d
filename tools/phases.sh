# kernel trace of tools/time_theta.py (64 chains) under two settings of an env knob, phase timeline
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1
for v in $2 $3; do
  rm -rf gpurun_out/ph_$v
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ph_$v -o run -- python3 tools/time_theta.py --batch 64 --reps 2 > /dev/null 2>&1
  T=$(find gpurun_out/ph_$v -name '*kernel_trace.csv' | head -1)
  echo "== $VAR=$v"; python3 tools/theta_phases.py $T
  find gpurun_out/ph_$v -name '*.csv' -delete
done

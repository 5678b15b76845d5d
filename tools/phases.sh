# kernel trace of tools/time_theta.py (64 chains) under settings of an env knob, phase timeline
# and a hash of the theta-call / u-call outputs (bitwise equality across settings)
#   bash tools/phases.sh VAR v1 v2 [v3 ...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1; shift
for v in "$@"; do
  rm -rf gpurun_out/ph_$v
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ph_$v -o run -- python3 tools/time_theta.py --batch 64 --reps 2 $TT_ARGS > gpurun_out/ph_$v.txt 2>&1
  T=$(find gpurun_out/ph_$v -name '*kernel_trace.csv' | head -1)
  echo "== $VAR=$v"; grep "^hash\|^newton iter" gpurun_out/ph_$v.txt; python3 tools/theta_phases.py $T
  find gpurun_out/ph_$v -name '*.csv' -delete
done

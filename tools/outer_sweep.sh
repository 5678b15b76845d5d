# time_theta (64 chains) under several values of blocking / launch-shape knobs (development tool):
#   bash tools/outer_sweep.sh VAR v1 v2 ...   (VAR: APM_OUTER, APM_OVERLAP_K, ... - DESIGN.md §7)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; shift
for v in "$@"; do
  env $VAR=$v timeout -k 10 200 python -u tools/time_theta.py --batch 64 --reps 3 2>&1 | grep "rep 2" | sed "s/^/$VAR=$v /"
done

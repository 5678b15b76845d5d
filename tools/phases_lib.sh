# phase timeline + output hash of tools/time_theta.py (64 chains) for several builds
# (tools/_oldlib/libapm_<name>.so):  bash tools/phases_lib.sh name1 name2 ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  rm -rf gpurun_out/phl_$v
  APM_LIB=tools/_oldlib/libapm_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/phl_$v -o run -- python3 tools/time_theta.py --batch 64 --reps 2 > gpurun_out/phl_$v.txt 2>&1
  T=$(find gpurun_out/phl_$v -name '*kernel_trace.csv' | head -1)
  echo "== $v"; grep "^hash" gpurun_out/phl_$v.txt; python3 tools/theta_phases.py $T
  find gpurun_out/phl_$v -name '*.csv' -delete
done

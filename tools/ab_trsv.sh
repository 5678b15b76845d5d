# TRSV variants: phase timeline (64 chains) for old/new builds and the WG-count knob, bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in r2 trsvpf; do
  rm -rf gpurun_out/ph_$v
  APM_LIB=tools/_oldlib/libapm_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ph_$v -o run -- python3 tools/time_theta.py --batch 64 --reps 2 > /dev/null 2>&1
  T=$(find gpurun_out/ph_$v -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python3 tools/theta_phases.py $T | grep -E "wall|newton|trsv"
  find gpurun_out/ph_$v -name '*.csv' -delete
done
for g in 8 2; do
  rm -rf gpurun_out/ph_g$g
  APM_TRSV_G=$g APM_LIB=tools/_oldlib/libapm_trsvpf.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ph_g$g -o run -- python3 tools/time_theta.py --batch 64 --reps 2 > /dev/null 2>&1
  T=$(find gpurun_out/ph_g$g -name '*kernel_trace.csv' | head -1)
  echo "== G=$g"; python3 tools/theta_phases.py $T | grep -E "wall|newton|trsv"
  find gpurun_out/ph_g$g -name '*.csv' -delete
done

# development: which refinement acceptance thresholds pass at N=4096 (fallback shows as fp64 logf)
set -e
for env in "APM_MIXED=0" "APM_REFINE=1 APM_REFINE_TOL=1e-3" "APM_REFINE=1 APM_REFINE_TOL=1e-2" "APM_REFINE=2 APM_REFINE_TOL=1e-6" "APM_REFINE=2 APM_REFINE_TOL=1e-7" "APM_REFINE=2 APM_REFINE_TOL=1e-8" "APM_REFINE=3 APM_REFINE_TOL=1e-10"; do
  echo "== $env"
  env $env timeout -k 10 60 python3 tools/time_theta.py --batch 4 --reps 1 | grep rep
done

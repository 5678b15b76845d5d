# Mixed-precision Newton modes at the stationary states vs the all-fp64 iteration, for the default
# and looser refinement tolerances (tools/refine_tol_study.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05rt; mkdir -p $O
timeout -k 10 600 python -u tools/refine_tol_study.py --tols 1e-3 3e-3 1e-2 --nread 16 2>&1 | tee $O/study.txt || exit $?

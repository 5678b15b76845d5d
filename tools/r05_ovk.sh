# chol(K) beside the first Newton iterations (APM_OVERLAP_K=1, default) or after the loop (0):
# stationary 64-chain theta-call A/B in one process
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05ok; mkdir -p $O
timeout -k 10 400 python -u tools/ab_knob.py APM_OVERLAP_K 1 0 1 0 --reps 3 2>&1 | tee $O/ab.txt || exit $?

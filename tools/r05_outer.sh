# fp64 outer panel width (APM_OUTER: chol(K), the posterior factor) at the stationary states:
# one-process A/B of the 64-chain theta-call
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05out; mkdir -p $O
timeout -k 10 500 python -u tools/ab_knob.py APM_OUTER 8 6 10 8 6 10 --reps 3 2>&1 | tee $O/ab.txt

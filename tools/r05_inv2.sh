# explicit-inverse panels: in-situ A/B at the stationary states (timing, |d log f|, refinement)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05inv; mkdir -p $O
timeout -k 10 300 python -u tools/ab_knob.py APM_DFINV 0 1 0 1 --reps 3 2>&1 | tee $O/ab_dfinv.txt

# advisor r04 (low): the fp32 posterior bottom block at the stationary N=4096 states against the
# all-fp64 posterior factor (APM_POST32=0): |d log f| of the 64-chain theta-call and u-call
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05post; mkdir -p $O
timeout -k 10 300 python -u tools/ab_knob.py APM_POST32 0 2 --reps 2 2>&1 | tee $O/ab.txt

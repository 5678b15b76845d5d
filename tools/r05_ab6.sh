# current build: stationary theta-call A/B vs the walk (hash check) and a Newton-iteration timeline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05ab6; mkdir -p $O
timeout -k 10 300 python -u tools/ab_knob.py APM_DFINV 0 1 0 1 --reps 3 2>&1 | tee $O/ab.txt || exit $?
bash tools/r05_timeline.sh

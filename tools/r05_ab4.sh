# fp64 update DMA order A/B (microbench) and the split far update A/B (in situ, stationary)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05ab4; mkdir -p $O
bash tools/r05_ab64.sh > $O/ab64.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_knob.py APM_LA_SPLIT 0 1 0 1 --reps 3 2>&1 | tee $O/ab_split.txt

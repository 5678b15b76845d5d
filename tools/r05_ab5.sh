# stationary theta-call timing of the current build (hash must stay 69742bb6f559 for DFINV=1)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05ab5; mkdir -p $O
timeout -k 10 300 python -u tools/ab_knob.py APM_Q256_GRID 0 192 224 0 192 224 --reps 3 2>&1 | tee $O/ab.txt

# K x with 1 / 2 / 4 lower tiles per workgroup (APM_SYMV_TPW): stationary theta-call A/B in one
# process (identical output hashes expected), then the stationary-state parity test
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05sv; mkdir -p $O
timeout -k 10 400 python -u tools/ab_knob.py APM_SYMV_TPW 1 2 4 1 2 4 --reps 3 2>&1 | tee $O/ab.txt || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -k "stationary or config2_full" 2>&1 | tee $O/tests.txt || exit $?

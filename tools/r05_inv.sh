# explicit-inverse panels: the kernel tests that pin them, then the in-situ A/B (stationary)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05inv; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -k "explicit_inverse or planes_bitwise or mixed_newton or fp16x3 or posterior_bottom" > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_knob.py APM_DFINV 0 1 0 1 --reps 3 2>&1 | tee $O/ab_dfinv.txt
